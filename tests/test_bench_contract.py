"""bench.py's output contract on the GPU, on a small frame: one JSON line with every key the task's
contract names, the metric string of BASELINE.json, value = rays per frame / ms per step, the
roofline's frac = achieved / peak (the measured bound; unmeasured without a PMC profile), a plan that covers --steps exactly (6 frames in batches of at most 4: 3 + 3),
and rays per frame equal to the oracle's count for the same frame with --orbit 0 (the reference's definition:
primary + traced reflection + traced shadow rays); with the default camera path (frame i moved by
i * 0.02) the BMP of frame 0 is still the reference camera's."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def oracle_frame(W, H):
    from tests.oracle_bind import OracleScene
    from tests.scenes import scene_paths
    o = OracleScene.load(*scene_paths("dragon"))
    o.build_bvh(3)
    return o.render(W, H, threads=16)


@pytest.mark.parametrize("output,orbit", [("bgra8", "0"), ("rgb", "0"), ("bgra8", "0.02")])
def test_bench_prints_the_contract_line(output, orbit, tmp_path):
    W, H = 320, 180
    bmp = tmp_path / "frame.bmp"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "6", "--warmup", "2",
                        "--frames", "4", "--width", str(W), "--height", str(H), "--no-cpu-baseline",
                        "--output", output, "--bmp", str(bmp), "--orbit", orbit], capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    d = json.loads(lines[0])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    for k in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["unit"] == "Mrays/s" and d["n_gpus"] == 1 and d["steps"] == 6 and d["warmup"] == 2
    assert d["higher_is_better"] is True and d["vs_baseline"] is None
    assert "workload" in d["config"] and d["config"]["output"] == output
    rays = d["config"]["rays_per_frame"]
    assert d["value"] == pytest.approx(rays / d["ms_per_step"] / 1e3, rel=1e-9)
    rf = d["roofline"]
    if rf["traffic"] is None:  # no PMC profile of this configuration and build: nothing claimed as measured
        assert rf["bound_measured"] is None and rf["issue_frac"] is None and rf["frac"] is None
        assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    else:  # the measured roofline: VALU issue when HBM carries < 5 % of the algorithmic bytes, else HBM
        assert rf["bound"] in ("issue", "hbm")
        assert rf["frac"] == pytest.approx(rf["achieved"] / rf["peak"], rel=1e-9) and 0 < rf["frac"] <= 1
    assert rf["alg_byte_frac"] == pytest.approx(rf["alg_byte_achieved"] / 8000.0, rel=1e-9) and rf["alg_byte_achieved"] > 0
    assert rf["frames_per_launch"] == 3
    ref = oracle_frame(W, H)
    c = ref["counters"]
    if orbit == "0":  # the reference's loop of one camera: every frame is the oracle's frame
        assert rays == c["primary"] + c["reflection"] + c["shadow"]
    else:  # a camera path (the default): frame 0 is the reference camera, the others moved a little
        assert abs(rays / (c["primary"] + c["reflection"] + c["shadow"]) - 1) < 0.05
    from prt import host
    assert bmp.read_bytes() == host.bmp_encode(ref["rgb"])  # frame 0 of the last launch, as bmp_write_file writes it


def test_bench_two_ranks_on_one_gpu_count_the_whole_frame(tmp_path):
    """the N > 1 flow (8-row blocks per rank, two streams, ping-pong gathers) rehearsed with 2 gloo ranks
    on the one GPU of the test box (PRT_DIST_ONE_GPU; RCCL refuses two ranks on one device), launched as the
    driver does it — `python bench.py --gpus 2`, no launcher: bench.py starts the ranks as child processes —
    the ranks' rays add up to the whole frame's, rank 0 prints the only line and writes the gathered frame's
    BMP (= the reference writer's bytes of the oracle's frame)"""
    env = dict(os.environ, PRT_DIST_ONE_GPU="1", PRT_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    args = ["--steps", "4", "--warmup", "2", "--frames", "2", "--width", "320", "--height", "180"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--bmp", str(tmp_path / "g.bmp")]
                       + args, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 4
    assert d["config"]["gather"].startswith("torch.distributed")  # gloo: the native RCCL gather needs one GPU per rank
    # the N > 1 diagnostics: each rank's kernel time, the render-only walls, the exposed gather, the gather that ran
    rk = d["config"]["ranks"]
    assert d["config"]["gather_mode"] == rk["gather_mode"] == "torch"
    assert len(rk["kernel_ms_per_frame"]["per_rank"]) == 2 and rk["kernel_ms_per_frame"]["min"] > 0
    assert rk["kernel_ms_per_frame"]["spread"] >= 0 and len(rk["render_wall_ms"]["per_rank"]) == 2
    assert rk["wall_ms"] > 0 and abs(rk["exposed_gather_ms"] - (rk["wall_ms"] - rk["render_wall_ms"]["max"])) < 1e-6
    assert len(rk["variant_per_rank"]) == 2
    one = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline"] + args,
                         capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert one.returncode == 0, one.stderr[-3000:]
    d1 = json.loads([l for l in one.stdout.splitlines() if l.startswith("{")][0])
    assert d["config"]["rays_per_frame"] == d1["config"]["rays_per_frame"]
    from prt import host
    assert (tmp_path / "g.bmp").read_bytes() == host.bmp_encode(oracle_frame(320, 180)["rgb"])


def test_bench_native_gather_one_rank(tmp_path):
    """--gather native at one rank: the frames go through rt_comm_init_rank / rt_comm_gather (prt.dist.NativeGather)
    and the setup check (rank 0's gathered frames == one GPU's) passes; the BMP is still the oracle's frame"""
    W, H = 320, 180
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "2", "--frames", "2",
                        "--width", str(W), "--height", str(H), "--no-cpu-baseline", "--gather", "native",
                        "--bmp", str(tmp_path / "n.bmp")], capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["config"]["gather"].startswith("rt_comm_gather") and "checked at setup" in d["config"]["gather"]
    from prt import host
    assert (tmp_path / "n.bmp").read_bytes() == host.bmp_encode(oracle_frame(W, H)["rgb"])
