"""HIP path (librt_hip.so via the rt_* C-ABI) vs the oracle and the reference's own fixtures.

Bar (BASELINE.json north_star):
  * primary (and per-bounce) hit indices: bit-exact;
  * colours: bit-exact against the strict oracle / reference fixtures for the STRICT kernel and for
    the FAST kernel on the reference BVH; any BVH the product builds must stay within the stated
    per-channel tolerance RGB_TOL = 1e-5 of the reference (hits still exact).
"""
import ctypes
import json
import os

import numpy as np
import pytest

from prt import host

pytestmark = pytest.mark.gpu
RGB_TOL = 1e-5
# every kernel and launch configuration the C-ABI exposes (rt_frame.kernel / rt_frame.variant): STRICT, FAST
# with its default rule ("fast"), and each variant forced: k_persist at 4 waves/SIMD ("persist4"), k_coop
# ("coopG": G lanes per ray). "shpool": k_persist with each level's shadow rays walked as a per-wave pool
# (rt_shpool.hpp); "shdefer": one pool for all levels' shadow rays.
KERNELS = ["strict", "fast", "persist4", "coop2", "coop4", "shpool", "shdefer"]


def select(kernel):
    """test kernel name -> the `kernel` argument of prt.device (a variant name selects RT_KERNEL_FAST + it)"""
    return kernel


GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
G = json.load(open(os.path.join(GOLD, "golden.json")))


@pytest.fixture(scope="module")
def dev():
    from prt import device
    assert device.device_count() > 0, "no GPU visible"
    return device


@pytest.fixture(scope="module")
def scenes():
    out = {}
    for name in ("car_boxed", "car_only"):
        s = host.Scene.named(name).build_bvh(3)
        out[name] = s
    return out


def render(dev, scene, W, H, kernel, rows=None, spp=1, bounces=4, counters=False, accel="auto"):
    r = dev.Renderer(0, counters=counters)
    r.upload(scene, accel=accel)
    import torch
    nr = rows[2] if rows else H
    hit = torch.empty((nr, W), dtype=torch.int32, device="cuda")
    t = torch.empty((nr, W), dtype=torch.float32, device="cuda")
    rgb = torch.empty((nr, W, 3), dtype=torch.float32, device="cuda")
    r.render(host.camera(W, H), W, H, rows=rows, bounces=bounces, spp=spp, kernel=select(kernel), rgb=rgb, hit=hit,
             t=t)
    r.sync()
    st = r.stats()
    out = {"rgb": rgb.cpu().numpy(), "hit": hit.cpu().numpy(), "t": t.cpu().numpy(), "stats": st}
    r.close()
    return out


def same_bits(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.int32), np.asarray(b, np.float32).view(np.int32))


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("scene", ["car_boxed", "car_only"])
@pytest.mark.parametrize("W,H", [(64, 36), (160, 90)])
def test_small_frames_vs_reference_fixture(dev, scenes, kernel, scene, W, H):
    out = render(dev, scenes[scene], W, H, kernel)
    ref = np.load(os.path.join(GOLD, f"{scene}_{W}x{H}_strict.npz"))
    np.testing.assert_array_equal(out["hit"], ref["hit"])
    assert same_bits(out["t"], ref["t"])
    assert same_bits(out["rgb"], ref["rgb"]), np.abs(out["rgb"] - ref["rgb"]).max()


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("scene", ["car_boxed", "car_only"])
def test_1080p_vs_reference_sample(dev, scenes, kernel, scene):
    out = render(dev, scenes[scene], 1920, 1080, kernel, counters=True)
    ref = np.load(os.path.join(GOLD, f"{scene}_1080p_strict_sample.npz"))
    idx = ref["idx"]
    np.testing.assert_array_equal(out["hit"].reshape(-1)[idx], ref["hit"])
    assert same_bits(out["t"].reshape(-1)[idx], ref["t"])
    assert same_bits(out["rgb"].reshape(-1, 3)[idx], ref["rgb"])
    import hashlib
    md5 = hashlib.md5(out["hit"].astype(np.int32).tobytes() + out["t"].tobytes() + out["rgb"].tobytes()).hexdigest()
    assert md5 == G["frames"][f"{scene}_1920x1080_strict"]["md5"]
    st = out["stats"]
    rays = G["rays"][f"{scene}_1920x1080"]
    assert st["primary"] + st["reflection"] == rays["closest"]
    assert st["shadow"] == rays["shadow"]
    assert st["pixels"] == 1920 * 1080


@pytest.mark.parametrize("kernel", KERNELS)
def test_row_subset_equals_full_frame(dev, scenes, kernel):
    """compact row sets (rt_frame rows): cyclic single rows, and blocks of rows (row_block; the last
    block partial) — every row equal to the full frame's"""
    full = render(dev, scenes["car_boxed"], 320, 180, kernel)
    part = render(dev, scenes["car_boxed"], 320, 180, kernel, rows=(5, 8, 22))
    rows = [5 + 8 * k for k in range(22)]
    assert same_bits(part["rgb"], full["rgb"][rows])
    np.testing.assert_array_equal(part["hit"], full["hit"][rows])
    part = render(dev, scenes["car_boxed"], 320, 180, kernel, rows=(8, 24, 37, 8))
    rows = [8 + (k // 8) * 24 + k % 8 for k in range(37)]
    assert same_bits(part["rgb"], full["rgb"][rows]), kernel
    np.testing.assert_array_equal(part["hit"], full["hit"][rows])


def test_ragged_and_tiny_frames(dev, scenes):
    """frames that are not multiples of the 8x8 tile, down to one pixel, against the oracle"""
    from tests.oracle_bind import OracleScene
    from tests.scenes import scene_paths
    o = OracleScene.load(*scene_paths("car_only"))
    o.build_bvh(3)
    for W, H in ((1, 1), (7, 3), (13, 9), (65, 17)):
        ref = o.render(W, H)
        for k in KERNELS:
            out = render(dev, scenes["car_only"], W, H, k)
            np.testing.assert_array_equal(out["hit"], ref["hit"], err_msg=f"{k} {W}x{H}")
            assert same_bits(out["rgb"], ref["rgb"]), (k, W, H)


def test_fast_kernel_traversing_a_sah_bvh_only(dev):
    """accel="reference" with a binned-SAH BVH passed as THE bvh: no reference order available, so only
    the stated tolerance is promised (hits exact on this scene, colours within RGB_TOL)"""
    s = host.Scene.named("car_boxed").build_bvh("binned_sah")
    out = render(dev, s, 160, 90, "fast", accel="reference")
    ref = np.load(os.path.join(GOLD, "car_boxed_160x90_strict.npz"))
    np.testing.assert_array_equal(out["hit"], ref["hit"])
    assert np.abs(out["rgb"] - ref["rgb"]).max() <= RGB_TOL


def test_random_mode(dev):
    s = host.Scene.random(10000).build_bvh(3)
    ref = np.load(os.path.join(GOLD, "random10k_160x90_strict.npz"))
    for k in KERNELS:
        out = render(dev, s, 160, 90, k)
        np.testing.assert_array_equal(out["hit"], ref["hit"])
        assert same_bits(out["rgb"], ref["rgb"])


def test_oracle_counts_and_bounces(dev, scenes):
    """per-bounce ray counters and BOUNCES variations against the oracle port"""
    from tests.oracle_bind import OracleScene
    from tests.scenes import scene_paths
    o = OracleScene.load(*scene_paths("car_boxed"))
    o.build_bvh(3)
    for b in (1, 2, 4, 6, 8):
        o.set_bounces(b)
        ref = o.render(128, 72)
        for kern in KERNELS:
            out = render(dev, scenes["car_boxed"], 128, 72, kern, bounces=b, counters=True)
            assert same_bits(out["rgb"], ref["rgb"]), (b, kern)
            c, st = ref["counters"], out["stats"]
            for k in ("primary", "reflection", "shadow", "shadow_skipped", "hits"):
                assert st[k] == c[k], (b, kern, k)


def test_strict_traversal_counters_match_reference_order(dev, scenes):
    """the strict kernel walks the reference BVH in the reference's order: identical visit counts"""
    from tests.oracle_bind import OracleScene
    from tests.scenes import scene_paths
    o = OracleScene.load(*scene_paths("car_only"))
    o.build_bvh(3)
    c = o.render(96, 54)["counters"]
    st = render(dev, scenes["car_only"], 96, 54, "strict", counters=True)["stats"]
    for k in ("ch_inner", "ch_leaf", "ch_tri", "sh_inner", "sh_leaf", "sh_tri"):
        assert st[k] == c[k], k


@pytest.mark.parametrize("kernel", ["fast", "persist4", "coop4", "shpool", "shdefer"])
@pytest.mark.parametrize("spp", [4, 16])
def test_spp_matches_oracle(dev, scenes, spp, kernel):
    from tests.oracle_bind import OracleScene
    from tests.scenes import scene_paths
    o = OracleScene.load(*scene_paths("car_only"))
    o.build_bvh(3)
    ref, c = o.render_spp(64, 36, spp)
    out = render(dev, scenes["car_only"], 64, 36, kernel, spp=spp, counters=True)
    assert same_bits(out["rgb"], ref)
    assert out["stats"]["primary"] == 64 * 36 * spp


@pytest.mark.parametrize("kernel", ["default", "shpool", "shdefer", "persist4"])
@pytest.mark.parametrize("spp", [4, 16])
def test_spp_of_a_two_light_scene_matches_oracle(dev, spp, kernel):
    """the default rule sends spp > 1 frames of 2+-light scenes through the shadow pool's multi-sample path
    (render_pixel_shp): dragon (2 lights) at 4 and 16 spp against the oracle's stratified render_spp, bit for bit,
    with the oracle's ray counts"""
    from tests.oracle_bind import OracleScene
    from tests.scenes import scene_paths
    o = OracleScene.load(*scene_paths("dragon"))
    o.build_bvh(3)
    ref, c = o.render_spp(64, 36, spp)
    s = host.Scene.named("dragon").build_bvh(3)
    out = render(dev, s, 64, 36, kernel, spp=spp, counters=True)
    assert same_bits(out["rgb"], ref), np.abs(out["rgb"] - ref).max()
    assert out["stats"]["primary"] == 64 * 36 * spp
    for k in ("primary", "reflection", "shadow"):
        assert out["stats"][k] == c[k], k


_SPP64 = {}


@pytest.mark.parametrize("kernel", ["fast", "persist4", "coop4", "shpool", "shdefer"])
def test_car_boxed_64spp_matches_oracle(dev, scenes, kernel):
    """BASELINE config 5 (car_boxed 3840x2160, 64 spp, multi-bounce): the reference has one corner ray per
    pixel (cpu/src/main.c:228-239); SURVEY §8d defines spp = s x s stratified sub-pixel samples, mean of the
    clamped samples (orc_render_spp restates it). Bit-exact against the oracle on the full 160x90 frame and
    on every 97th row of the 4K frame, with primary rays = 64 x pixels and the same reflection / shadow
    counts; spp = 1 of the same renderer is the reference's own fixture."""
    import torch
    from tests.oracle_bind import OracleScene
    from tests.scenes import scene_paths
    if "oracle" not in _SPP64:
        o = OracleScene.load(*scene_paths("car_boxed"))
        o.build_bvh(3)
        _SPP64["oracle"] = o
        _SPP64["small"] = o.render_spp(160, 90, 64)
        n4k = (2160 + 96) // 97
        _SPP64["4k"] = o.render_spp(3840, 2160, 64, rows=(0, 97, n4k))
    small, c_small = _SPP64["small"]
    out = render(dev, scenes["car_boxed"], 160, 90, kernel, spp=64, counters=True)
    assert same_bits(out["rgb"], small), np.abs(out["rgb"] - small).max()
    st = out["stats"]
    assert st["primary"] == 64 * 160 * 90 == c_small["primary"]
    for k in ("reflection", "shadow", "shadow_skipped"):
        assert st[k] == c_small[k], k
    big, c_big = _SPP64["4k"]
    n4k = (2160 + 96) // 97
    out = render(dev, scenes["car_boxed"], 3840, 2160, kernel, rows=(0, 97, n4k), spp=64, counters=True)
    assert same_bits(out["rgb"], big[0:2160:97]), np.abs(out["rgb"] - big[0:2160:97]).max()
    st = out["stats"]
    assert st["primary"] == 64 * 3840 * n4k == c_big["primary"]
    for k in ("reflection", "shadow", "shadow_skipped"):
        assert st[k] == c_big[k], k
    one = render(dev, scenes["car_boxed"], 160, 90, kernel, spp=1)
    ref = np.load(os.path.join(GOLD, "car_boxed_160x90_strict.npz"))
    assert same_bits(one["rgb"], ref["rgb"])
    np.testing.assert_array_equal(one["hit"], ref["hit"])


@pytest.mark.parametrize("name", ["dragon", "sportscar", "two_cars"])
def test_standin_scenes_vs_reference_fixture(dev, name):
    """stand-ins exercise the reference's IEEE corner cases (a zero direction component at the image centre
    column meets grid edges at x = 0: 0/0 NaN slabs cull boxes) and exact-tie hits on shared edges."""
    import hashlib
    s = host.Scene.named(name).build_bvh(3)
    ref = np.load(os.path.join(GOLD, f"{name}_96x54_strict.npz"))
    for k in KERNELS:
        out = render(dev, s, 96, 54, k)
        np.testing.assert_array_equal(out["hit"], ref["hit"], err_msg=k)
        assert same_bits(out["t"], ref["t"]), k
        assert same_bits(out["rgb"], ref["rgb"]), k
        out = render(dev, s, 320, 180, k)
        md5 = hashlib.md5(out["hit"].astype(np.int32).tobytes() + out["t"].tobytes() + out["rgb"].tobytes())
        assert md5.hexdigest() == G["standin"][name]["320x180_md5"], k


@pytest.mark.parametrize("name", ["car_only", "dragon"])
def test_exact_ties_everywhere_match_strict(dev, name):
    """every triangle twice: every closest hit is an exact tie, which the fast walks must detect -- through the
    packed triangle tests' tie flags too (shdefer, persist4) -- and resolve by the strict re-walk, so the frame equals
    the strict kernel's (the reference's first-found rule, bvh.c:331) bit for bit; occlusion is unchanged"""
    base = host.Scene.named(name)
    s = host.Scene(np.concatenate([base.triangles, base.triangles]), base.lights).build_bvh(3)
    ref = render(dev, s, 96, 54, "strict")
    for k in ("fast", "persist4", "shpool", "shdefer", "coop4"):
        out = render(dev, s, 96, 54, k, counters=True)
        np.testing.assert_array_equal(out["hit"], ref["hit"], err_msg=k)
        assert same_bits(out["t"], ref["t"]) and same_bits(out["rgb"], ref["rgb"]), k
        assert out["stats"]["fallbacks"] > 0, k


_ORACLE_FRAMES = {}


@pytest.mark.slow
@pytest.mark.parametrize("kernel", ["fast", "coop4", "shdefer"])
def test_bench_config_full_frame_vs_oracle(dev, kernel):
    """the bench workload (dragon stand-in, 1920x1080, fast kernel, library SAH BVH) against the oracle
    at full size: hit indices, t and colours bit-exact"""
    from tests.oracle_bind import OracleScene
    from tests.scenes import scene_paths
    s = host.Scene.named("dragon").build_bvh(3)
    out = render(dev, s, 1920, 1080, kernel, counters=True)
    if "dragon1080" not in _ORACLE_FRAMES:  # one oracle frame for both kernels
        o = OracleScene.load(*scene_paths("dragon"))
        o.build_bvh(3)
        _ORACLE_FRAMES["dragon1080"] = o.render(1920, 1080, threads=min(32, os.cpu_count() or 8))
    ref = _ORACLE_FRAMES["dragon1080"]
    bad = np.argwhere(out["hit"] != ref["hit"])
    assert len(bad) == 0, (len(bad), bad[:10])
    assert same_bits(out["t"], ref["t"])
    assert same_bits(out["rgb"], ref["rgb"])
    st, c = out["stats"], ref["counters"]
    assert (st["primary"], st["reflection"], st["shadow"]) == (c["primary"], c["reflection"], c["shadow"])
    assert st["fallbacks"] > 0  # the centre column (dir.x == 0) takes the strict walk


def test_errors_are_reported(dev, scenes):
    r = dev.Renderer(0)
    with pytest.raises(dev.RtError):
        r.render(host.camera(16, 16), 16, 16)  # before upload: RT_E_STATE
    r.upload(scenes["car_only"])
    with pytest.raises(dev.RtError):
        r.render(host.camera(16, 16), 16, 16, rows=(10, 1, 10))  # rows outside the frame
    with pytest.raises(dev.RtError):
        r.render(host.camera(16, 16), 16, 16, spp=3)
    with pytest.raises(dev.RtError):
        r.render(host.camera(16, 16), 16, 16, bounces=0)
    r.close()


@pytest.mark.parametrize("kernel", KERNELS)
def test_bounce_hits_match_oracle(dev, scenes, kernel):
    """per-level closest-hit indices: -1 miss, -2 level not reached, every level bit-exact"""
    import torch
    from tests.oracle_bind import OracleScene
    from tests.scenes import scene_paths
    o = OracleScene.load(*scene_paths("car_boxed"))
    o.build_bvh(3)
    ref = o.render(128, 72, bounce_hits=True)
    r = dev.Renderer(0)
    r.upload(scenes["car_boxed"])
    bh = torch.full((72, 128, 4), -9, dtype=torch.int32, device="cuda")
    rgb = torch.empty((72, 128, 3), dtype=torch.float32, device="cuda")
    r.render(host.camera(128, 72), 128, 72, kernel=select(kernel), rgb=rgb, bounce_hit=bh)
    r.sync()
    np.testing.assert_array_equal(bh.cpu().numpy(), ref["bounce_hit"])
    assert same_bits(rgb.cpu().numpy(), ref["rgb"])
    r.close()


def test_download_bmp_is_the_reference_writers_bytes(dev, scenes):
    """on-GPU BGRA8 quantisation == rth_bmp_encode == bmp_write_file (tests/test_host.py)"""
    ref = np.load(os.path.join(GOLD, "car_boxed_160x90_strict.npz"))
    r = dev.Renderer(0)
    r.upload(scenes["car_boxed"])
    r.render(host.camera(160, 90), 160, 90)
    data = r.download_bmp()
    assert data == host.bmp_encode(ref["rgb"])
    rgb, _ = r.download()
    assert data == host.bmp_encode(rgb)
    with pytest.raises(dev.RtError):  # a row subset is not a BMP
        r.render(host.camera(160, 90), 160, 90, rows=(1, 2, 45))
        r.download_bmp()
    r.close()


@pytest.mark.parametrize("n", [2, 3])
def test_gather_rows_of_several_contexts(dev, scenes, n):
    """rt_gather (in-process multi-GPU): n contexts render cyclic row sets, the root
    gathers them; equal to one full-frame render, BMP included (same-device path on a 1-GPU box)"""
    import torch
    W, H = 200, 113
    full = render(dev, scenes["car_boxed"], W, H, "fast")
    rs = [dev.Renderer(0) for _ in range(n)]
    bufs = []
    from prt.dist import rank_rows
    for block in (1, 8):  # cyclic rows, then 8-row blocks dealt cyclically (the bench's N > 1 layout)
        for g, r in enumerate(rs):
            r.upload(scenes["car_boxed"])
            rows = rank_rows(H, g, n, block)
            hit = torch.empty((rows[2], W), dtype=torch.int32, device="cuda")
            r.render(host.camera(W, H), W, H, rows=rows, hit=hit)
            bufs.append(hit)
        dev.gather(rs, root=1)
        rgb, hit = rs[1].download(hit=True)
        assert same_bits(rgb, full["rgb"]), block
        np.testing.assert_array_equal(hit, full["hit"])
        assert rs[1].download_bmp() == host.bmp_encode(full["rgb"])
    bad = dev.Renderer(0)
    bad.upload(scenes["car_boxed"])
    bad.render(host.camera(W, H), W, H, rows=(0, 2, 57))
    with pytest.raises(dev.RtError):  # rows 1, 3, ... missing
        dev.gather([bad], root=0)
    for r in rs + [bad]:
        r.close()


def test_cli_drop_in_writes_the_reference_bmp(tmp_path):
    """bin/raytracer (the cpu/raytracer drop-in): stdout metric lines and <scene>.bmp byte-identical to
    the reference renderer's output for the same frame (fixture rgb -> bmp_write_file bytes)"""
    import subprocess
    from tests.scenes import scene_paths
    exe = os.path.join(os.path.dirname(GOLD), "..", "parallel-ray-tracer_amd", "bin", "raytracer")
    assets = os.path.dirname(os.path.dirname(scene_paths("car_boxed")[0]))
    ref = np.load(os.path.join(GOLD, "car_boxed_160x90_strict.npz"))
    cache = tmp_path / "cache"
    cache.mkdir()
    for run in range(2):  # the second run reads triangles and BVH from the binary cache
        out = tmp_path / f"car_boxed{run}.bmp"
        r = subprocess.run([exe, "4", "--scene", "car_boxed", "--assets", assets, "--width", "160", "--height", "90",
                            "--iterations", "3", "--out", str(out), "--cache", str(cache)], capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        for line in ("Number of triangles: 45999", "Frame time (median):",
                     "Rays per frame (primary+reflection+shadow):"):
            assert line in r.stdout, line
        assert out.read_bytes() == host.bmp_encode(ref["rgb"])
    assert len(list(cache.iterdir())) == 2


def test_tune_is_the_default_rule_and_removed_variants_are_refused(dev, scenes):
    """rt_frame.tune: 1 is accepted and runs the default rule (the round-2 autotuner it selected was slower than the
    measured rule everywhere and was removed), other values are refused; so are the removed variants (k_fan = 7, ...)
    and hot kernels (RT_HOT_FAN = 2). A tune = 1 frame equals a tune = 0 frame bit for bit, with the same ray counts."""
    import torch
    W, H = 96, 54
    outs = []
    for tune in (0, 1):
        r = dev.Renderer(0, counters=True)
        r.upload(scenes["car_boxed"])
        rgb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        r.render(host.camera(W, H), W, H, rgb=rgb, tune=tune)
        r.sync()
        outs.append((rgb.cpu().numpy(), r.stats()["rays"]))
        r.close()
    assert same_bits(outs[0][0], outs[1][0]) and outs[0][1] == outs[1][1]
    r = dev.Renderer(0)
    r.upload(scenes["car_boxed"])
    for kw in ({"tune": 2}, {"variant": 7}, {"variant": 3}, {"variant": 14}, {"hot_pct": 50, "hot_kernel": 2}):
        fr = _frame_with(r, W, H, kw)
        rc = dev._L.rt_render(r._ctx, ctypes.byref(host.camera(W, H)), ctypes.byref(fr), ctypes.byref(dev.Outputs()))
        assert rc == -1, (kw, rc)  # RT_E_ARG
    r.close()


def test_launch_pixel_bound_is_refused(dev, scenes):
    """the kernels index a launch's output pixels (frames x rows x width) with 32-bit integers: rt_render refuses a
    launch of more than 2^31 - 1 pixels (RT_E_ARG) before it allocates or launches anything"""
    r = dev.Renderer(0)
    r.upload(scenes["car_boxed"])
    W = H = 46341  # 2,147,488,281 pixels
    fr = _frame_with(r, W, H, {})
    rc = dev._L.rt_render(r._ctx, ctypes.byref(host.camera(W, H)), ctypes.byref(fr), ctypes.byref(dev.Outputs()))
    msg = dev._L.rt_last_error(r._ctx).decode()
    r.close()
    assert rc == -1 and "2^31" in msg, (rc, msg)


def _frame_with(r, W, H, f):
    """an rt_frame for the full W x H frame with raw launch fields (values the Python mirror would not produce)"""
    fr, _ = r._frame(W, H, None, 4, 1, "fast", 0, False, 0, "default", 0)
    fr.tune = f.get("tune", 0)
    fr.variant = f.get("variant", 0)
    fr.hot_pct = f.get("hot_pct", 0)
    fr.hot_kernel = f.get("hot_kernel", 0)
    return fr


def moved_camera(W, H, dx, dz):
    """the reference camera translated by (dx, 0, dz): another frame of a camera sequence"""
    c = host.camera(W, H)
    for v in (c.pos, c.ul):
        v.x += dx
        v.z += dz
    return c


@pytest.mark.parametrize("kernel", ["fast", "coop4", "strict", "shpool", "shdefer"])
@pytest.mark.parametrize("name", ["car_boxed", "dragon"])
def test_frame_batch_equals_single_frames(dev, name, kernel):
    """rt_render_frames: a batch of frames (different cameras, one persistent launch on the fast paths)
    renders every frame bit for bit as rt_render does it alone, including a row subset; its counters
    are the sum of the frames'; frame 0 (the reference camera) matches the reference fixture"""
    import torch
    s = host.Scene.named(name).build_bvh(3)
    W, H = 96, 54
    cams = [host.camera(W, H), moved_camera(W, H, 0.25, 0.0), moved_camera(W, H, -0.4, 0.3)]
    for rows in (None, (1, 3, 18)):
        nr = rows[2] if rows else H
        singles = []
        for c in cams:
            r = dev.Renderer(0, counters=True)
            r.upload(s)
            rgb = torch.empty((nr, W, 3), dtype=torch.float32, device="cuda")
            hit = torch.empty((nr, W), dtype=torch.int32, device="cuda")
            r.render(c, W, H, rows=rows, kernel=select(kernel), rgb=rgb, hit=hit)
            r.sync()
            singles.append((rgb.cpu().numpy(), hit.cpu().numpy(), r.stats()))
            r.close()
        r = dev.Renderer(0, counters=True)
        r.upload(s)
        rgb = torch.full((len(cams), nr, W, 3), -1.0, dtype=torch.float32, device="cuda")
        hit = torch.full((len(cams), nr, W), -7, dtype=torch.int32, device="cuda")
        r.render_frames(cams, W, H, rows=rows, kernel=select(kernel), rgb=rgb, hit=hit)
        r.sync()
        st = r.stats()
        r.close()
        for i, (srgb, shit, _) in enumerate(singles):
            assert same_bits(rgb[i].cpu().numpy(), srgb), (kernel, rows, i)
            np.testing.assert_array_equal(hit[i].cpu().numpy(), shit)
        for k in ("primary", "reflection", "shadow", "shadow_skipped", "hits", "pixels"):
            assert st[k] == sum(x[2][k] for x in singles), (kernel, rows, k)
        assert not np.array_equal(singles[0][1], singles[1][1])  # the cameras differ
        if rows is None and name != "car_boxed":
            ref = np.load(os.path.join(GOLD, f"{name}_96x54_strict.npz"))
            assert same_bits(rgb[0].cpu().numpy(), ref["rgb"])


@pytest.mark.parametrize("kernel", ["fast"])
@pytest.mark.parametrize("dealing", ["global", "rows", "columns", "row_major"])
def test_xcd_aware_dealing_renders_the_same_frames(dev, dealing, kernel):
    """the persistent kernels' tile dealing (rt_frame.dealing, rtd::next_item): one global counter, 8 row
    bands, 8 column bands, row-major, against 4 x 2 blocks drained first by their own XCD — the same bits
    for a frame, a row subset and a frame batch, and the same ray counts"""
    import torch
    s = host.Scene.named("dragon").build_bvh(3)
    W, H = 200, 120
    outs = {}
    for v in ("blocks", dealing):
        a = render_dealt(dev, s, W, H, kernel, v, counters=True)
        b = render_dealt(dev, s, W, H, kernel, v, rows=(8, 24, 40, 8))
        r = dev.Renderer(0)
        r.upload(s)
        rgb = torch.empty((3, H, W, 3), dtype=torch.float32, device="cuda")
        r.render_frames([host.camera(W, H)] * 3, W, H, kernel=kernel, rgb=rgb, dealing=v)
        r.sync()
        outs[v] = (a, b, rgb.cpu().numpy())
        r.close()
    (a0, b0, f0), (a1, b1, f1) = outs["blocks"], outs[dealing]
    assert same_bits(a0["rgb"], a1["rgb"]) and same_bits(b0["rgb"], b1["rgb"]) and same_bits(f0, f1)
    np.testing.assert_array_equal(a0["hit"], a1["hit"])
    assert a0["stats"]["rays"] == a1["stats"]["rays"]
    for i in range(3):
        assert same_bits(f1[i], a0["rgb"])


def render_dealt(dev, scene, W, H, kernel, dealing, rows=None, counters=False):
    import torch
    r = dev.Renderer(0, counters=counters)
    r.upload(scene)
    nr = rows[2] if rows else H
    rgb = torch.empty((nr, W, 3), dtype=torch.float32, device="cuda")
    hit = torch.empty((nr, W), dtype=torch.int32, device="cuda")
    r.render(host.camera(W, H), W, H, rows=rows, kernel=kernel, rgb=rgb, hit=hit, dealing=dealing)
    r.sync()
    out = {"rgb": rgb.cpu().numpy(), "hit": hit.cpu().numpy(), "stats": r.stats()}
    r.close()
    return out


def quantise(rgb):
    """vec_to_bgra (cpu/src/bmp_writer.c:88-95) of f32 pixels -> packed uint32 B | G << 8 | R << 16 | 255 << 24"""
    q = (np.asarray(rgb, np.float32) * np.float32(255.0)).astype(np.uint8).astype(np.uint32)
    return q[..., 2] | (q[..., 1] << 8) | (q[..., 0] << 16) | np.uint32(255 << 24)


@pytest.mark.parametrize("kernel", KERNELS)
def test_bgra_output_is_the_bmp_writers_quantisation(dev, scenes, kernel):
    """rt_outputs.bgra (the kernels quantise as they store): equal to vec_to_bgra of the same
    frame's f32 pixels, with or without an rgb output, for a frame, a row-block subset and a frame batch;
    the full frame's rows bottom-up are bmp_write_file's pixel bytes of the reference fixture"""
    import torch
    W, H = 160, 90
    s = scenes["car_boxed"]
    ref = np.load(os.path.join(GOLD, "car_boxed_160x90_strict.npz"))
    for rows in (None, (8, 24, 24, 8)):
        nr = rows[2] if rows else H
        r = dev.Renderer(0)
        r.upload(s)
        rgb = torch.empty((nr, W, 3), dtype=torch.float32, device="cuda")
        both = torch.zeros((nr, W), dtype=torch.int32, device="cuda")
        only = torch.zeros((nr, W), dtype=torch.int32, device="cuda")
        r.render(host.camera(W, H), W, H, rows=rows, kernel=select(kernel), rgb=rgb, bgra=both)
        r.render(host.camera(W, H), W, H, rows=rows, kernel=select(kernel), bgra=only)
        r.sync()
        q = quantise(rgb.cpu().numpy())
        np.testing.assert_array_equal(both.cpu().numpy().view(np.uint32), q)
        np.testing.assert_array_equal(only.cpu().numpy().view(np.uint32), q)
        with pytest.raises(dev.RtError):  # a bgra-only frame has no f32 pixels to download
            r.download()
        if rows is None:
            bmp = host.bmp_encode(ref["rgb"])
            assert only.cpu().numpy()[::-1].tobytes() == bmp[54:]
        batch = torch.zeros((2, nr, W), dtype=torch.int32, device="cuda")
        r.render_frames([host.camera(W, H), moved_camera(W, H, 0.25, 0.0)], W, H, rows=rows,
                        kernel=select(kernel), bgra=batch)
        r.sync()
        np.testing.assert_array_equal(batch[0].cpu().numpy().view(np.uint32), q)
        assert not np.array_equal(batch[1].cpu().numpy(), batch[0].cpu().numpy())
        r.close()


@pytest.mark.parametrize("name", ["dragon", "car_boxed"])
def test_path_level_placements_render_the_same_frames(dev, name):
    """path levels in registers (k_persist, 3 waves/SIMD), in the LDS path buffer (k_persist at 4 waves/SIMD, and the
    shadow pool's hand-off slots): the same bits for a frame, a frame batch with a moved camera and 4 spp, with the same ray counts"""
    import torch
    s = host.Scene.named(name).build_bvh(3)
    W, H = 200, 120
    outs = {}
    for v in ("persist", "persist4", "shpool"):
        a = render(dev, s, W, H, v, counters=True)
        b = render(dev, s, W, H, v, spp=4)
        r = dev.Renderer(0)
        r.upload(s)
        rgb = torch.empty((3, H, W, 3), dtype=torch.float32, device="cuda")
        r.render_frames([host.camera(W, H), moved_camera(W, H, 0.25, 0.0), host.camera(W, H)], W, H,
                        kernel=v, rgb=rgb)
        r.sync()
        outs[v] = (a, b, rgb.cpu().numpy())
        r.close()
    a0, b0, f0 = outs["persist"]
    assert same_bits(f0[0], a0["rgb"]) and same_bits(f0[2], a0["rgb"])
    for v in ("persist4", "shpool"):
        a1, b1, f1 = outs[v]
        assert same_bits(a0["rgb"], a1["rgb"]) and same_bits(b0["rgb"], b1["rgb"]) and same_bits(f0, f1), v
        np.testing.assert_array_equal(a0["hit"], a1["hit"])
        assert a0["stats"]["rays"] == a1["stats"]["rays"], v


@pytest.mark.parametrize("kernel", ["fast", "coop4", "shpool", "shdefer"])
def test_rotated_row_blocks_cover_every_frame(dev, kernel):
    """rt_frame.frame_shift: frame f of rank q renders block residue (q + f) % N (prt.dist rotate), rows
    past the image skipped — over the N ranks every frame of the batch is rendered exactly once, bit for
    bit the single full-frame renders, with the full frames' ray counts"""
    import torch
    from prt.dist import padded_rows
    s = host.Scene.named("dragon").build_bvh(3)
    W, H, N, B = 96, 54, 3, 8
    cams = [host.camera(W, H), moved_camera(W, H, 0.25, 0.0), moved_camera(W, H, -0.4, 0.3), host.camera(W, H)]
    full, rays = [], 0
    for c in cams:
        r = dev.Renderer(0, counters=True)
        r.upload(s)
        rgb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        r.render(c, W, H, kernel=select(kernel), rgb=rgb)
        r.sync()
        full.append(rgb.cpu().numpy())
        rays += r.stats()["rays"]
        r.close()
    n = padded_rows(H, N, B)
    got = np.full((len(cams), H, W, 3), -1.0, np.float32)
    seen = np.zeros((len(cams), H), np.int32)
    total = 0
    for q in range(N):
        r = dev.Renderer(0, counters=True)
        r.upload(s)
        rgb = torch.full((len(cams), n, W, 3), -2.0, dtype=torch.float32, device="cuda")
        r.render_frames(cams, W, H, rows=(q * B, N * B, n, B, B), kernel=select(kernel), rgb=rgb)
        r.sync()
        total += r.stats()["rays"]
        r.close()
        out = rgb.cpu().numpy()
        for f in range(len(cams)):
            off = (q * B + f * B) % (N * B)
            for k in range(n):
                y = off + (k // B) * N * B + k % B
                if y < H:
                    got[f, y] = out[f, k]
                    seen[f, y] += 1
    assert (seen == 1).all()
    for f in range(len(cams)):
        assert same_bits(got[f], full[f]), (kernel, f)
    assert total == rays
    r = dev.Renderer(0)
    r.upload(s)
    with pytest.raises(dev.RtError):  # rotation is a fast-kernel feature
        r.render_frames(cams, W, H, rows=(0, N * B, n, B, B), kernel="strict")
    r.close()


@pytest.mark.parametrize("name", ["dragon", "car_boxed"])
def test_hybrid_frames_equal_persistent_frames(dev, name):
    """RT_VARIANT_HYBRID (rt_hip.hip launch_hybrid): the measuring frame (k_persist with per-tile times), frames
    while the measurement is in flight, and the frames after it (the costliest tiles through k_coop<4> on a second
    stream, the rest through k_persist) all equal a forced k_persist frame bit for bit, with the same ray counts;
    also for a row subset, a moved camera (measured again), and the thresholds that make every / no tile hot"""
    import torch
    s = host.Scene.named(name).build_bvh(3)
    W, H = 200, 120
    for rows, pct in ((None, 0), (None, 1), (None, 100), ((8, 24, 40, 8), 0), (None, 60)):
        nr = rows[2] if rows else H
        cams = [host.camera(W, H), moved_camera(W, H, 0.25, 0.0)]
        for cam in cams:
            ref = render_cam(dev, s, W, H, cam, "persist", rows=rows)
            r = dev.Renderer(0, counters=True)
            r.upload(s)
            # frame 0 measures, frame 1 is issued while the measurement is in flight (the default launch, most
            # likely), frames 2.. (each after a sync) try the candidate thresholds and k_persist, then the choice
            for group in ((0, 1),) + tuple((i,) for i in range(2, 27)):
                outs = []
                for frame in group:
                    hit = torch.full((nr, W), -7, dtype=torch.int32, device="cuda")
                    rgb = torch.zeros((nr, W, 3), dtype=torch.float32, device="cuda")
                    r.render(cam, W, H, rows=rows, kernel="hybrid", hot_pct=pct, rgb=rgb, hit=hit)
                    outs.append((frame, hit, rgb))
                r.sync()
                for frame, hit, rgb in outs:
                    np.testing.assert_array_equal(hit.cpu().numpy(), ref["hit"])
                    assert same_bits(rgb.cpu().numpy(), ref["rgb"]), (rows, pct, frame)
                st = r.stats()
                for k in ("primary", "reflection", "shadow", "shadow_skipped", "hits", "pixels"):
                    assert st[k] == ref["stats"][k], (rows, pct, group, k)
            r.close()


def render_cam(dev, scene, W, H, cam, kernel, rows=None):
    import torch
    r = dev.Renderer(0, counters=True)
    r.upload(scene)
    nr = rows[2] if rows else H
    hit = torch.empty((nr, W), dtype=torch.int32, device="cuda")
    rgb = torch.empty((nr, W, 3), dtype=torch.float32, device="cuda")
    r.render(cam, W, H, rows=rows, kernel=kernel, rgb=rgb, hit=hit)
    r.sync()
    out = {"rgb": rgb.cpu().numpy(), "hit": hit.cpu().numpy(), "stats": r.stats()}
    r.close()
    return out


def test_kernel_errors_fail_sync_and_download(dev):
    """a traversal-stack overflow (rtd::C_ERR) fails rt_sync, rt_download and rt_get_stats (RT_E_KERNEL, -8) instead of
    passing a truncated walk's frame as good: a handed-over BVH (accel="reference") 40 levels deep, whose nearer child
    at every level is the interior one, so the farther leaf of each level stays on the walk's 34-entry stack"""
    import torch
    base = host.Scene.named("car_only")
    n = 41
    tris = np.ascontiguousarray(base.triangles[:n])
    s = host.Scene(tris, base.lights)
    nodes = [None]
    big = ((-1e4, -1e4, -1e4), (1e4, 1e4, 1e4))

    def node(tr_len, child):
        return (big[0], big[1], tr_len, child)
    cur, leaf = 0, 0
    for level in range(n - 1):
        c = len(nodes)
        last = level == n - 2
        nodes += [None, node(1, leaf)]  # (left, right = a leaf); ties: the left (interior) child is walked first
        leaf += 1
        nodes[cur] = node(0, c)
        if last:
            nodes[c] = node(1, leaf)
            leaf += 1
        cur = c
    s.nodes = np.array(nodes, dtype=host.NODE_DTYPE)
    s.tri_idx = np.arange(n, dtype=np.int32)
    for kernel in ("strict", "fast"):
        r = dev.Renderer(0)
        r.upload(s, accel="reference")
        rgb = torch.empty((16, 16, 3), dtype=torch.float32, device="cuda")
        r.render(host.camera(16, 16), 16, 16, kernel=kernel, rgb=rgb)
        with pytest.raises(dev.RtError, match="-8"):
            r.sync()
        with pytest.raises(dev.RtError, match="-8"):
            r.download()
        with pytest.raises(dev.RtError, match="-8"):
            r.stats()
        r.close()


@pytest.mark.parametrize("scale", [0.25, 8.0, 1000.0])
def test_scaled_scene_vs_oracle(dev, tmp_path, scale):
    """car_boxed with every vertex and light position scaled (the camera stays): the fast walks' box tests on
    rescaled t (the shadow walks' [BOX_TMIN, reach] -> [0, 1], the closest walks' 2^-40 scale) and the inflation
    margins hold from a scene a quarter the size to one a thousand times it; every kernel against the oracle"""
    import shutil
    from tests.oracle_bind import OracleScene
    from tests.scenes import scene_paths
    obj, mtl, lts = scene_paths("car_boxed")
    out_lines = []
    for ln in open(obj).read().splitlines():
        if ln.startswith("v "):
            x, y, z = (float(v) * scale for v in ln.split()[1:4])
            ln = f"v {x:.6f} {y:.6f} {z:.6f}"
        out_lines.append(ln)
    o2, m2, l2 = tmp_path / "triangles.obj", tmp_path / "triangles.mtl", tmp_path / "lights.obj"
    o2.write_text("\n".join(out_lines) + "\n")
    shutil.copy(mtl, m2)
    lines = []
    for ln in open(lts).read().splitlines():
        f = ln.split()
        lines.append(" ".join([f"{float(v) * scale:.6f}" for v in f[:3]] + f[3:]))
    l2.write_text("\n".join(lines) + "\n")
    o = OracleScene.load(str(o2), str(m2), str(l2))
    o.build_bvh(3)
    ref = o.render(96, 54)
    s = host.Scene.load(str(o2), str(m2), str(l2)).build_bvh(3)
    assert ref["counters"]["shadow"] > 0
    for k in KERNELS:
        out = render(dev, s, 96, 54, k, counters=True)
        np.testing.assert_array_equal(out["hit"], ref["hit"], err_msg=f"{k} x{scale}")
        assert same_bits(out["rgb"], ref["rgb"]), (k, scale)
        assert out["stats"]["shadow"] == ref["counters"]["shadow"], (k, scale)
