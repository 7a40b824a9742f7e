#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: Mrays/s (primary + secondary) on dragon at 1920x1080, 1/2/4/8 MI355X.

One step = one full frame of the hot path (ray generation, BVH traversal, ray-triangle intersection,
shading with shadow rays, 4 reflection bounces, clamp, and the BMP writer's BGRA8 quantisation written by
the kernel itself: --output bgra8) for the workload below, with the scene resident in HBM
before timing starts; for N > 1 the frame's rows are dealt over the ranks in 8-row blocks (block j on
rank j % N: cost-balanced) and gathered to rank 0 over RCCL inside the timed region (4 bytes
per pixel; --output rgb writes and gathers the 12-byte f32 pixels instead).

Frames in flight: the K timed frames (the reference's ITERATIONS loop of one camera, main.c) are traced
in batches of F frames per launch (rt_render_frames: one persistent launch whose tile dealing interleaves
the batch's frames, so the long reflection chains of one frame overlap the others' work instead of
leaving the chip idle at the frame's tail), and each batch's gather overlaps the next batch's render
(ping-pong blocks). Every frame is traced in full into its own output (bit-exact to a single rt_render,
tests/test_gpu_parity.py::test_frame_batch_equals_single_frames); the single-frame kernel latency is
reported next to the throughput (frame_latency_ms).

Rays counted as the reference defines its work: primary + traced reflection + traced
shadow rays (light_v calls past the back-face test), from the kernel's own counters (equal to the
oracle's; tests/test_gpu_parity.py).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 via torch.distributed.run (one rank
per GPU, RCCL). Prints ONE JSON line on rank 0.
"""
import argparse
import json
import math
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "parallel-ray-tracer_amd"))
sys.path.insert(0, ROOT)

METRIC = "Mrays/sec (primary+secondary) on dragon at 1920×1080, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
N_SIMD = 1024  # 256 CUs x 4 SIMDs


def alg_bytes(st, pixels, n_lights, px_bytes=12):
    """Algorithmic bytes of one launch from the kernel's traversal counters:
    BVH records read (node_bytes, counted on the device: 80 B per wide-node visit of the fast walk,
    64 B per child-pair node + 8 B per leaf record of the strict fallback walk), 48 B per triangle
    test (v0, e1, e2, n), per closest hit 4 + 32 + 48 B (tri_orig, normals + material id, material),
    32 B per light per hit, px_bytes per pixel written (4: the BGRA8 pixel, 12: f32 rgb)."""
    tri = st["ch_tri"] + st["sh_tri"]
    nodes = st.get("node_bytes") or (64 * (st["ch_inner"] + st["sh_inner"]) + 8 * (st["ch_leaf"] + st["sh_leaf"]))
    return nodes + 48 * tri + (84 + 32 * n_lights) * st["hits"] + px_bytes * pixels


def pmc_key(args, frames, world):
    """profiles/pmc_traffic.json key of one bench configuration (tools/pmc_traffic.py takes it from the bench line):
    every argument that changes what the profiled launches run"""
    a = args
    return (f"{a.scene}_{a.width}x{a.height}_spp{a.spp}_b{a.bounces}_{a.kernel}_{a.variant}_"
            f"{a.bvh}_{a.accel}_r{a.ploc_radius}_{a.output}_o{a.orbit:g}_rb{a.row_block}_s{a.streams}"
            f"{'_norot' if a.no_rotate else ''}_f{frames}_n{world}")


def data_note(name, n_tris, is_standin):
    if name.startswith("random"):
        return (f"synthetic: the reference's random-triangle mode (cpu/src/main.c:115-131, srand(1)), {n_tris} "
                "triangles in [-5, 5]^3, no lights")
    if name in ("dragon", "dragon871k") and is_standin(name):
        return ("synthetic stand-in mesh: the reference snapshot has no assets/dragon/triangles.obj "
                "(.MISSING_LARGE_BLOBS); prt/scenes.py generates a Cornell room + torus-knot tube "
                f"({n_tris} triangles) with the real dragon .mtl and lights.obj")
    if is_standin(name):
        return (f"synthetic stand-in mesh ({n_tris} triangles, prt/scenes.py) with the real {name} .mtl and "
                "lights.obj: the snapshot has no mesh for this scene (.MISSING_LARGE_BLOBS)")
    return "reference asset"


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def parse_count(txt):
    """'1m' -> 1000000, '200k' -> 200000, '5000' -> 5000"""
    mul = {"k": 1000, "m": 1000000}.get(txt[-1:].lower(), 1)
    return int(txt[:-1] if mul > 1 else txt) * mul


def avx512_host():
    """the AVX-512 subsets -march=x86-64-v4 needs are on this host (and the v4 reference build exists)"""
    try:
        flags = next(l for l in open("/proc/cpuinfo") if l.startswith("flags")).split()
    except (OSError, StopIteration):
        return False
    need = ("avx512f", "avx512bw", "avx512cd", "avx512dq", "avx512vl")
    return all(f in flags for f in need) and os.access(os.path.join(ROOT, "oracle", "_ref", "rt_ref_v4"), os.X_OK)


def usable_cpus():
    """CPUs this process can actually use: its affinity set, capped by the cgroup v2 CPU quota (the GPU box
    shares a 256-CPU host: 16 CPUs of quota per GPU)"""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def survey_bytes(st, pixels, n_lights, px_bytes):
    """SURVEY §8d's byte model on the same counters: B_ray = 32 (1 + 2 I) + 40 T with the reference's record
    sizes (32-B bvh_t box per tested box, 36 B of vertices + 4 B tri_idx per triangle test), plus per hit 12 B
    normal + 36 B material + 24 B per light and the pixel. The wide walk tests the 8 child boxes of every
    visited node (8 x 32 B per visit); strict fallbacks' binary visits are in the same counters (2 boxes
    would be the exact figure: the difference is < 0.1 %)."""
    rays = st["primary"] + st["reflection"] + st["shadow"]
    boxes = 8 * (st["ch_inner"] + st["sh_inner"])
    return 32 * (rays + boxes) + 40 * (st["ch_tri"] + st["sh_tri"]) + (48 + 24 * n_lights) * st["hits"] + \
        px_bytes * pixels


def cpu_baseline(scene_files, W, H, gpu_rays_for_rows, args, threads):
    """The reference itself (oracle/_ref/rt_ref_fast: cpu/src/*.c built with the makefile's flags) timed
    on this host, pthreads with the reference's atomic row scheduler; falls back to the C restatement
    built the same way (kind "port") when the prebuilt reference binary is absent."""
    stride = args.cpu_row_stride
    v4 = avx512_host()
    ref = os.path.join(ROOT, "oracle", "_ref", "rt_ref_v4" if v4 else "rt_ref_fast")
    obj, mtl, lts = scene_files
    if os.path.exists(ref) and os.access(ref, os.X_OK):
        kind = "reference"

        def run(rows_stride, reps, nthreads=threads):
            out = subprocess.run([ref, "time", obj, mtl, lts, str(W), str(H), str(nthreads), "0", str(rows_stride),
                                  str(reps)], check=True, capture_output=True, text=True, timeout=600)
            return json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    else:
        kind = "port"
        from tests.oracle_bind import OracleScene

        o = OracleScene.load(obj, mtl, lts, flavour="fast")
        o.build_bvh(3)

        def run(rows_stride, reps, nthreads=threads):
            nr = (H + rows_stride - 1) // rows_stride
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                o.render(W, H, rows=(0, rows_stride, nr), threads=nthreads)
                ts.append((time.perf_counter() - t0) * 1e3)
            ts.sort()
            return {"median_ms": ts[len(ts) // 2], "rows": nr, "threads": nthreads, "reps": reps}
    if not stride:  # calibrate: aim at ~15 s of CPU work in total
        probe = run(16, 1)
        frame_s = probe["median_ms"] / 1e3 * 16
        stride = max(1, min(H, int(math.ceil(frame_s / 5.0))))
        reps = max(1, min(5, int(15.0 / max(frame_s / stride, 1e-3))))
    else:
        reps = args.cpu_reps
    res = run(stride, reps)
    rays = gpu_rays_for_rows(stride)
    out = {"value": rays / (res["median_ms"] / 1e3) / 1e6, "unit": "Mrays/s", "cores": threads, "kind": kind,
           "sample": f"rows y = k*{stride} of the same {W}x{H} frame ({res['rows']} rows, {rays} rays), "
                     f"median of {reps} frames, {threads} pthreads, reference atomic row scheduler, "
                     f"heuristic-3 BVH (build untimed)",
           "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
           "build": ("cpu/src/*.c with the reference makefile's -O3 -ffast-math -flto; -march=native (cpu/makefile:14) "
                     "is not available for a binary built in the build container (no reference sources on the GPU "
                     "box), so " + ("-march=x86-64-v4 -mtune=znver3 (AVX-512, what this host supports; gcc 11 "
                                    "knows no znver4/5)" if v4 else "-march=x86-64-v3 (AVX2 + FMA; no AVX-512 here)")
                     + " (oracle/Makefile)") if kind == "reference" else "oracle/port/oracle.c, -O3 -ffast-math"}
    # the same at 1 thread, on a ~5 s sample (every stride1-th row, one frame)
    if threads > 1 and not args.no_single_thread:
        frame_1t = res["median_ms"] / 1e3 * stride * threads
        stride1 = max(1, min(H, int(math.ceil(frame_1t / 5.0))))
        r1 = run(stride1, 1, 1)
        rays1 = gpu_rays_for_rows(stride1)
        out["single_thread"] = {"value": rays1 / (r1["median_ms"] / 1e3) / 1e6, "unit": "Mrays/s", "cores": 1,
                                "sample": f"rows y = k*{stride1} ({r1['rows']} rows, {rays1} rays), one frame"}
    return out


def spawn_ranks(n):
    """torch.distributed.run with n ranks on this node (rendezvous on 127.0.0.1, a free port) as a child
    process running this same command line; returns its exit status (non-zero if any rank failed)"""
    import socket
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64, help="timed frames")
    ap.add_argument("--warmup", type=int, default=16, help="untimed frames (after the tuning launches)")
    ap.add_argument("--frames", type=int, default=0,
                    help="frames per launch, at most --steps (0: 32 at N = 1, 16 at N > 1, where two streams' "
                         "alternating launches and the ping-pong gathers want at least two launches)")
    ap.add_argument("--streams", type=int, default=0, help="contexts on their own streams, launches alternating "
                    "(0: 1 at N = 1, 2 at N > 1)")
    ap.add_argument("--row-block", type=int, default=0,
                    help="N > 1: rows dealt to ranks in blocks of this many (0: 8, so 8x8 tiles stay 8x8 in the image)")
    ap.add_argument("--output", choices=("bgra8", "rgb"), default="bgra8",
                    help="what each frame's kernel writes and the gather moves: bgra8 = the BMP writer's quantised "
                         "pixel (rt_outputs.bgra, 4 B), rgb = the f32 vec_t pixel (12 B)")
    ap.add_argument("--variant", default="default", help="rt_frame.variant of the batches (prt.device.VARIANTS)")
    ap.add_argument("--no-rotate", action="store_true",
                    help="N > 1: keep each rank on its own block residue in every frame (default: frame f of rank "
                         "q renders residue (q + f) %% N, so every rank's batch costs the same)")
    ap.add_argument("--orbit", type=float, default=0.02,
                    help="camera path: frame i of a launch is the reference camera moved by i * ORBIT along x (0: the "
                         "reference's ITERATIONS loop of one camera, main.c:141-160)")
    ap.add_argument("--scene", default="dragon")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--bounces", type=int, default=4)
    ap.add_argument("--spp", type=int, default=1)
    ap.add_argument("--bvh", default="random", help="bvh_build heuristic handed over (reference default: 3 = random)")
    ap.add_argument("--accel", default="auto", help="auto / gpu: the library builds the fast walk's BVH on the GPU "
                    "(PLOC, rt_build.hpp; auto falls back to host); host: binned SAH on the host; reference: the "
                    "handed-over BVH")
    ap.add_argument("--ploc-radius", type=int, default=0, help="the GPU BVH build's neighbourhood (0: library default)")
    ap.add_argument("--no-single-thread", action="store_true", help="skip the 1-thread CPU baseline sample")
    ap.add_argument("--kernel", default="fast")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the single-frame latency measurement (tools/profile.sh: the profiled launches are then "
                         "only the batches, whose kernel is the same instantiation as a single frame's)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the CPU baseline (default 16, the GPU box's CPU share; also timed at every "
                         "host CPU, the line's cpu_baseline.all_cpus)")
    ap.add_argument("--no-all-cpus", action="store_true", help="skip the all-host-CPUs baseline sample")
    ap.add_argument("--cpu-row-stride", type=int, default=0)
    ap.add_argument("--cpu-reps", type=int, default=3)
    ap.add_argument("--bmp", default="", help="after timing, rank 0 writes the last frame (gathered) as a BMP "
                    "(bmp_write_file's bytes; from the device-quantised pixels with --output bgra8)")
    ap.add_argument("--gather", choices=("auto", "native", "torch"), default="auto",
                    help="N > 1: how frames reach rank 0 — native: the library's RCCL gather (rt_comm_init_rank / "
                         "rt_comm_gather_from, one communicator per rank shared by its contexts; torch.distributed only hands out "
                         "the id); "
                         "torch: torch.distributed.gather of the compact blocks (prt.dist.FrameGather); auto: native "
                         "on RCCL, torch on gloo (the one-GPU rehearsal: RCCL refuses two ranks on one device)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--timeout", type=float, default=240.0,
                    help="N > 1: seconds any rank may wait on a native gather (x 2 on the process group's collectives, "
                         "which agree on a gather's failure) and, x 2.5, on the whole run (a watchdog prints every thread's stack and "
                         "exits non-zero): a first multi-GPU run that deadlocks fails loudly instead of hanging")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` without a launcher: start the N ranks as CHILD processes (one per GPU, before
        # this process touches any GPU) and relay their exit status; rank 0 prints the line on the shared stdout
        sys.exit(spawn_ranks(args.gpus))

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:  # watchdog: a deadlock anywhere in a multi-rank run ends it with stacks and a non-zero status
        import faulthandler
        faulthandler.dump_traceback_later(2.5 * args.timeout + 60, exit=True)
    rank = int(os.environ.get("RANK", "0"))
    if args.gpus != world:  # never a silent one-GPU run labelled N
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-rank flow on a one-GPU box (never set by the driver): PRT_DIST_ONE_GPU=1 puts
    # every rank on device 0, PRT_DIST_BACKEND=gloo replaces RCCL (which refuses two ranks on one GPU)
    if os.environ.get("PRT_DIST_ONE_GPU") == "1":
        local = 0
    backend = os.environ.get("PRT_DIST_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import datetime

        import torch.distributed as dist

        tmo = datetime.timedelta(seconds=2 * args.timeout)  # (twice the native gather's: its failures are agreed on)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)

    from prt import device, host
    from prt.dist import FrameGather, NativeGather
    from prt.scenes import is_standin, scene_paths

    W, H = args.width, args.height
    if args.scene.startswith("random"):  # random-triangle mode (main.c:115-131): random<N>, e.g. random1m, random200k
        n_rand = parse_count(args.scene[len("random"):] or "10k")
        files = (f"random:{n_rand}", "-", "-")
        scene = host.Scene.random(n_rand).build_bvh(args.bvh)
    else:
        files = scene_paths(args.scene)
        scene = host.Scene.load(*files).build_bvh(args.bvh)
    stream = torch.cuda.current_stream().cuda_stream
    # N > 1: two contexts on two streams, launches alternating: a launch's tail (its longest reflection
    # chains) overlaps the next launch's work (tools/rank_rows.py --streams 2: 8-GPU rank rows 0.191 ->
    # 0.160 ms per frame; a whole frame at N = 1 gains ~1 %, and one stream keeps its launch durations —
    # the roofline's denominator — unshared)
    n_streams = args.streams or (1 if world == 1 else 2)
    streams = [torch.cuda.Stream() for _ in range(n_streams)]
    rends = [device.Renderer(local, stream=s.cuda_stream) for s in streams]
    for rr_ in rends:
        rr_.upload(scene, accel=args.accel, ploc_radius=args.ploc_radius)
    info = rends[0].scene_info()  # what the upload built (rt_get_scene_info): accel, wide depth, build time
    cam = host.camera(W, H)
    # a camera path: frame i of every launch is the reference camera moved by i * orbit along x (frame 0 IS the
    # reference's camera), so a batch's frames are all different (no identical rays in flight sharing caches)
    def path(nf):
        out = []
        for i in range(nf):
            c = host.camera(W, H)
            c.pos.x += i * args.orbit
            c.ul.x += i * args.orbit
            out.append(c)
        return out
    K = args.steps
    # launches covering exactly K frames, as few as --frames allows and of (nearly) equal size: K = 20 at 16
    # frames per launch is 10 + 10, not 16 + 4 (a 4-frame launch is tail-bound: 1.3 vs 0.93 ms per frame)
    # (N = 1, K = 20, same box: one 20-frame launch 0.813 ms per frame vs 10 + 10 0.845: the launch tail, its
    # longest reflection chains, is paid once)
    frames_cap = args.frames or (32 if world == 1 else 16)
    n_launch = -(-K // max(1, min(frames_cap, K)))
    plan = [K // n_launch + (1 if i < K % n_launch else 0) for i in range(n_launch)]
    F = plan[0]
    # rows: 8-row blocks dealt cyclically to the ranks (an 8x8 tile of a rank's rows is an 8x8 tile of the
    # image; costs average out over the blocks), gathered to rank 0 with one RCCL collective per batch
    # (prt/dist.py, tested with gloo in tests/test_multi.py); two ping-pong blocks so a batch's gather
    # overlaps the next batch's render
    B = args.row_block if args.row_block > 0 else (8 if world > 1 else 1)
    bgra = args.output == "bgra8"
    fg = FrameGather(H, W, 1 if bgra else 3, rank, world, dist,
                     like=torch.empty(0, dtype=torch.int32 if bgra else torch.float32, device="cuda"),
                     frames=F, buffers=2, block=B, rotate=not args.no_rotate)

    # N > 1: the frames reach rank 0 through the library's own RCCL gather (rt_comm_gather) unless --gather torch or
    # the gloo rehearsal; a native gather that cannot start, or whose frames differ from one GPU's at setup, is
    # replaced by torch.distributed's and the line says so (config.gather)
    gmode = ("native" if args.gather == "native" else "none") if world == 1 else \
        (args.gather if args.gather != "auto" else ("native" if backend == "nccl" else "torch"))
    gather_note = {"none": "single GPU", "torch": "torch.distributed.gather of the compact row blocks (prt.dist."
                   "FrameGather)", "native": "rt_comm_gather_from (the library's RCCL send/recv group, one communicator per rank "
                   "shared by its contexts, row sets exchanged once per layout; prt.dist.NativeGather)"}[gmode]
    ng = None
    if gmode == "native":
        err = ""
        try:
            ng = NativeGather(rends, H, W, 1 if bgra else 3, rank, world, dist, like=fg.blocks[0], frames=F, block=B,
                              rotate=not args.no_rotate, timeout=args.timeout)
        except Exception as e:  # e.g. RCCL not loadable: every rank sees the same
            err = repr(e)
        errs = [err]
        if dist:
            errs = [None] * world
            dist.all_gather_object(errs, err)
        if any(errs):
            if ng:
                ng.close()
            ng, gmode = None, "torch"
            gather_note = "torch.distributed.gather (native rt_comm_init_rank failed: " + next(e for e in errs if e) + ")"

    def out(blk):  # the kernel's output argument for a gather block
        return {"bgra": blk} if bgra else {"rgb": blk}
    my_rows = fg.rows()
    n_r = my_rows[2]
    launch_no = [0]
    latest = [0, 0, 0]  # (block, frames, context) of the latest launch
    # N > 1: the rule's choice for each launch size (frames per launch), agreed over the ranks after setup
    variant = {}

    def launch(nf, gather=True):
        # gather=False: the render alone (the N > 1 line's render-only timing: exposed gather = wall - render)
        b = launch_no[0] % 2
        c = launch_no[0] % n_streams
        launch_no[0] += 1
        latest[:] = [b, nf, c]
        if gmode == "native":  # render, then the gather on the context's stream (ordered after the render)
            rends[c].render_frames(path(nf), W, H, rows=my_rows, bounces=args.bounces, spp=args.spp,
                                   kernel=args.kernel, variant=variant.get(nf, args.variant), **out(ng.target(c)[:nf]))
            if gather:
                ng.gather(c, nf)
            return
        with torch.cuda.stream(streams[c]):  # block b is rendered by context c on its stream
            if fg.pending(b):
                fg.finish(b)
            rends[c].render_frames(path(nf), W, H, rows=my_rows, bounces=args.bounces, spp=args.spp,
                                   kernel=args.kernel, variant=variant.get(nf, args.variant), **out(fg.target(b)))
            if gather:
                fg.start(b)

    def drain():
        if gmode == "native":
            return  # ordered on the contexts' streams (the caller synchronises)
        for b in ((latest[0] + 1) % 2, latest[0]):  # launch order: rank 0's frame ends as the latest batch
            with torch.cuda.stream(streams[b % n_streams]):
                if fg.pending(b):
                    fg.finish(b)

    if gmode == "native":
        # the first multi-rank run of the native gather must not end the run: one probe launch + gather with bounded
        # waits (the descriptor exchange, the coverage check, rt_comm_wait); any rank's failure -> every rank falls
        # back to torch.distributed's gather (agreed over the process group, whose timeout is twice the gather's)
        err = ""
        try:
            launch(min(plan))
            ng.wait()
            torch.cuda.synchronize()
        except Exception as e:
            err = repr(e)
        errs = [err]
        if dist:
            errs = [None] * world
            dist.all_gather_object(errs, err)
        if any(errs):
            try:
                ng.close()
            except Exception:
                pass
            ng, gmode = None, "torch"
            gather_note = "torch.distributed.gather (the native gather's probe failed: " + next(e for e in errs if e) + ")"

    # setup, like the upload: the library's default rule measures its candidates on the first launches of a shape
    # (PERSIST4 vs the shadow pool, rt_get_launch_info: trial / settled), so
    # each batch size of the plan runs here until every context has settled, then `warmup` frames run untimed.
    rays_of = {}  # this rank's rays of a launch of nf frames (the same camera path every launch: deterministic)
    for nf in sorted(set(plan)):
        for i in range(32):
            launch(nf)
            if i >= 2 * n_streams - 1:
                if ng:
                    ng.wait()  # (bounded: a collective that never completes raises instead of hanging)
                torch.cuda.synchronize()
                settled = [all(r.launch_info()["settled"] for r in rends)]
                if dist:  # every rank stops together (the gathers are collective), once all have settled
                    every = [None] * world
                    dist.all_gather_object(every, settled[0])
                    settled = [all(every)]
                if settled[0]:
                    break
        if dist and args.variant == "default":
            # every rank measured the rule's candidates on its own row set; small, noisy launches may choose
            # differently, and a rank on the slower kernel would set the pace: every rank takes the choice most
            # contexts made for this launch size (ties: rank 0's), explicitly
            mine = [r.launch_info()["variant"] for r in rends]
            every = [None] * world
            dist.all_gather_object(every, mine)
            votes = [v for vs in every for v in vs]
            variant[nf] = max(dict.fromkeys(votes), key=votes.count)
            for _ in range(n_streams):
                launch(nf)
        rays_of[nf] = rends[(launch_no[0] - 1) % n_streams].stats()["rays"]
    if gmode == "native":  # untimed check of the native gather: rank 0's gathered frames == one GPU's frames
        drain()
        torch.cuda.synchronize()
        same = True
        if rank == 0:
            nf, c = latest[1], latest[2]
            rv = device.Renderer(local, stream=stream)
            rv.upload(scene, accel=args.accel, ploc_radius=args.ploc_radius)
            ref = torch.zeros_like(ng.frames_of(c)[:nf])
            rv.render_frames(path(nf), W, H, bounces=args.bounces, spp=args.spp, kernel=args.kernel, **out(ref))
            torch.cuda.synchronize()
            rv.close()
            same = bool(torch.equal(ref, ng.frames_of(c)[:nf]))
        flag = [same]
        if dist:
            dist.broadcast_object_list(flag, src=0)
        if not flag[0]:
            ng.close()
            ng, gmode = None, "torch"
            gather_note = "torch.distributed.gather (native rt_comm_gather's frames differed from one GPU's at setup)"
            for nf in sorted(set(plan)):
                launch(nf)
        else:
            gather_note += "; checked at setup: rank 0's gathered frames equal one GPU's"
    for _ in range(max(1, -(-args.warmup // F))):
        launch(F)
    drain()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    timed = []  # (context, frames) of every timed launch
    for nf in plan:
        timed.append((launch_no[0] % n_streams, nf))
        launch(nf)
    drain()
    if ng:  # bounded: a gather whose peer never came aborts the communicator and raises instead of hanging below
        ng.wait()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # per-launch kernel times of both contexts (HIP events on each launch's stream; overlapping launches
    # share the chip, so each one's duration is longer than its share of the wall time)
    kfull = []
    for b, rr_ in enumerate(rends):
        mine = [nf for (c, nf) in timed if c == b][-64:]  # this context's timed launches (the last ones)
        ts_ = rr_.kernel_times(len(mine)) if mine else []
        kfull += [t for t, nf in zip(ts_, mine) if nf == F]
    kfull = kfull or [float("nan")]
    # N > 1 (verdict r5 item 6: a first multi-rank run must be attributable from its one line): every rank's median
    # kernel ms per frame, and the exposed gather -- the timed region's wall time minus the slowest rank's wall time
    # for the same launches rendered without their gathers (each rank timed alone: no barrier inside)
    ranks_detail = None
    if world > 1:
        kmed = sorted(kfull)[len(kfull) // 2] / F
        launch_no[0] = 0  # (the same contexts in the same order as the timed launches)
        torch.cuda.synchronize()
        t_r = time.perf_counter()
        for nf in plan:
            launch(nf, gather=False)
        torch.cuda.synchronize()
        render_wall = time.perf_counter() - t_r
        every = [None] * world
        dist.all_gather_object(every, {"rank": rank, "kernel_ms_per_frame": kmed, "render_wall_ms": render_wall * 1e3,
                                       "variant": rends[timed[-1][0]].launch_info()["variant"]})
        ks = [e["kernel_ms_per_frame"] for e in every]
        walls = [e["render_wall_ms"] for e in every]
        ranks_detail = {"kernel_ms_per_frame": {"per_rank": ks, "min": min(ks), "max": max(ks),
                                                "spread": max(ks) / min(ks) - 1.0 if min(ks) > 0 else None},
                        "render_wall_ms": {"per_rank": walls, "max": max(walls)},
                        "variant_per_rank": [e["variant"] for e in every]}
    # whole-job rays of the timed launches: each launch's count (the counters of a launch of that many frames of
    # the camera path) summed over the plan and over the ranks (rotated rows: a rank's share differs frame by
    # frame, the frames' totals do not)
    assert rends[timed[-1][0]].stats()["rays"] == rays_of[plan[-1]]  # (deterministic: the same launch, again)
    rays_local = sum(rays_of[nf] for nf in plan)
    timed_launch = rends[timed[-1][0]].launch_info()  # what the timed launches ran (the rule's choice)
    if args.bmp and rank == 0:  # the BMP written from the root rank (untimed): frame 0 = the reference camera
        frames = ng.frames_of(latest[2]) if gmode == "native" else (fg.frame if world > 1 else fg.target(latest[0]))
        px = (frames if frames.dim() == 3 else frames[0]).cpu().numpy()
        data = host.bmp_from_bgra(px) if bgra else host.bmp_encode(px)
        with open(args.bmp, "wb") as fbmp:
            fbmp.write(data)
    el = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    rays_t = torch.tensor([rays_local], dtype=torch.float64, device="cuda")
    if dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(rays_t, op=dist.ReduceOp.SUM)
    elapsed = el.item()
    rays_total = int(rays_t.item())
    rays_frame = rays_total / K
    if ranks_detail is not None:
        ranks_detail["wall_ms"] = elapsed * 1e3
        ranks_detail["exposed_gather_ms"] = elapsed * 1e3 - ranks_detail["render_wall_ms"]["max"]
        ranks_detail["gather_mode"] = gmode
        ranks_detail["rule"] = ("kernel_ms_per_frame: each rank's median HIP-event time of its timed full-size launches "
                                "/ frames per launch; render_wall_ms: each rank's wall time for the timed plan's launches "
                                "without their gathers (timed alone after the timed region); exposed_gather_ms = the "
                                "timed region's wall time (max over ranks) - the slowest rank's render_wall_ms")

    # algorithmic bytes of this rank's full-batch launch: one extra untimed launch with traversal counters
    # (the timed launches' own configuration; a hybrid single frame's counters are its whole-frame kernel's, or
    # k_persist's when hot tiles went to k_coop: the counting launch never measures or tries)
    cv = timed_launch["variant"] if args.kernel != "strict" else args.variant
    if cv == "hybrid":
        cv = timed_launch["cold_variant"] if not timed_launch["hot_pct"] else "persist"
    rc = device.Renderer(local, counters=True, stream=stream)
    rc.upload(scene, accel=args.accel, ploc_radius=args.ploc_radius)
    rc.render_frames(path(F), W, H, rows=my_rows, bounces=args.bounces, spp=args.spp, kernel=args.kernel, variant=cv,
                     **out(fg.target(0)))
    stc = rc.stats()
    rc.close()
    bytes_launch = alg_bytes(stc, F * W * n_r, len(scene.lights), 4 if bgra else 12)
    survey_launch = survey_bytes(stc, F * W * n_r, len(scene.lights), 4 if bgra else 12)
    simd_eff = (stc["ch_inner"] + stc["sh_inner"]) / max(1, 64 * stc["wave_steps"])
    k_avg_ms = sum(kfull) / len(kfull)
    # Single-frame latency of this rank's rows: the drop-in seam as the reference drives it (cpu/src/main.c:171-185,
    # gpu/src/main.cu:110-115: one render_frame per iteration, each waited for) with the library's default rule.
    # RT_VARIANT_HYBRID measures and tries its candidates on the first frames of a shape (rt_get_launch_info: trial /
    # settled); the latency is the median HIP-event time of the frames after the rule has settled -- 72 of them for the
    # fixed camera (with the per-frame feedback no refresh frame is among them; a build without it refreshes the
    # lists with a settled measuring frame every 64 frames, `refresh`, reported on its own). Measured for the reference's fixed camera (frame_latency_ms), for a
    # walkthrough (every frame's camera moved: the rule is keyed by the frame's shape, so a moving camera settles the
    # same way), and for the fixed camera at the walkthrough's middle measured camera (fixed_at_walk_ms: the walk's
    # cameras see more of the reflective knot, so the walk is compared with a fixed camera where the walk is).
    px_out = out(fg.target(0)[0] if F > 1 else fg.target(0))

    def seam(cam_of, n_after=9, limit=120):
        rl = device.Renderer(local, stream=stream)
        rl.upload(scene, accel=args.accel, ploc_radius=args.ploc_radius)
        ts, idx, refresh, n, info = [], [], [], 0, {}
        while n < limit and len(ts) < n_after:
            rl.render(cam_of(n), W, H, rows=my_rows, bounces=args.bounces, spp=args.spp, kernel=args.kernel, **px_out)
            ms = rl.sync()
            info = rl.launch_info()
            if info["settled"]:
                ts.append(ms)
                idx.append(n)
                if info["refresh"]:
                    refresh.append(ms)
            n += 1
        rl.close()
        srt = sorted(ts)
        return {"median": srt[len(srt) // 2] if ts else float("nan"), "mean": sum(ts) / len(ts) if ts else float("nan"),
                "settle": n - len(ts), "info": info, "mid_camera": idx[len(idx) // 2] if idx else 0,
                "refresh_ms": refresh, "frames": len(ts), "ts": ts, "idx": idx}

    def walk(i):
        c = host.camera(W, H)
        c.pos.x += i * args.orbit
        c.ul.x += i * args.orbit
        return c
    nan = float("nan")
    if not args.no_latency:
        sd = seam(lambda i: cam, n_after=72)
        sw = seam(walk, n_after=16)
        # the walk against fixed cameras where it was: at 3 of its measured cameras (its quartiles), the fixed camera's
        # settled median vs the walk's frame at that camera (the walk's cameras differ in cost -- one may look past the
        # model, one may put the centre column's primary rays on a box face -- so a frame is compared with its own
        # camera, not with the walk's median or its neighbours)
        wcams, wat, wfix = [], [], []
        for q in (1, 2, 3):
            j = min(len(sw["idx"]) - 1, q * len(sw["idx"]) // 4)
            if j < 0:
                break
            k = sw["idx"][j]
            wcams.append(k)
            wat.append(sw["ts"][j])
            wfix.append(seam(lambda i, k=k: walk(k))["median"])
        sf = {"median": wfix[1] if len(wfix) > 1 else nan}
    else:
        sd = sw = sf = {"median": nan, "mean": nan, "settle": None, "info": None, "mid_camera": None, "refresh_ms": [],
                        "frames": 0}
        wcams, wat, wfix = [], [], []
    lat_default, settle_frames, seam_info = sd["median"], sd["settle"], sd["info"]
    lat_walk, settle_walk = sw["median"], sw["settle"]
    lat = torch.tensor([lat_default], dtype=torch.float64, device="cuda")
    if dist:
        dist.all_reduce(lat, op=dist.ReduceOp.MAX)

    if rank == 0:
        # PMC counters of THIS configuration, measured by tools/profile.sh on launches of THIS many frames with
        # THIS library build (pmc_key / lib_md5); anything else is reported under pmc_stale, never as measured
        pmc, pmc_stale = {}, None
        key = pmc_key(args, F, world)
        if os.path.exists(args.traffic_json):
            try:
                ent = json.load(open(args.traffic_json)).get(key)
            except (OSError, ValueError):
                ent = None
            if ent is not None:
                if ent.get("lib_md5") == device.lib_md5():
                    pmc = ent
                else:
                    pmc_stale = {"source": ent.get("source"), "reason": "measured on another librt_hip.so build"}
        traffic = pmc.get("hbm_bytes_per_launch")
        alg_gbs = bytes_launch / (k_avg_ms / 1e3) / 1e9  # algorithmic bytes per second (served by L1/L2/MALL)
        valu = pmc.get("valu_issue_frac")
        insts = pmc.get("sq_insts_valu_per_launch")
        # The roofline the line reports is the one that binds (verdict r4 item 7). With the scene cache-resident, HBM
        # carries a few % of the algorithmic bytes and binds nothing; the kernel is bound by VALU issue and dependent
        # loads. Its measured roofline is then the issue of USEFUL wave-VALU instructions (SQ_INSTS_VALU x SIMD
        # efficiency: the share of lanes doing node work) against the SIMDs' issue peak, one wave64 fp32 instruction per
        # 2 cycles per SIMD at the clock the PMC pass measured (GRBM_GUI_ACTIVE over the trace's launch time):
        # frac = issue_frac = valu_issue_frac x simd_efficiency.
        roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None}
        if traffic is None:
            bound_measured, limiter = None, "unmeasured: no PMC profile of this configuration and build (tools/profile.sh)"
        elif traffic < 0.05 * bytes_launch and valu is not None:
            bound_measured = "issue"
            limiter = (f"dependent-load latency and VALU issue: HBM traffic is {traffic / bytes_launch:.1%} of the "
                       "algorithmic bytes (the scene is L2/MALL-resident), VALU issues "
                       f"{valu:.0%} of the cycles, of which {simd_eff:.0%} of the lanes do node work")
            if insts and pmc.get("trace_avg_ms"):
                cycles = insts * 2 / (N_SIMD * valu)  # GRBM_GUI_ACTIVE / 8 XCDs per launch (PMC pass)
                clk_hz = cycles / (pmc["trace_avg_ms"] / 1e3)
                peak_i = N_SIMD * clk_hz / 2 / 1e9
                ach_i = insts * simd_eff / (k_avg_ms / 1e3) / 1e9
                roof = {"bound": "issue", "achieved": ach_i, "peak": peak_i, "unit": "G useful wave-VALU instr/s",
                        "frac": ach_i / peak_i, "clock_mhz_measured": clk_hz / 1e6}
        else:
            bound_measured = "hbm" if traffic / (k_avg_ms / 1e3) / 1e9 > 0.5 * HBM_PEAK_GBS else "mixed"
            limiter = "see DESIGN.md §5"
            hbm_gbs = traffic / (k_avg_ms / 1e3) / 1e9
            roof = {"bound": "hbm", "achieved": hbm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": hbm_gbs / HBM_PEAK_GBS}
        result = {
            "metric": METRIC,
            "value": rays_total / elapsed / 1e6,
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": data_note(args.scene, scene.n_triangles, is_standin),
            "config": {"workload": f"{args.scene} {W}x{H}, {args.spp} spp, {args.bounces} bounces, one fused "
                                   f"traversal+intersect+shade persistent launch per batch of {F} frames, "
                                   f"output {args.output}",
                       "scene": args.scene, "triangles": scene.n_triangles, "lights": len(scene.lights),
                       "width": W, "height": H, "bvh": args.bvh, "accel": args.accel, "kernel": args.kernel,
                       "rays_per_frame": rays_frame, "output": args.output, "parallelism": f"{B}-row blocks cyclic x{world} + RCCL gather"
                       if world > 1 else "single GPU", "frames_per_launch": F, "gather": gather_note,
                       # the native gather's communicator over the whole run: gathers, row-set exchanges (1 per layout)
                       "gather_comm": ng.info() if ng else None,
                       "gather_mode": gmode, "ranks": ranks_detail,
                       "launch": timed_launch, "accel_built": info["accel_built"], "accel_build_ms": info["build_ms"],
                       # its stages over every view: GPU PLOC, host treelet passes, host layout + 8-wide collapse
                       "accel_build_stages_ms": {k: info[k] for k in ("ploc_ms", "treelet_ms", "collapse_ms")},
                       "wide_depth": info["wide_depth"]},
            "frame_latency_ms": lat.item() if not args.no_latency else None,
            "frame_latency_detail": {"default_rule_ms": lat_default, "default_rule_mean_ms": sd["mean"],
                                     "refresh_frame_ms": sd["refresh_ms"], "walkthrough_ms": lat_walk,
                                     "walkthrough_mean_ms": sw["mean"], "walkthrough_refresh_ms": sw["refresh_ms"],
                                     "fixed_at_walk_ms": sf["median"], "walk_mid_camera": sw["mid_camera"],
                                     "walk_cameras": wcams, "walk_at_cameras_ms": wat, "fixed_at_cameras_ms": wfix,
                                     "walk_vs_fixed": (sum(a / b for a, b in zip(wat, wfix)) / len(wat)) if wat else None,
                                     "settle_frames": settle_frames, "settle_frames_walkthrough": settle_walk,
                                     "choice": seam_info,
                                     "rule": "frame_latency_ms = the default rule (rt_render with rt_frame's launch fields "
                                             "zeroed, render + sync per frame as the reference's loop): median HIP-event "
                                             "time of the 72 frames after rt_get_launch_info reports the rule settled (its "
                                             "measuring and trial frames excluded; every later frame's tile lists are "
                                             "built on the device from the frame before it, RT_BUILD_FEEDBACK -- a "
                                             "measuring refresh frame only without it: refresh_frame_ms), fixed reference "
                                             "camera; default_rule_mean_ms: their mean; walkthrough_ms: the median of 16 "
                                             "settled frames with the camera moved every frame (walkthrough_mean_ms: their "
                                             "mean); "
                                             "fixed_at_walk_ms: the fixed "
                                             "camera placed at the walkthrough's middle measured camera (walk_mid_camera); "
                                             "walk_vs_fixed: the mean over walk_cameras (the walk's measured quartiles) of "
                                             "the walk's frame at that camera (walk_at_cameras_ms) / "
                                             "the settled median of a fixed camera there (fixed_at_cameras_ms)"},
            "roofline": {**roof, "traffic": traffic,
                         "kernel_ms": k_avg_ms, "alg_bytes_per_launch": bytes_launch, "frames_per_launch": F,
                         # the algorithmic bytes per second and against the HBM peak: not a bound (the
                         # records come from L1/L2/MALL; it exceeds 1 on scenes with more bytes per ray)
                         "alg_byte_achieved": alg_gbs, "alg_byte_frac": alg_gbs / HBM_PEAK_GBS,
                         "alg_byte_achieved_steady": bytes_launch / F * K / elapsed / 1e9, "streams": n_streams,
                         # L1 -> L2 read bytes per second (PMC TCP_TCC_READ_REQ x 64 B): the cache side that serves them
                         "l2_read_gbs": (pmc["l2_read_bytes_per_launch"] / (k_avg_ms / 1e3) / 1e9
                                         if pmc.get("l2_read_bytes_per_launch") else None),
                         # the same launch priced with SURVEY §8d's formula (reference record sizes): comparable
                         # with BASELINE.md's 3.45 / 6.3 Grays/s roofline-equivalent rates
                         "survey_bytes_per_launch": survey_launch,
                         "survey_achieved": survey_launch / (k_avg_ms / 1e3) / 1e9,
                         "survey_frac": survey_launch / (k_avg_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                         # (read first: neither byte fraction is a bound, both may exceed 1)
                         "byte_fracs_are_bounds": False,
                         "byte_fracs_note": "alg_byte_frac and survey_frac price every record a ray reads as an HBM "
                                            "byte; the records are L1/L2/MALL hits (hbm_frac_measured is the real HBM "
                                            "share), so values above 1 are expected and bound nothing; frac is the "
                                            "binding (issue) roofline",
                         "simd_efficiency": simd_eff,
                         # VALU instructions per walk step (PMC SQ_INSTS_VALU of the launch / its wave-level node steps)
                         "valu_per_wave_step": (pmc["sq_insts_valu_per_launch"] / max(1, stc["wave_steps"])
                                                if pmc.get("sq_insts_valu_per_launch") else None),
                         # the launch's work per ray (RT_FLAG_COUNTERS): wide-node visits, leaf slots and
                         # triangle tests of the closest (primary + reflection) and the shadow walks
                         "per_ray": {"closest_nodes": stc["ch_inner"] / max(1, stc["primary"] + stc["reflection"]),
                                     "closest_leaves": stc["ch_leaf"] / max(1, stc["primary"] + stc["reflection"]),
                                     "closest_tris": stc["ch_tri"] / max(1, stc["primary"] + stc["reflection"]),
                                     "shadow_nodes": stc["sh_inner"] / max(1, stc["shadow"]),
                                     "shadow_leaves": stc["sh_leaf"] / max(1, stc["shadow"]),
                                     "shadow_tris": stc["sh_tri"] / max(1, stc["shadow"]),
                                     "wave_steps_per_frame": stc["wave_steps"] / F,
                                     "shadow_wave_step_frac": stc["shadow_wave_steps"] / max(1, stc["wave_steps"]),
                                     # wave steps by active lanes 1-16 / 17-32 / 33-48 / 49-64 (fractions)
                                     "wave_steps_by_active_lanes": [stc[k] / max(1, stc["wave_steps"]) for k in (
                                         "steps_lanes_16", "steps_lanes_32", "steps_lanes_48", "steps_lanes_64")],
                                     "strict_fallbacks": stc["fallbacks"],
                                     # the same wave steps by walk kind x bounce level (0, 1, 2, 3+) x active lanes
                                     # (1-16, 17-32, 33-48, 49-64), each a fraction of all the launch's wave steps
                                     "wave_steps_by_kind_level": {
                                         kind: [[round(v / max(1, stc["wave_steps"]), 5) for v in lv]
                                                for lv in stc["steps_hist"][k]]
                                         for k, kind in enumerate(("closest", "shadow"))}},
                         # measured by rocprofv3 PMC passes of this command (profiles/pmc_traffic.json)
                         "hbm_frac_measured": (traffic / (k_avg_ms / 1e3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
                         "traffic_over_pixels": (traffic / (F * W * n_r * (4 if bgra else 12))) if traffic else None,
                         "valu_issue_frac": valu,
                         # the measured bound: the share of the SIMDs' peak lane-issue that does useful node work
                         "issue_frac": (valu * simd_eff) if valu is not None else None,
                         "wave_wait_frac": pmc.get("wave_wait_frac"),
                         "l2_hit_rate": pmc.get("l2_hit_rate"),
                         "fetch_bytes_per_launch": pmc.get("fetch_bytes_per_launch"),
                         "write_bytes_per_launch": pmc.get("write_bytes_per_launch"),
                         "l2_read_bytes_per_launch": pmc.get("l2_read_bytes_per_launch"),
                         "pmc_key": key, "pmc_source": pmc.get("source"), "pmc_stale": pmc_stale,
                         "pmc_trace_avg_ms": pmc.get("trace_avg_ms"),
                         # what binds the kernel, measured (the contract's `bound` names the priced roofline)
                         "bound_measured": bound_measured, "limiter": limiter,
                         "note": "bound / achieved / peak / frac: the roofline that binds, from this build's PMC "
                                 "passes (profiles/pmc_traffic.json): with HBM traffic under 5 % of the algorithmic bytes, "
                                 "'issue' = useful wave-VALU instructions (SQ_INSTS_VALU x simd_efficiency) per second "
                                 "against the SIMDs' issue peak at the measured clock, so frac = issue_frac; else HBM "
                                 "traffic against 8 TB/s. alg_byte_*: algorithmic bytes (DESIGN.md §5) per HIP-event "
                                 "launch time, served by L1/L2/MALL (not a bound). hbm_frac_measured = (2 x FETCH_SIZE + "
                                 "WRITE_SIZE) / time / peak"},
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or min(16, usable_cpus())
            def gpu_rays_for_rows(stride):
                nr = (H + stride - 1) // stride
                rr = device.Renderer(local, stream=stream)
                rr.upload(scene, accel=args.accel, ploc_radius=args.ploc_radius)
                tmp = torch.empty((nr, W, 3), dtype=torch.float32, device="cuda")
                rr.render(cam, W, H, rows=(0, stride, nr), bounces=args.bounces, kernel=args.kernel, rgb=tmp)
                n = rr.stats()["rays"]
                rr.close()
                return n
            try:
                result["cpu_baseline"] = cpu_baseline(files, W, H, gpu_rays_for_rows, args, threads)
                allc = min(256, usable_cpus())  # nproc: the CPUs this process may use (affinity, cgroup quota)
                result["cpu_baseline"]["nproc"] = allc
                if allc != threads and not args.no_all_cpus:  # also at nproc threads
                    a1 = argparse.Namespace(**vars(args))
                    a1.no_single_thread = True
                    a1.cpu_row_stride = 0
                    r = cpu_baseline(files, W, H, gpu_rays_for_rows, a1, allc)
                    result["cpu_baseline"]["all_cpus"] = {k: r[k] for k in ("value", "unit", "cores", "sample")}
            except Exception as e:  # reported, never silently replaced
                result["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(result), flush=True)
    if ng:
        ng.close()
    for rr_ in rends:
        rr_.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
