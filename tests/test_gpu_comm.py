"""The frame gathers of the native boundary on the GPU: rt_comm_* (RCCL send / recv over
xGMI) and rt_gather (xGMI peer copies; several contexts on one device here).

RCCL takes one rank per device, so on a one-GPU box the RCCL path runs with ONE rank — through both
constructors (rt_comm_init over the contexts of one process, rt_comm_init_rank with an id as a multi-process
job does) — while the row layouts of N ranks (cyclic rows, 8-row blocks, rotated residues in frame batches)
are exercised through rt_gather, which shares the descriptor check and the un-interleaving kernel with it
(rt_hip.hip: check_parts, k_unshuffle_frames). Bar: the gathered frames equal one full render bit for bit.
"""
import os
import subprocess

import numpy as np
import pytest
import torch

from prt import host
from prt.dist import rank_rows

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H = 200, 113


@pytest.fixture(scope="module")
def dev():
    from prt import device
    assert device.device_count() > 0
    return device


@pytest.fixture(scope="module")
def scene():
    return host.Scene.named("car_boxed").build_bvh(3)


def cams(n):  # distinct frames: the camera moved a little per frame
    out = []
    for f in range(n):
        c = host.camera(W, H)
        c.pos.x += 0.05 * f
        out.append(c)
    return out


def full_frames(dev, scene, n, kind):
    r = dev.Renderer(0)
    r.upload(scene)
    t = torch.empty((n, H, W) if kind == "bgra" else (n, H, W, 3), dtype=torch.int32 if kind == "bgra" else torch.float32,
                    device="cuda")
    r.render_frames(cams(n), W, H, **{kind: t})
    r.sync()
    r.close()
    return t.cpu()


def rank_render(dev, scene, r, rows, n, kind, shift=0):
    t = torch.empty((n, rows[2], W) if kind == "bgra" else (n, rows[2], W, 3),
                    dtype=torch.int32 if kind == "bgra" else torch.float32, device="cuda")
    r.render_frames(cams(n), W, H, rows=tuple(rows) + ((shift,) if shift else ()), **{kind: t})
    return t


@pytest.mark.parametrize("kind", ["rgb", "bgra"])
@pytest.mark.parametrize("frames", [1, 3])
@pytest.mark.parametrize("ctor", ["all", "rank"])
def test_rccl_gather_one_rank(dev, scene, kind, frames, ctor):
    ref = full_frames(dev, scene, frames, kind)
    r = dev.Renderer(0)
    r.upload(scene)
    comm = dev.Comm([r]) if ctor == "all" else dev.Comm([r], nranks=1, rank=0, uid=dev.comm_id())
    keep = rank_render(dev, scene, r, (0, 1, H), frames, kind)  # (the render's output lives until the gather has run)
    out = torch.empty_like(ref, device="cuda")
    comm.gather(0, out)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu().view(torch.int32), ref.view(torch.int32))
    if frames == 1:  # into the context's own buffer: download_bmp reads the gathered frame
        comm.gather(0)
        want = host.bmp_from_bgra(ref[0].numpy()) if kind == "bgra" else host.bmp_encode(ref[0].numpy())
        assert r.download_bmp() == want
    comm.close()
    r.close()
    del keep


@pytest.mark.parametrize("kind", ["rgb", "bgra"])
@pytest.mark.parametrize("n,block,shift", [(2, 1, 0), (3, 8, 0), (4, 8, 8), (3, 8, 8)])
def test_gather_of_rank_row_sets_batches(dev, scene, kind, n, block, shift):
    """n contexts render their rank row sets of a 4-frame batch (single rows, 8-row blocks, and 8-row blocks
    whose residue rotates frame by frame, rt_frame.frame_shift); rt_gather un-interleaves them into the full
    frames on the root"""
    frames = 4
    ref = full_frames(dev, scene, frames, kind)
    rs = [dev.Renderer(0) for _ in range(n)]
    keep = []
    for g, r in enumerate(rs):
        r.upload(scene)
        rows = rank_rows(H, g, n, block)
        if shift:  # every rank renders the largest rank's row count (rows past the image are skipped)
            rows = (rows[0], rows[1], max(rank_rows(H, q, n, block)[2] for q in range(n)), rows[3])
        keep.append(rank_render(dev, scene, r, rows, frames, kind, shift))
    out = torch.empty_like(ref, device="cuda")
    dev.gather(rs, root=n - 1, out=out)
    rs[n - 1].sync()
    assert torch.equal(out.cpu().view(torch.int32), ref.view(torch.int32))
    for r in rs:
        r.close()


def test_gather_refuses_mixed_or_incomplete_row_sets(dev, scene):
    a, b = dev.Renderer(0), dev.Renderer(0)
    for r in (a, b):
        r.upload(scene)
    rank_render(dev, scene, a, rank_rows(H, 0, 2, 8), 1, "rgb")
    rank_render(dev, scene, b, rank_rows(H, 1, 2, 8), 1, "bgra")
    with pytest.raises(dev.RtError):  # rgb on one context, bgra on the other
        dev.gather([a, b], root=0)
    rank_render(dev, scene, b, rank_rows(H, 1, 2, 8), 2, "rgb")
    with pytest.raises(dev.RtError):  # frame counts differ
        dev.gather([a, b], root=0)
    rank_render(dev, scene, b, rank_rows(H, 0, 2, 8), 1, "rgb")
    with pytest.raises(dev.RtError):  # both render rank 0's rows
        dev.gather([a, b], root=0)
    a.close()
    b.close()


def test_cli_rccl_gather_writes_the_reference_bmp(tmp_path):
    """the CLI's frame gather through RCCL (--gather rccl; one GPU: a one-rank communicator)"""
    from tests.scenes import scene_paths
    exe = os.path.join(ROOT, "parallel-ray-tracer_amd", "bin", "raytracer")
    assets = os.path.dirname(os.path.dirname(scene_paths("car_boxed")[0]))
    ref = np.load(os.path.join(ROOT, "tests", "golden", "car_boxed_160x90_strict.npz"))
    out = tmp_path / "g.bmp"
    r = subprocess.run([exe, "4", "--scene", "car_boxed", "--assets", assets, "--width", "160", "--height", "90",
                        "--gather", "rccl", "--out", str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Frame gather: RCCL" in r.stdout
    assert out.read_bytes() == host.bmp_encode(ref["rgb"])


@pytest.mark.parametrize("kind", ["rgb", "bgra"])
def test_rccl_rank_comm_exchanges_once_per_layout(dev, scene, kind):
    """rt_comm_init_rank's gather (the multi-process path, one rank here): the row-set descriptors are exchanged
    once per layout -- 4 gathers of an unchanged layout, from two contexts sharing ONE communicator
    (rt_comm_gather_from, as bench.py alternates them), exchange once -- and a new layout (a different frame count)
    exchanges again; the root checks every layout's first gather pixel by pixel; every gather equals one GPU's frames"""
    frames = 3
    ref = full_frames(dev, scene, frames, kind)
    rs = [dev.Renderer(0), dev.Renderer(0)]
    for r in rs:
        r.upload(scene)
    comm = dev.Comm([rs[0]], nranks=1, rank=0, uid=dev.comm_id())
    for g in range(4):
        r = rs[g % 2]
        keep = rank_render(dev, scene, r, (0, 1, H), frames, kind)
        out = torch.zeros_like(ref, device="cuda")
        torch.cuda.synchronize()
        comm.gather(0, out, src=r)
        r.sync()
        assert torch.equal(out.cpu().view(torch.int32), ref.view(torch.int32)), g
    info = comm.info()
    assert info["gathers"] == 4 and info["exchanges"] == 1 and info["checked"] == 1, info
    keep = rank_render(dev, scene, rs[1], (0, 1, H), 1, kind)  # a new layout: one frame
    out = torch.zeros_like(ref[:1], device="cuda")
    torch.cuda.synchronize()
    comm.gather(0, out, src=rs[1])
    rs[1].sync()
    assert torch.equal(out.cpu().view(torch.int32), ref[:1].view(torch.int32))
    info = comm.info()
    assert info["gathers"] == 5 and info["exchanges"] == 2 and info["checked"] == 2, info
    comm.close()
    for r in rs:
        r.close()


def test_rccl_rank_comm_refuses_a_partial_layout(dev, scene):
    """a layout whose row sets do not cover the frame (here: one rank rendering only half the rows) fails the
    exchange's partition check instead of gathering a frame with holes"""
    r = dev.Renderer(0)
    r.upload(scene)
    comm = dev.Comm([r], nranks=1, rank=0, uid=dev.comm_id())
    keep = rank_render(dev, scene, r, (0, 2, (H + 1) // 2), 1, "bgra")
    with pytest.raises(dev.RtError):
        comm.gather(0, torch.zeros((1, H, W), dtype=torch.int32, device="cuda"), src=r)
    comm.close()
    r.close()


def test_rccl_rank_comm_deadline_does_not_cover_the_render(dev, scene):
    """the deadline of the collective waits starts when the render before the gather has completed, so a
    render much longer than the communicator's timeout (here car_boxed 1920x1080 at 16 spp, ~15 ms, under a 2 ms
    timeout) gathers, waits (rt_comm_wait) and syncs (rt_sync, which settles the communicator first) without an abort;
    the gathered frame equals the render"""
    Wl, Hl = 1920, 1080
    r = dev.Renderer(0)
    r.upload(scene)
    comm = dev.Comm([r], nranks=1, rank=0, uid=dev.comm_id())
    comm.set_timeout(0.002)
    px = torch.zeros((1, Hl, Wl), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    for g in range(3):  # the first gather exchanges and checks coverage (host waits); the others reuse the layout
        r.render_frames([host.camera(Wl, Hl)], Wl, Hl, spp=16, bgra=px)
        out = torch.zeros((1, Hl, Wl), dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        comm.gather(0, out, src=r)
        if g == 1:
            comm.wait()
        ms = r.sync()
        assert ms > 0.002 * 1e3, ms  # (the render did outlast the timeout)
        assert torch.equal(out, px), g
    info = comm.info()
    assert info["gathers"] == 3 and info["exchanges"] == 1 and info["checked"] == 1, info
    comm.close()
    r.close()
