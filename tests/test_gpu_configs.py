"""Every BASELINE.json configuration at the size it names, on the HIP path, against the reference itself
(fixtures from tests/golden/make_golden.py: oracle/_ref/rt_ref_strict = cpu/src/*.c, rt_ref_count's rays).

  configs[0]  dragon 640x360 (cpu/src/main.c's own WIDTH x HEIGHT)           -> dragon_360p_strict_sample.npz
  configs[1]  dragon 1920x1080 (the bench workload)                          -> dragon_1080p_strict_sample.npz
  configs[2]  sportscar 1920x1080                                            -> sportscar_1080p_strict_sample.npz
  configs[3]  two_cars 3840x2160                                             -> two_cars_2160p_strict_sample.npz
  configs[4]  car_boxed 3840x2160 at 64 spp                                  -> test_gpu_parity.py (64 spp)

Two seams per configuration:
  * rt_render with rgb / hit / t (the drop-in's render_frame, one frame per call): every sampled pixel, the
    full frame's md5 and the ray counts equal the reference's;
  * the instantiation bench.py times: rt_render_frames (one persistent launch of several frames, the 4-wave
    batch kernel's spp = 1 build with the LDS path buffer) writing BGRA8 only, on bench.py's camera path
    (frame i moved by i * 0.02 along x; frame 0 IS the reference camera). Frame 0 equals vec_to_bgra of the
    reference's frame at every sampled pixel and of the md5-checked rgb frame everywhere; frames 1.. equal
    rt_render of their own cameras bit for bit; and the same batch dealt over 8 ranks' rotated 8-row blocks
    (bench.py's N = 8 layout) renders every pixel of every frame exactly once, with the same bits.
Bar: bit-exact (hit indices, t, every colour bit, every BGRA8 byte), ray counts equal.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from prt import host

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
G = json.load(open(os.path.join(GOLD, "golden.json")))
ORBIT = 0.02  # bench.py --orbit default
_SCENES = {}

# (+ dragon871k: the stand-in at the real Stanford dragon's triangle count, 868,352 + the room, that assets/dragon's
# missing mesh has, .MISSING_LARGE_BLOBS:1 -> dragon871k_1080p_strict_sample.npz)
CONFIGS = [("dragon", 640, 360, "360p"), ("dragon", 1920, 1080, "1080p"), ("sportscar", 1920, 1080, "1080p"),
           ("two_cars", 3840, 2160, "2160p"), ("dragon871k", 1920, 1080, "1080p")]


def scene(name):
    if name not in _SCENES:
        _SCENES[name] = host.Scene.named(name).build_bvh(3)
    return _SCENES[name]


def cam_path(W, H, n):
    """bench.py's camera path: frame i = the reference camera moved by i * ORBIT along x"""
    out = []
    for i in range(n):
        c = host.camera(W, H)
        c.pos.x += i * ORBIT
        c.ul.x += i * ORBIT
        out.append(c)
    return out


def quantise(rgb):
    """vec_to_bgra (cpu/src/bmp_writer.c:88-95) -> packed uint32 B | G << 8 | R << 16 | 255 << 24"""
    q = (np.asarray(rgb, np.float32) * np.float32(255.0)).astype(np.uint8).astype(np.uint32)
    return q[..., 2] | (q[..., 1] << 8) | (q[..., 0] << 16) | np.uint32(255 << 24)


def same_bits(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.int32), np.asarray(b, np.float32).view(np.int32))


def single(name, W, H, kernel="fast", cam=None, counters=False, bgra=False):
    import torch
    from prt import device
    r = device.Renderer(0, counters=counters)
    r.upload(scene(name))
    out = {}
    if bgra:
        px = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        r.render(cam or host.camera(W, H), W, H, kernel=kernel, bgra=px)
        r.sync()  # the context's own stream: finish before torch reads the outputs
        out["bgra"] = px.cpu().numpy().view(np.uint32)
    else:
        hit = torch.empty((H, W), dtype=torch.int32, device="cuda")
        t = torch.empty((H, W), dtype=torch.float32, device="cuda")
        rgb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        r.render(cam or host.camera(W, H), W, H, kernel=kernel, rgb=rgb, hit=hit, t=t)
        r.sync()
        out.update(rgb=rgb.cpu().numpy(), hit=hit.cpu().numpy(), t=t.cpu().numpy())
    out["stats"] = r.stats()
    r.close()
    return out


_FRAMES = {}


def reference_frame(name, W, H):
    """the drop-in seam's frame, checked against the reference once per configuration (cached for the batch
    tests)"""
    key = (name, W, H)
    if key not in _FRAMES:
        out = single(name, W, H, counters=True)
        _FRAMES[key] = out
    return _FRAMES[key]


@pytest.mark.parametrize("kernel", ["fast", "persist4", "strict"])
@pytest.mark.parametrize("name,W,H,tag", CONFIGS)
def test_config_single_frame_vs_reference(name, W, H, tag, kernel):
    out = reference_frame(name, W, H) if kernel == "fast" else single(name, W, H, kernel, counters=True)
    ref = np.load(os.path.join(GOLD, f"{name}_{tag}_strict_sample.npz"))
    idx = ref["idx"]
    np.testing.assert_array_equal(out["hit"].reshape(-1)[idx], ref["hit"])
    assert same_bits(out["t"].reshape(-1)[idx], ref["t"])
    assert same_bits(out["rgb"].reshape(-1, 3)[idx], ref["rgb"])
    md5 = hashlib.md5(out["hit"].astype(np.int32).tobytes() + out["t"].tobytes() + out["rgb"].tobytes())
    assert md5.hexdigest() == G["standin"][name][f"{W}x{H}_md5"]
    st, rays = out["stats"], G["rays"][f"{name}_{W}x{H}"]
    assert st["primary"] + st["reflection"] == rays["closest"]
    assert st["shadow"] == rays["shadow"]
    assert st["stack_overflows"] == 0


@pytest.mark.parametrize("variant", ["default", "persist4", "shpool", "shdefer"])
@pytest.mark.parametrize("name,W,H,tag", CONFIGS)
def test_config_bench_batch_vs_reference(name, W, H, tag, variant):
    """bench.py's instantiation (4 frames of its camera path in one rt_render_frames launch, BGRA8 only) against
    the reference and against single-frame renders. The default rule measures PERSIST4 and the shadow pool on the
    first launches of a shape and keeps the faster, so the bench runs either: both are pinned here, and the default
    rule's own launches (its trials, then its choice)."""
    import torch
    from prt import device
    n = 4
    cams = cam_path(W, H, n)
    r = device.Renderer(0)
    r.upload(scene(name))
    px = torch.zeros((n, H, W), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()  # torch's fill before the context's stream writes
    for _ in range(8 if variant == "default" else 1):  # (default: its trial launches, then the choice)
        r.render_frames(cams, W, H, bgra=px, variant=variant)
        r.sync()
        if variant == "default" and r.launch_info()["settled"]:
            break
    if variant == "default":
        assert r.launch_info()["settled"] and r.launch_info()["variant"] in ("persist4", "shpool", "shdefer"), r.launch_info()
    frames = px.cpu().numpy().view(np.uint32)
    r.close()
    ref = np.load(os.path.join(GOLD, f"{name}_{tag}_strict_sample.npz"))
    np.testing.assert_array_equal(frames[0].reshape(-1)[ref["idx"]], quantise(ref["rgb"]))
    np.testing.assert_array_equal(frames[0], quantise(reference_frame(name, W, H)["rgb"]))
    for i in range(1, n):
        np.testing.assert_array_equal(frames[i], single(name, W, H, cam=cams[i], bgra=True)["bgra"], err_msg=str(i))
    assert not np.array_equal(frames[0], frames[1])  # the path's frames differ
    if variant != "default":
        return
    # the same batch over bench.py's N = 8 layout: 8-row blocks, residues rotated by frame, compact rows
    from prt.dist import padded_rows
    N, B = 8, 8
    nmax = padded_rows(H, N, B)
    full = np.zeros((n, H, W), np.uint32)
    seen = np.zeros((n, H), np.int32)
    for q in range(N):
        rr = device.Renderer(0)
        rr.upload(scene(name))
        part = torch.zeros((n, nmax, W), dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        rr.render_frames(cams, W, H, rows=(q * B, N * B, nmax, B, B), bgra=part)
        rr.sync()
        p = part.cpu().numpy().view(np.uint32)
        rr.close()
        for f in range(n):
            res = (q + f) % N
            for k in range(nmax):
                y = res * B + (k // B) * N * B + k % B
                if y < H:
                    full[f, y] = p[f, k]
                    seen[f, y] += 1
    assert (seen == 1).all()
    np.testing.assert_array_equal(full, frames)
