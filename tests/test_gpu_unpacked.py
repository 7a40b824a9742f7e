"""The k_persist builds that only scenes past the packed builds' field bounds run, pinned on scenes of test size.

The packed builds store a wide-stack entry in 5 bytes (a 24-bit child base: at most 2^24 wide nodes per view) and a
packed triangle-test job with a 26-bit triangle index (fewer than 2^26 triangles). Larger scenes run the unpacked
builds (rt_hip.hip persist_kernel): PERSIST4 with two-word stack entries, and the 3-wave spp = 1 build without packed
triangle tests. No BASELINE scene comes near those bounds, so rt_opts.flags RT_FLAG_UNPACKED_STACK /
RT_FLAG_UNPACKED_TRIS select them for any scene; rt_launch_info.build reports the instantiation that ran.

Bar: bit-exact against the reference's fixtures (cpu/src/raytracer.c:101-177 through oracle/_ref/rt_ref_strict:
hit indices, t, every colour bit), the 1080p frame's md5 and ray counts; frame batches equal to the packed builds'.
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
_SCENES = {}


def scene(name):
    if name not in _SCENES:
        _SCENES[name] = host.Scene.named(name).build_bvh(3)
    return _SCENES[name]


def same_bits(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.int32), np.asarray(b, np.float32).view(np.int32))


def flag_sets():
    from prt import device
    return {"stack": device.FLAG_UNPACKED_STACK, "tris": device.FLAG_UNPACKED_TRIS,
            "both": device.FLAG_UNPACKED_STACK | device.FLAG_UNPACKED_TRIS}


def render(name, W, H, kernel, flags, counters=False):
    import torch
    from prt import device
    r = device.Renderer(0, counters=counters, flags=flags)
    r.upload(scene(name))
    hit = torch.empty((H, W), dtype=torch.int32, device="cuda")
    t = torch.empty((H, W), dtype=torch.float32, device="cuda")
    rgb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    r.render(host.camera(W, H), W, H, kernel=kernel, rgb=rgb, hit=hit, t=t)
    r.sync()
    out = {"rgb": rgb.cpu().numpy(), "hit": hit.cpu().numpy(), "t": t.cpu().numpy(), "stats": r.stats(),
           "launch": r.launch_info()}
    r.close()
    return out


def expected_bits(kernel, fl):
    """the RT_BUILD_* bits persist_kernel must report for a forced variant under unpacked flags `fl` (lds_paths aside:
    the unpacked PERSIST4 keeps its path levels in LDS only where its two-word stack entries leave room for 4 workgroups
    per CU, and otherwise in a global slab)"""
    if kernel == "persist":  # the 3-wave spp = 1 build: packed triangle tests unless they are refused
        return {"packed_tris"} if fl == "stack" else set()
    return {"waves4"}  # PERSIST4 / SHPOOL / SHDEFER: the unpacked PERSIST4 (the pools need both packings)


@pytest.mark.parametrize("fl", ["stack", "tris", "both"])
@pytest.mark.parametrize("kernel", ["persist", "persist4", "shpool", "shdefer"])
@pytest.mark.parametrize("name", ["car_boxed", "car_only"])
@pytest.mark.parametrize("W,H", [(64, 36), (160, 90)])
def test_unpacked_builds_vs_reference_fixture(name, W, H, kernel, fl):
    out = render(name, W, H, kernel, flag_sets()[fl])
    assert set(out["launch"]["build_bits"]) - {"lds_paths"} == expected_bits(kernel, fl), out["launch"]
    ref = np.load(os.path.join(GOLD, f"{name}_{W}x{H}_strict.npz"))
    np.testing.assert_array_equal(out["hit"], ref["hit"])
    assert same_bits(out["t"], ref["t"])
    assert same_bits(out["rgb"], ref["rgb"]), np.abs(out["rgb"] - ref["rgb"]).max()


@pytest.mark.parametrize("kernel", ["persist", "persist4", "fast"])
def test_unpacked_builds_1080p_vs_reference(kernel):
    """car_boxed 1920x1080 (the reference asset, 13.2 M rays) through the unpacked builds: every 97th pixel, the full
    frame's md5 and the ray counts of the reference itself (rt_ref_count); "fast" = the default single-frame rule
    (its measuring frame) with neither packing"""
    out = render("car_boxed", 1920, 1080, kernel, flag_sets()["both"], counters=True)
    assert not {"packed_stack", "packed_tris"} & set(out["launch"]["build_bits"]), out["launch"]
    ref = np.load(os.path.join(GOLD, "car_boxed_1080p_strict_sample.npz"))
    idx = ref["idx"]
    np.testing.assert_array_equal(out["hit"].reshape(-1)[idx], ref["hit"])
    assert same_bits(out["t"].reshape(-1)[idx], ref["t"])
    assert same_bits(out["rgb"].reshape(-1, 3)[idx], ref["rgb"])
    md5 = hashlib.md5(out["hit"].astype(np.int32).tobytes() + out["t"].tobytes() + out["rgb"].tobytes()).hexdigest()
    assert md5 == G["frames"]["car_boxed_1920x1080_strict"]["md5"]
    st, rays = out["stats"], G["rays"]["car_boxed_1920x1080"]
    assert st["primary"] + st["reflection"] == rays["closest"]
    assert st["shadow"] == rays["shadow"]
    assert st["stack_overflows"] == 0


@pytest.mark.parametrize("variant", ["persist4", "shdefer", "default"])
def test_unpacked_frame_batch_equals_packed(variant):
    """dragon 1920x1080 (the bench scene), a 3-frame batch in BGRA8 through the unpacked PERSIST4 (the pool variants and
    the default rule fall back to it without packed stack entries): equal to the packed production build's frames, and
    frame 0 to the reference's quantised pixels at every sampled pixel"""
    import torch
    from prt import device
    W, H, n = 1920, 1080, 3
    cams = []
    for i in range(n):
        c = host.camera(W, H)
        c.pos.x += i * 0.02
        c.ul.x += i * 0.02
        cams.append(c)
    frames = {}
    for fl in (0, flag_sets()["both"]):
        r = device.Renderer(0, flags=fl)
        r.upload(scene("dragon"))
        px = torch.zeros((n, H, W), dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        for _ in range(8 if variant == "default" else 1):
            r.render_frames(cams, W, H, bgra=px, variant=variant)
            r.sync()
            if variant != "default" or r.launch_info()["settled"]:
                break
        bits = set(r.launch_info()["build_bits"])
        if fl:
            assert not {"packed_stack", "packed_tris"} & bits and "waves4" in bits, r.launch_info()
        frames[fl] = px.cpu().numpy().view(np.uint32)
        r.close()
    np.testing.assert_array_equal(frames[flag_sets()["both"]], frames[0])
    ref = np.load(os.path.join(GOLD, "dragon_1080p_strict_sample.npz"))
    q = (np.asarray(ref["rgb"], np.float32) * np.float32(255.0)).astype(np.uint8).astype(np.uint32)
    want = q[..., 2] | (q[..., 1] << 8) | (q[..., 0] << 16) | np.uint32(255 << 24)
    np.testing.assert_array_equal(frames[0][0].reshape(-1)[ref["idx"]], want)
