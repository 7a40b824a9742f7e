"""k_relay (RT_VARIANT_RELAY, rt_relay.hpp): one workgroup of 1 + lights waves per 8x8 tile, wave 0 walking the
closest-hit chains and wave j level i's shadow rays toward light j - 1 while wave 0 walks level i + 1 (LDS
hand-off). The reference's recursion (cpu/src/raytracer.c:101-177) split over waves must keep every bit:
fixtures of the reference itself (1, 2 and 4 lights), the 1080p frames' md5s and ray counts, per-bounce hits,
row subsets, quantised output, and the hybrid launch with the relay kernel on the hot tiles."""
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


def render(name, W, H, kernel, rows=None, counters=False, bounces=4, spp=1, **kw):
    import torch
    from prt import device
    r = device.Renderer(0, counters=counters)
    r.upload(scene(name))
    nr = rows[2] if rows else H
    hit = torch.full((nr, W), -7, dtype=torch.int32, device="cuda")
    t = torch.zeros((nr, W), dtype=torch.float32, device="cuda")
    rgb = torch.zeros((nr, W, 3), dtype=torch.float32, device="cuda")
    bh = torch.full((nr, W, bounces), -9, dtype=torch.int32, device="cuda")
    bg = torch.zeros((nr, W), dtype=torch.int32, device="cuda")
    r.render(host.camera(W, H), W, H, rows=rows, kernel=kernel, rgb=rgb, hit=hit, t=t, bounce_hit=bh, bgra=bg,
             bounces=bounces, spp=spp, **kw)
    st = r.stats()
    out = {"rgb": rgb.cpu().numpy(), "hit": hit.cpu().numpy(), "t": t.cpu().numpy(), "bh": bh.cpu().numpy(),
           "bgra": bg.cpu().numpy(), "stats": st}
    r.close()
    return out


def same_bits(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.int32), np.asarray(b, np.float32).view(np.int32))


def md5(out):
    return hashlib.md5(out["hit"].astype(np.int32).tobytes() + out["t"].tobytes() + out["rgb"].tobytes()).hexdigest()


@pytest.mark.parametrize("name,W,H", [("car_boxed", 64, 36), ("car_boxed", 160, 90), ("car_only", 160, 90),
                                      ("dragon", 96, 54), ("sportscar", 96, 54), ("two_cars", 96, 54)])
def test_relay_vs_reference_fixture(name, W, H):
    """1 (car scenes), 2 (dragon, two_cars) and 4 (sportscar) lights: 2 to 5 waves per workgroup"""
    out = render(name, W, H, "relay")
    ref = np.load(os.path.join(GOLD, f"{name}_{W}x{H}_strict.npz"))
    np.testing.assert_array_equal(out["hit"], ref["hit"])
    assert same_bits(out["t"], ref["t"])
    assert same_bits(out["rgb"], ref["rgb"]), np.abs(out["rgb"] - ref["rgb"]).max()


@pytest.mark.parametrize("name", ["car_boxed", "dragon", "sportscar"])
def test_relay_1080p_frame_and_ray_counts(name):
    """the whole 1080p frame's md5 and the ray counts of the reference (rt_ref_count)"""
    out = render(name, 1920, 1080, "relay", counters=True)
    want = G["frames"]["car_boxed_1920x1080_strict"]["md5"] if name == "car_boxed" else \
        G["standin"][name]["1920x1080_md5"]
    assert md5(out) == want
    st, rays = out["stats"], G["rays"][f"{name}_1920x1080"]
    assert st["primary"] + st["reflection"] == rays["closest"]
    assert st["shadow"] == rays["shadow"]
    assert st["pixels"] == 1920 * 1080 and st["stack_overflows"] == 0


@pytest.mark.parametrize("name", ["dragon", "sportscar"])
def test_relay_equals_persistent_kernel_everywhere(name):
    """per-bounce hits (bounces 1, 2, 4, 6), the quantised pixels and every counter equal k_persist's; a row-block
    subset equals the full frame's rows; a request the relay cannot serve (4 spp) takes k_persist"""
    W, H = 200, 120
    for b in (1, 2, 4, 6):
        a = render(name, W, H, "persist", counters=True, bounces=b)
        c = render(name, W, H, "relay", counters=True, bounces=b)
        for k in ("hit", "bh", "bgra"):
            np.testing.assert_array_equal(a[k], c[k], err_msg=f"{k} b{b}")
        assert same_bits(a["rgb"], c["rgb"]) and same_bits(a["t"], c["t"]), b
        for k in ("primary", "reflection", "shadow", "shadow_skipped", "hits", "pixels", "fallbacks"):
            assert a["stats"][k] == c["stats"][k], (b, k)
    full = render(name, W, H, "relay")
    part = render(name, W, H, "relay", rows=(8, 24, 40, 8))
    rows = [8 + (k // 8) * 24 + k % 8 for k in range(40)]
    assert same_bits(part["rgb"], full["rgb"][rows])
    np.testing.assert_array_equal(part["hit"], full["hit"][rows])
    a = render(name, 96, 54, "persist", spp=4)
    c = render(name, 96, 54, "relay", spp=4)
    assert same_bits(a["rgb"], c["rgb"])


@pytest.mark.parametrize("name", ["dragon", "car_boxed", "sportscar"])
def test_hybrid_with_relay_hot_tiles(name):
    """RT_VARIANT_HYBRID with rt_frame.hot_kernel = relay: the measuring frame, the in-flight frame and the hybrid
    frames (hot tiles through k_relay on the second stream, the rest through k_persist) equal k_persist's frame, with
    the same ray counts, for thresholds that make every / some / no tile hot"""
    import torch
    from prt import device
    W, H = 200, 120
    ref = render(name, W, H, "persist", counters=True)
    for pct in (1, 60, 100):
        r = device.Renderer(0, counters=True)
        r.upload(scene(name))
        for group in ((0, 1), (2,), (3,), (4,)):
            outs = []
            for _ in group:
                hit = torch.full((H, W), -7, dtype=torch.int32, device="cuda")
                rgb = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
                r.render(host.camera(W, H), W, H, kernel="hybrid", hot_pct=pct, hot_kernel="relay", rgb=rgb, hit=hit)
                outs.append((hit, rgb))
            r.sync()
            for hit, rgb in outs:
                np.testing.assert_array_equal(hit.cpu().numpy(), ref["hit"])
                assert same_bits(rgb.cpu().numpy(), ref["rgb"]), (pct, group)
            st = r.stats()
            for k in ("primary", "reflection", "shadow", "shadow_skipped", "hits", "pixels"):
                assert st[k] == ref["stats"][k], (pct, group, k)
        r.close()
