"""GPU-side BVH build (rt_scene.accel = RT_ACCEL_GPU, also the default RT_ACCEL_AUTO: PLOC over Morton-sorted triangles on the device,
rt_build.hpp) on the HIP path.

The fast walk returns the reference's answer for ANY conservative BVH (minimum t over all triangles; exact ties
and zero direction components re-walked strictly over the reference's own tree), so a GPU-built tree must render
exactly the reference fixtures' bits; only the speed depends on the tree. Bar: hit indices, t and colours
bit-exact against the fixtures made by the reference itself, ray counts equal, and rt_get_scene_info reporting
the GPU build (or the documented fallback to the host build for a tree too deep for the wide walk).
"""
import json
import os

import numpy as np
import pytest

from prt import host

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
G = json.load(open(os.path.join(GOLD, "golden.json")))


def render(scene, W, H, kernel, accel="gpu", counters=False):
    import torch
    from prt import device
    r = device.Renderer(0, counters=counters)
    r.upload(scene, accel=accel)
    info = r.scene_info()
    hit = torch.empty((H, W), dtype=torch.int32, device="cuda")
    t = torch.empty((H, W), dtype=torch.float32, device="cuda")
    rgb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    r.render(host.camera(W, H), W, H, kernel=kernel, rgb=rgb, hit=hit, t=t)
    st = r.stats()
    out = {"rgb": rgb.cpu().numpy(), "hit": hit.cpu().numpy(), "t": t.cpu().numpy(), "stats": st, "info": info}
    r.close()
    return out


def same_bits(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.int32), np.asarray(b, np.float32).view(np.int32))


@pytest.mark.parametrize("kernel", ["fast", "persist4", "coop4", "shdefer"])
@pytest.mark.parametrize("name,W,H,fixture", [("car_boxed", 160, 90, "car_boxed_160x90_strict"),
                                              ("car_only", 160, 90, "car_only_160x90_strict"),
                                              ("dragon", 96, 54, "dragon_96x54_strict"),
                                              ("sportscar", 96, 54, "sportscar_96x54_strict")])
def test_gpu_built_bvh_renders_the_reference_fixture(name, W, H, fixture, kernel):
    s = host.Scene.named(name).build_bvh(3)
    out = render(s, W, H, kernel)
    assert out["info"]["accel_built"] == "gpu", out["info"]
    assert out["info"]["wide_nodes"] > 0 and out["info"]["wide_depth"] <= 16
    ref = np.load(os.path.join(GOLD, fixture + ".npz"))
    np.testing.assert_array_equal(out["hit"], ref["hit"])
    assert same_bits(out["t"], ref["t"])
    assert same_bits(out["rgb"], ref["rgb"]), np.abs(out["rgb"] - ref["rgb"]).max()


@pytest.mark.parametrize("name", ["dragon", "dragon871k"])
def test_gpu_built_bvh_1080p_vs_reference(name):
    s = host.Scene.named(name).build_bvh(3)
    out = render(s, 1920, 1080, "fast", counters=True)
    assert out["info"]["accel_built"] == "gpu", out["info"]
    ref = np.load(os.path.join(GOLD, f"{name}_1080p_strict_sample.npz"))
    idx = ref["idx"]
    np.testing.assert_array_equal(out["hit"].reshape(-1)[idx], ref["hit"])
    assert same_bits(out["rgb"].reshape(-1, 3)[idx], ref["rgb"])
    st, rays = out["stats"], G["rays"][f"{name}_1920x1080"]
    assert st["primary"] + st["reflection"] == rays["closest"] and st["shadow"] == rays["shadow"]
    assert st["stack_overflows"] == 0


def test_host_built_bvh_still_renders_the_fixture():
    s = host.Scene.named("car_boxed").build_bvh(3)
    out = render(s, 160, 90, "fast", accel="host")
    assert out["info"]["accel_built"] == "host"
    ref = np.load(os.path.join(GOLD, "car_boxed_160x90_strict.npz"))
    assert same_bits(out["rgb"], ref["rgb"])
    np.testing.assert_array_equal(out["hit"], ref["hit"])
    assert render(s, 160, 90, "fast", accel="auto")["info"]["accel_built"] == "gpu"


def test_gpu_build_random_mode_and_fallback():
    """random-triangle mode: 10k and 1M triangles; a tree the wide walk cannot take falls back to the host
    build (reported), and either way the frame is the reference's"""
    for n, W, H, fx in ((10000, 160, 90, "random10k_160x90_strict"), (1000000, 96, 54, "random1m_96x54_strict")):
        s = host.Scene.random(n).build_bvh(3)
        out = render(s, W, H, "fast")
        assert out["info"]["accel_built"] in ("gpu", "host")
        ref = np.load(os.path.join(GOLD, fx + ".npz"))
        np.testing.assert_array_equal(out["hit"], ref["hit"])
        assert same_bits(out["rgb"], ref["rgb"])


def unit_hittable_count(scene, dmax=1.0):
    """triangles a direction of length <= dmax can hit: |e1 x e2| (float, tri_records' roundings) >=
    EPSILON (1 - 1e-5) / dmax (hit_triangle's |det| < EPSILON cull, cpu/src/raytracer.c:41-45)"""
    co = np.array(np.asarray(scene.triangles)["coords"].tolist(), dtype=np.float32)
    e1, e2 = co[:, 1] - co[:, 0], co[:, 2] - co[:, 0]
    n = np.stack([e1[:, 1] * e2[:, 2] - e1[:, 2] * e2[:, 1], e1[:, 2] * e2[:, 0] - e1[:, 0] * e2[:, 2],
                  e1[:, 0] * e2[:, 1] - e1[:, 1] * e2[:, 0]], axis=1).astype(np.float64)
    return int((np.sqrt((n * n).sum(1)) >= (1.0 - 1e-5) * float(np.float32(1e-3)) / dmax).sum())


@pytest.mark.parametrize("name,W,H,fixture", [("car_boxed", 160, 90, "car_boxed_160x90_strict"),
                                              ("dragon", 96, 54, "dragon_96x54_strict"),
                                              ("sportscar", 96, 54, "sportscar_96x54_strict")])
def test_unit_direction_view_renders_the_reference_fixture(name, W, H, fixture):
    """the unit-direction view (reflection and shadow rays walk a wide BVH without the triangles hit_triangle's
    |det| < EPSILON cull hides from every unit-length ray, rt_hip.hip unit_hittable): built over exactly the
    triangles the criterion keeps, and every kernel still renders the reference fixture's bits with the
    reference's ray counts"""
    s = host.Scene.named(name).build_bvh(3)
    want = unit_hittable_count(s)
    n = s.n_triangles
    ref = np.load(os.path.join(GOLD, fixture + ".npz"))
    for kernel in ("fast", "persist4", "coop4", "shpool"):
        out = render(s, W, H, kernel, counters=True)
        info = out["info"]
        assert 0 < want < n and info["unit_triangles"] == want, (info, want, n)
        assert info["unit_nodes"] > 0 and info["unit_depth"] <= 16
        np.testing.assert_array_equal(out["hit"], ref["hit"])
        assert same_bits(out["t"], ref["t"]) and same_bits(out["rgb"], ref["rgb"]), kernel


@pytest.mark.parametrize("name", ["sportscar", "car_boxed"])
def test_primary_view_and_long_primary_directions(name):
    """the primary view (primary rays of a launch whose directions are all <= 3 long walk a wide BVH without the
    triangles no such direction can hit): built over exactly the triangles the criterion keeps; a camera whose
    directions are longer (the reference camera with ul - pos and the pixel steps doubled: |d| up to 5.5) walks
    the full view and still equals the strict kernel (the reference's walk) bit for bit"""
    import torch
    from prt import device
    s = host.Scene.named(name).build_bvh(3)
    W, H = 96, 54
    r = device.Renderer(0, counters=True)
    r.upload(s)
    info = r.scene_info()
    assert info["primary_triangles"] == unit_hittable_count(s, 3.0) < s.n_triangles, info
    c = host.camera(W, H)
    for a, b in ((c.ul, c.pos),):
        a.x, a.y, a.z = b.x + 2 * (a.x - b.x), b.y + 2 * (a.y - b.y), b.z + 2 * (a.z - b.z)
    for v in (c.inc_x, c.inc_y):
        v.x, v.y, v.z = 2 * v.x, 2 * v.y, 2 * v.z
    outs = {}
    for kernel in ("strict", "fast", "persist4"):
        hit = torch.empty((H, W), dtype=torch.int32, device="cuda")
        rgb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        r.render(c, W, H, kernel=kernel, rgb=rgb, hit=hit)
        r.sync()
        outs[kernel] = (hit.cpu().numpy(), rgb.cpu().numpy(), r.stats()["rays"])
    r.close()
    for kernel in ("fast", "persist4"):
        np.testing.assert_array_equal(outs[kernel][0], outs["strict"][0])
        assert same_bits(outs[kernel][1], outs["strict"][1]) and outs[kernel][2] == outs["strict"][2], kernel

