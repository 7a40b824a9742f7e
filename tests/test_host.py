"""librt_host.so (the product's host half) against the oracle and the reference fixtures."""
import ctypes
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from prt import host
from tests.oracle_bind import OracleScene, camera as orc_camera
from tests.scenes import scene_paths

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
G = json.load(open(os.path.join(GOLD, "golden.json")))


def test_rand_matches_libc():
    libc = ctypes.CDLL("libc.so.6")
    for seed in (1, 7, 12345, 0):
        libc.srand(seed)
        r = host.Rand(seed)
        ours = [r.rand() for _ in range(5000)]
        theirs = [libc.rand() for _ in range(5000)]
        assert ours == theirs, seed


@pytest.mark.parametrize("scene", ["car_boxed", "car_only"])
def test_loader_matches_oracle(scene):
    obj, mtl, lts = scene_paths(scene)
    tris = host.triangles_load(obj, mtl)
    lights = host.lights_load(lts)
    o = OracleScene.load(obj, mtl, lts)
    assert len(tris) == o.ntris
    assert tris.tobytes() == o.triangles_bytes()
    assert lights.tobytes() == o.lights_bytes()


def test_loader_missing_file_is_an_error(tmp_path):
    with pytest.raises(RuntimeError):
        host.triangles_load(str(tmp_path / "nope.obj"), str(tmp_path / "nope.mtl"))


def test_loader_edge_cases(tmp_path):
    """fgets(256) chunking, 5-line MTL window, unknown usemtl keeps previous, missing keys = 0."""
    mtl = tmp_path / "m.mtl"
    mtl.write_text("newmtl a\nKd 1 0 0\nKs 0 1 0\nKr .5 .5 .5\n\n\nnewmtl b\nNs 1\nNs 1\nNs 1\nNs 1\nNs 1\nKd 9 9 9\n")
    obj = tmp_path / "t.obj"
    long_comment = "#" + "x" * 600 + "\n"
    obj.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\n" + long_comment + "f 1 2 3\nusemtl a\nf 1 2 3\n"
                   "usemtl zzz\nf 3 2 1\nusemtl b\nf 1 3 2\n")
    tris = host.triangles_load(str(obj), str(mtl))
    o = OracleScene.load(str(obj), str(mtl), None)
    assert tris.tobytes() == o.triangles_bytes()
    assert len(tris) == 4
    assert tris[0]["kd"].tolist() == [0, 0, 0]
    assert tris[1]["kd"].tolist() == [1, 0, 0] and tris[2]["kd"].tolist() == [1, 0, 0]
    assert tris[3]["kd"].tolist() == [0, 0, 0]  # Kd of b is outside the 5-line window


@pytest.mark.parametrize("scene", ["car_boxed", "car_only"])
def test_bvh_h3_bit_identical_to_reference(scene):
    s = host.Scene.named(scene).build_bvh(3)
    raw = np.int32(len(s.nodes)).tobytes() + s.nodes.tobytes() + s.tri_idx.astype(np.int32).tobytes()
    assert hashlib.md5(raw).hexdigest() == G["bvh"][scene + "_h3"]["md5"]
    st = s.bvh_stats
    if scene == "car_boxed":  # bvh.c:381-387 as printed by the reference
        assert (st["leaves"], st["min_leaf"], st["max_leaf"]) == (29421, 1, 61)


def test_bvh_h6_matches_oracle():
    """heuristic 6 (gpu default) is FP-contraction sensitive: the strict build (this library) equals the
    strict oracle; SURVEY's md5 is the fast-math build's (checked in test_oracle)."""
    s = host.Scene.named("car_boxed").build_bvh(6)
    o = OracleScene.load(*scene_paths("car_boxed"))
    assert o.build_bvh(6) == len(s.nodes) == 57733
    nodes, idx = o.bvh_export()
    assert s.nodes.tobytes() == nodes
    np.testing.assert_array_equal(s.tri_idx, idx)


@pytest.mark.parametrize("scene", ["dragon", "two_cars", "sportscar", "dragon871k"])
def test_bvh_h3_standins_match_reference(scene):
    """multi-material scenes exercise the reference's axis-3 read (bvh.c:229-231) as laid out by O-strict"""
    s = host.Scene.named(scene).build_bvh(3)
    raw = np.int32(len(s.nodes)).tobytes() + s.nodes.tobytes() + s.tri_idx.astype(np.int32).tobytes()
    assert hashlib.md5(raw).hexdigest() == G["standin"][scene]["bvh_h3_md5"]


def test_bvh_random_mode_matches_reference():
    s = host.Scene.random(10000).build_bvh(3)
    raw = np.int32(len(s.nodes)).tobytes() + s.nodes.tobytes() + s.tri_idx.astype(np.int32).tobytes()
    assert hashlib.md5(raw).hexdigest() == G["bvh"]["random10k_h3"]["md5"]
    o = OracleScene.random(10000)
    assert s.triangles.tobytes() == o.triangles_bytes()


def test_bvh_random_mode_one_million_matches_reference():
    """random mode at 1M triangles (SURVEY §8d's BVH stress): the heuristic-3 tree is the reference's"""
    s = host.Scene.random(1000000).build_bvh(3)
    raw = np.int32(len(s.nodes)).tobytes() + s.nodes.tobytes() + s.tri_idx.astype(np.int32).tobytes()
    assert hashlib.md5(raw).hexdigest() == G["bvh"]["random1m_h3"]["md5"]


def _check_tree(nodes, idx, tris):
    n = len(tris)
    assert sorted(idx.tolist()) == list(range(n))
    seen = np.zeros(n, int)
    stack = [(0, 0)]
    maxd = 0
    while stack:
        i, d = stack.pop()
        maxd = max(maxd, d)
        nd = nodes[i]
        if nd["tr_len"] > 0:
            sl = idx[nd["child"]:nd["child"] + nd["tr_len"]]
            seen[sl] += 1
            v = tris["coords"][sl].reshape(-1, 3)
            assert (v >= nd["min"] - 1e-6).all() and (v <= nd["max"] + 1e-6).all()
        elif nd["child"]:
            for c in (nd["child"], nd["child"] + 1):
                ch = nodes[c]
                if ch["tr_len"] > 0 or ch["child"]:
                    assert (ch["min"] >= nd["min"]).all() and (ch["max"] <= nd["max"]).all()
                stack.append((c, d + 1))
    assert (seen == 1).all()
    return maxd


@pytest.mark.parametrize("scene", ["car_boxed", "dragon"])
def test_binned_sah_is_a_valid_bvh(scene):
    s = host.Scene.named(scene).build_bvh("binned_sah")
    assert _check_tree(s.nodes, s.tri_idx, s.triangles) <= 24  # the fast kernels' stack bound
    assert s.bvh_stats["max_leaf"] <= 8


def test_binned_sah_random_mode_depth_cap():
    s = host.Scene.random(20000).build_bvh("binned_sah")
    assert _check_tree(s.nodes, s.tri_idx, s.triangles) <= 24


@pytest.mark.parametrize("W,H", [(1920, 1080), (640, 360), (160, 90), (7, 3)])
def test_camera_matches_oracle(W, H):
    c = host.camera_array(host.camera(W, H))
    np.testing.assert_array_equal(c.view(np.int32), orc_camera(W, H).view(np.int32))


def test_bmp_matches_reference_writer(tmp_path):
    ref = np.load(os.path.join(GOLD, "car_boxed_160x90_strict.npz"))
    data = host.bmp_encode(ref["rgb"])
    p = tmp_path / "x.bmp"
    host.bmp_write_file(ref["rgb"], str(p))
    assert p.read_bytes() == data
    refbin = os.path.join(os.path.dirname(GOLD), "..", "oracle", "_ref", "rt_ref_strict")
    if os.path.exists(refbin) and os.path.exists("/root/reference"):
        q = tmp_path / "ref.bmp"
        subprocess.run([refbin, "bmp", *scene_paths("car_boxed"), "160", "90", "4", str(q)], check=True,
                       stdout=subprocess.DEVNULL)
        assert q.read_bytes() == data
    # header and layout (bmp_writer.c:97-143)
    assert data[:2] == b"BM" and int.from_bytes(data[2:6], "little") == 54 + 160 * 90 * 4
    px = np.frombuffer(data[54:], np.uint8).reshape(90, 160, 4)
    np.testing.assert_array_equal(px[-1, :, 2], (ref["rgb"][0, :, 0] * np.float32(255)).astype(np.uint8))
    assert (px[..., 3] == 255).all()


def test_empty_scene_bvh_is_an_error():
    with pytest.raises(RuntimeError):
        host.bvh_build(np.zeros(0, host.TRI_DTYPE), 3, host.Rand(1))


def _check_wbvh(s, inflate):
    """every triangle reachable exactly once; every decoded child box contains its subtree's triangles
    grown by `inflate` (the conservativeness the fast walk relies on); leaf slots hold 1..4 triangles
    inside the node's 32-triangle window; children of a node are consecutive records"""
    words, order, info = host.wbvh_build(s.nodes, s.tri_idx, s.triangles, inflate)
    D = host.wbvh_decode(words)
    memo = {}
    n = len(s.triangles)
    assert sorted(order.tolist()) == list(range(n))
    v = s.triangles["coords"].astype(np.float32)  # [n, 3, 3]
    tlo, thi = v.min(1), v.max(1)
    N = len(words)
    seen_node = np.zeros(N, int)
    seen_tri = np.zeros(n, int)
    stack = [(0, 1)]
    maxd = 0
    while stack:
        k, d = stack.pop()
        seen_node[k] += 1
        maxd = max(maxd, d)
        internal = [s_ for s_ in range(8) if (D["imask"][k] >> s_) & 1]
        for s_ in range(8):
            m = int(D["meta"][k, s_])
            lo, hi = D["lo"][k, s_], D["hi"][k, s_]
            if s_ in internal:
                c = int(D["child_base"][k]) + sum(1 for j in internal if j < s_)
                stack.append((c, d + 1))
                sub = _wbvh_subtree_tris(D, c, order, memo)
            elif m:
                cnt, off = m >> 5, m & 31
                assert 1 <= cnt <= 4 and off + cnt <= 32
                sub = order[int(D["tri_base"][k]) + off: int(D["tri_base"][k]) + off + cnt]
                seen_tri[sub] += 1
            else:
                continue
            assert (lo <= tlo[sub] - inflate).all() and (hi >= thi[sub] + inflate).all(), (k, s_)
    assert (seen_node == 1).all() and (seen_tri == 1).all()
    assert maxd == info["depth"]
    return info


def _wbvh_subtree_tris(D, k, order, memo):
    """the triangles under wide node k (memo: one dict per decoded tree -- a module-level cache keyed by id(D) would
    serve a collected tree's entries to a later tree that reuses its address)"""
    key = k
    if key in memo:
        return memo[key]
    out = []
    internal = [s_ for s_ in range(8) if (D["imask"][k] >> s_) & 1]
    for s_ in range(8):
        m = int(D["meta"][k, s_])
        if s_ in internal:
            c = int(D["child_base"][k]) + sum(1 for j in internal if j < s_)
            out.append(_wbvh_subtree_tris(D, c, order, memo))
        elif m:
            off, cnt = m & 31, m >> 5
            out.append(order[int(D["tri_base"][k]) + off: int(D["tri_base"][k]) + off + cnt])
    memo[key] = np.concatenate(out) if out else np.zeros(0, np.int32)
    return memo[key]


@pytest.mark.parametrize("scene", ["car_boxed", "dragon"])
def test_wide_bvh_is_conservative_and_complete(scene):
    s = host.Scene.named(scene).build_bvh("binned_sah")
    mx = max(16.0, float(np.abs(s.triangles["coords"]).max()))
    info = _check_wbvh(s, np.ldexp(np.float32(mx), -18))
    assert info["depth"] <= 16 and info["max_children"] <= 8  # the fast walk's LDS stack bound


def test_wide_bvh_from_reference_layout_and_random_mode():
    """any reference-layout tree works, incl. the reference's own h3 BVH with leaves > 4 triangles"""
    s = host.Scene.named("car_only").build_bvh(3)
    assert s.bvh_stats["max_leaf"] > 4
    _check_wbvh(s, 0.0)
    _check_wbvh(host.Scene.random(5000).build_bvh("binned_sah"), 1e-4)


def test_wide_bvh_single_triangle():
    s = host.Scene.random(1).build_bvh("binned_sah")
    words, order, info = host.wbvh_build(s.nodes, s.tri_idx, s.triangles, 0.0)
    assert info["n_nodes"] == 1 and order.tolist() == [0]


def test_scene_cache_returns_the_loaders_bytes(tmp_path):
    """SURVEY §8f.2 binary cache: identical triangles and BVH (and RNG state after it) from the cache;
    a changed source file or a damaged cache file is never trusted"""
    import shutil
    obj, mtl, lts = scene_paths("car_only")
    o2, m2 = tmp_path / "t.obj", tmp_path / "t.mtl"
    shutil.copy(obj, o2)
    shutil.copy(mtl, m2)
    cache = tmp_path / "tris.prtc"
    ref = host.triangles_load(obj, mtl)
    a = host.triangles_load(str(o2), str(m2), cache=cache)
    assert not host.triangles_load.last_from_cache and cache.exists()
    b = host.triangles_load(str(o2), str(m2), cache=cache)
    assert host.triangles_load.last_from_cache
    assert a.tobytes() == b.tobytes() == ref.tobytes()
    with open(o2, "a") as f:  # stale: the OBJ changed
        f.write("f 1 2 3\n")
    c = host.triangles_load(str(o2), str(m2), cache=cache)
    assert not host.triangles_load.last_from_cache and len(c) == len(ref) + 1
    raw = bytearray(cache.read_bytes())  # damaged: one flipped payload byte
    raw[100] ^= 0xFF
    cache.write_bytes(bytes(raw))
    d = host.triangles_load(str(o2), str(m2), cache=cache)
    assert not host.triangles_load.last_from_cache and d.tobytes() == c.tobytes()
    # the reference BVH (heuristic 3 consumes rand()): cached == built, RNG continues identically
    bc = tmp_path / "bvh.prtc"
    r1, r2, r3 = host.Rand(1), host.Rand(1), host.Rand(1)
    n0, i0, _ = host.bvh_build(ref, 3, r1)
    n1, i1, _, hit1 = host.bvh_build_cached(ref, 3, r2, bc)
    n2, i2, _, hit2 = host.bvh_build_cached(ref, 3, r3, bc)
    assert (hit1, hit2) == (False, True)
    assert n0.tobytes() == n1.tobytes() == n2.tobytes() and i0.tobytes() == i2.tobytes()
    assert r1.rand() == r2.rand() == r3.rand()
