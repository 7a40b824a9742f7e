"""Host mirror of the reference cpu/ front end (loader, random mode, BVH, camera, BMP) over
librt_host.so (include/rt_host.h). Names follow the reference: triangles_load, lights_load,
bvh_build, cam_* -> camera(), bmp_write_file.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import BvhNode, BvhStats, Camera, Light, Rng, Triangle

P = ctypes.POINTER

TRI_DTYPE = np.dtype([("coords", np.float32, (3, 3)), ("centroid", np.float32, 3), ("ks", np.float32, 3),
                      ("kd", np.float32, 3), ("kr", np.float32, 3), ("norm", np.float32, (2, 3))])
NODE_DTYPE = np.dtype([("min", np.float32, 3), ("max", np.float32, 3), ("tr_len", np.int32), ("child", np.int32)])
LIGHT_DTYPE = np.dtype([("pos", np.float32, 3), ("kl", np.float32, 3)])
assert TRI_DTYPE.itemsize == 108 and NODE_DTYPE.itemsize == 32 and LIGHT_DTYPE.itemsize == 24

HEURISTICS = {"axis0": 0, "largest": 1, "random": 3, "sah32": 6, "binned_sah": 16}


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed with status {rc}")


class Rand:
    """glibc srand/rand restatement (rth_srand / rth_rand)."""

    def __init__(self, seed=1):
        self.state = Rng()
        _lib.host().rth_srand(ctypes.byref(self.state), seed)

    def rand(self):
        return _lib.host().rth_rand(ctypes.byref(self.state))


def _take(ptr, n, dtype):
    """copy n records from a malloc'd C array into numpy and free it"""
    L = _lib.host()
    if n:
        arr = np.frombuffer(ctypes.string_at(ptr, n * dtype.itemsize), dtype=dtype).copy()
    else:
        arr = np.zeros(0, dtype)
    L.rth_free(ptr)
    return arr


def triangles_load(obj, mtl, cache=None):
    """triangles_load(objname, mtlname, &size), cpu/src/triangle.c:74-126 -> structured array.
    cache: binary cache file (rth_triangles_load_cached): identical triangles, no re-parse when unchanged."""
    L = _lib.host()
    out = P(Triangle)()
    n = ctypes.c_size_t()
    if cache is None:
        _check(L.rth_triangles_load(obj.encode(), mtl.encode(), ctypes.byref(out), ctypes.byref(n)),
               f"triangles_load({obj})")
    else:
        hit = ctypes.c_int()
        _check(L.rth_triangles_load_cached(obj.encode(), mtl.encode(), str(cache).encode(), ctypes.byref(out),
                                           ctypes.byref(n), ctypes.byref(hit)), f"triangles_load({obj})")
        triangles_load.last_from_cache = bool(hit.value)
    return _take(out, n.value, TRI_DTYPE)


def bvh_build_cached(tris, heuristic, rng, cache):
    """bvh_build through the binary cache (rth_bvh_build_cached) -> (nodes, tri_idx, stats, from_cache);
    the RNG is left as after a real build"""
    L = _lib.host()
    h = HEURISTICS.get(heuristic, heuristic)
    tris = np.ascontiguousarray(tris, dtype=TRI_DTYPE)
    nodes = P(BvhNode)()
    idx = P(ctypes.c_int)()
    nlen = ctypes.c_int()
    st = BvhStats()
    hit = ctypes.c_int()
    _check(L.rth_bvh_build_cached(tris.ctypes.data_as(P(Triangle)), len(tris), h,
                                  ctypes.byref(rng.state) if rng is not None else None, str(cache).encode(),
                                  ctypes.byref(nodes), ctypes.byref(nlen), ctypes.byref(idx), ctypes.byref(st),
                                  ctypes.byref(hit)), "bvh_build_cached")
    return _take(nodes, nlen.value, NODE_DTYPE), _take(idx, len(tris), np.dtype(np.int32)), \
        {"leaves": st.leaves, "max_leaf": st.max_leaf, "max_depth": st.max_depth}, bool(hit.value)


def lights_load(path):
    """lights_load(filename, &size), cpu/src/light.c:6-29"""
    L = _lib.host()
    out = P(Light)()
    n = ctypes.c_size_t()
    _check(L.rth_lights_load(path.encode(), ctypes.byref(out), ctypes.byref(n)), f"lights_load({path})")
    return _take(out, n.value, LIGHT_DTYPE)


def triangles_random(n, rng):
    """random-triangle mode, cpu/src/main.c:115-131"""
    L = _lib.host()
    out = P(Triangle)()
    _check(L.rth_triangles_random(n, ctypes.byref(rng.state), ctypes.byref(out)), "triangles_random")
    return _take(out, n, TRI_DTYPE)


def bvh_build(tris, heuristic=3, rng=None):
    """bvh_build(triangles, n), cpu/src/bvh.c:360-388 -> (nodes, tri_idx, stats dict)"""
    L = _lib.host()
    h = HEURISTICS.get(heuristic, heuristic)
    tris = np.ascontiguousarray(tris, dtype=TRI_DTYPE)
    nodes = P(BvhNode)()
    idx = P(ctypes.c_int)()
    nlen = ctypes.c_int()
    st = BvhStats()
    _check(L.rth_bvh_build(tris.ctypes.data_as(P(Triangle)), len(tris), h,
                           ctypes.byref(rng.state) if rng is not None else None,
                           ctypes.byref(nodes), ctypes.byref(nlen), ctypes.byref(idx), ctypes.byref(st)),
           "bvh_build")
    nodes_np = _take(nodes, nlen.value, NODE_DTYPE)
    idx_np = _take(idx, len(tris), np.dtype(np.int32))
    stats = {"leaves": st.leaves, "min_leaf": st.min_leaf, "max_leaf": st.max_leaf,
             "max_depth": st.max_depth, "avg_leaf": st.avg_leaf, "nodes": nlen.value}
    return nodes_np, idx_np, stats


def wbvh_build(nodes, tri_idx, tris, inflate=0.0):
    """the fast walk's 8-wide quantised BVH (rth_wbvh_build, rt_wide.cpp) from a reference-layout BVH
    -> (words uint32 [n_nodes, 20], tri_order int32 [n], info dict)"""
    L = _lib.host()
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    tri_idx = np.ascontiguousarray(tri_idx, dtype=np.int32)
    tris = np.ascontiguousarray(tris, dtype=TRI_DTYPE)
    words = P(ctypes.c_uint32)()
    order = P(ctypes.c_int)()
    info = _lib.WbvhInfo()
    _check(L.rth_wbvh_build(nodes.ctypes.data_as(P(_lib.BvhNode)), len(nodes), tri_idx.ctypes.data_as(P(ctypes.c_int)),
                            tris.ctypes.data_as(P(Triangle)), len(tris), float(inflate), ctypes.byref(words),
                            ctypes.byref(order), ctypes.byref(info)), "wbvh_build")
    w = _take(words, 20 * info.n_nodes, np.dtype(np.uint32)).reshape(-1, 20)
    o = _take(order, info.n_tris, np.dtype(np.int32))
    return w, o, {"n_nodes": info.n_nodes, "depth": info.depth, "max_children": info.max_children}


def wbvh_decode(words):
    """decoded view of wide nodes: p [N,3] f32, scale [N,3] f32, imask [N], child_base [N], tri_base [N],
    meta [N,8] u8, qlo/qhi [N,3,8] u8 and the decoded child boxes lo/hi [N,8,3] (fmaf(scale, 1024 + q, p): the planes'
    f16-ready bias, rt_wide.cpp QBIAS)"""
    w = np.ascontiguousarray(words, dtype=np.uint32)
    p = w[:, 0:3].view(np.float32)
    e = np.stack([(w[:, 3] >> (8 * a)) & 0xFF for a in range(3)], 1).astype(np.uint8).view(np.int8)  # signed bytes
    scale = np.ldexp(np.float32(1), e.astype(np.int32)).astype(np.float32)
    imask = (w[:, 3] >> 24) & 0xFF
    meta = w[:, 6:8].copy().view(np.uint8).reshape(-1, 8)
    q = w[:, 8:20].copy().view(np.uint8).reshape(-1, 3, 8, 2)  # per axis: slot pairs' (lo, hi) side by side
    qlo, qhi = q[..., 0], q[..., 1]
    # fmaf(scale, 1024 + q, p) == p + scale * (1024 + q) rounded once (the product is exact): evaluate in f64, round
    lo = (p[:, :, None].astype(np.float64) + scale[:, :, None].astype(np.float64) * (1024.0 + qlo)).astype(np.float32)
    hi = (p[:, :, None].astype(np.float64) + scale[:, :, None].astype(np.float64) * (1024.0 + qhi)).astype(np.float32)
    return {"p": p, "scale": scale, "imask": imask, "child_base": w[:, 4].astype(np.int64),
            "tri_base": w[:, 5].astype(np.int64), "meta": meta, "qlo": qlo, "qhi": qhi,
            "lo": lo.transpose(0, 2, 1), "hi": hi.transpose(0, 2, 1)}


def camera(width, height):
    """cam_init + cam_calculate_screen_coords + inc_x/inc_y (cpu/src/cam.c, main.c:105-106,243-250)"""
    c = Camera()
    _check(_lib.host().rth_camera(width, height, ctypes.byref(c)), "camera")
    return c


def camera_array(cam):
    return np.array([[cam.pos.x, cam.pos.y, cam.pos.z], [cam.ul.x, cam.ul.y, cam.ul.z],
                     [cam.inc_x.x, cam.inc_x.y, cam.inc_x.z], [cam.inc_y.x, cam.inc_y.y, cam.inc_y.z]], np.float32)


def bmp_encode(rgb):
    """bmp_writer.c:148-175 -> bytes (32-bpp BGRA, bottom-up)"""
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    H, W = rgb.shape[:2]
    buf = np.zeros(54 + 4 * W * H, np.uint8)
    _check(_lib.host().rth_bmp_encode(rgb.ctypes.data, W, H, buf.ctypes.data, buf.size), "bmp_encode")
    return buf.tobytes()


def bmp_from_bgra(px):
    """bmp_write_file's bytes from pixels the kernels already quantised (rt_outputs.bgra: [H, W] or
    [H, W, 1] packed B|G<<8|R<<16|255<<24, top-down rows): the 54-byte header (bmp_writer.c:97-120,
    rth_bmp_header) + the rows bottom-up (bmp_writer.c:131-143). The root rank's BMP of a gathered frame."""
    px = np.ascontiguousarray(px)
    H, W = px.shape[:2]
    hdr = np.zeros(54, np.uint8)
    _check(_lib.host().rth_bmp_header(W, H, hdr.ctypes.data), "bmp_header")
    return hdr.tobytes() + px.reshape(H, W).view(np.uint32)[::-1].astype("<u4").tobytes()


def bmp_write_file(rgb, path):
    """bmp_write_file(pixels, width, height, filename), cpu/src/bmp_writer.c:177-211"""
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    H, W = rgb.shape[:2]
    _check(_lib.host().rth_bmp_write(rgb.ctypes.data, W, H, path.encode()), "bmp_write_file")


class Scene:
    """A loaded scene + its BVH: what the reference's main() holds in globals (main.c:27-43)."""

    def __init__(self, triangles, lights, seed=1, rng=None):
        self.triangles = triangles
        self.lights = lights
        self.rng = rng if rng is not None else Rand(seed)
        self.nodes = self.tri_idx = None
        self.bvh_stats = None
        self.amb = (0.5, 0.5, 0.5)  # amb_light, main.c:37

    @classmethod
    def load(cls, obj, mtl, lights, seed=1):
        rng = Rand(seed)  # srand(SEED) precedes loading, main.c:91-95
        return cls(triangles_load(obj, mtl), lights_load(lights) if lights else np.zeros(0, LIGHT_DTYPE), rng=rng)

    @classmethod
    def named(cls, name, seed=1):
        from .scenes import scene_paths
        return cls.load(*scene_paths(name), seed=seed)

    @classmethod
    def random(cls, ntris, seed=1):
        rng = Rand(seed)
        return cls(triangles_random(ntris, rng), np.zeros(0, LIGHT_DTYPE), rng=rng)

    def build_bvh(self, heuristic=3):
        self.nodes, self.tri_idx, self.bvh_stats = bvh_build(self.triangles, heuristic, self.rng)
        return self

    @property
    def n_triangles(self):
        return len(self.triangles)
