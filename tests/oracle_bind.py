"""ctypes binding to oracle/liboracle.so — TEST INFRASTRUCTURE ONLY (the checker, never the product).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
NCOUNT = 16
COUNTERS = ["primary", "reflection", "shadow", "shadow_skipped", "ch_inner", "ch_leaf", "ch_tri",
            "sh_inner", "sh_leaf", "sh_tri", "hits"]

_libs = {}


def lib(flavour="strict"):
    name = "liboracle.so" if flavour == "strict" else "liboracle_fast.so"
    if name not in _libs:
        path = os.path.join(ORACLE_DIR, name)
        if not os.path.exists(path):
            import subprocess
            subprocess.run(["make", "-C", ORACLE_DIR, "port"], check=True, stdout=subprocess.DEVNULL)
        L = ctypes.CDLL(path)
        vp, ci = ctypes.c_void_p, ctypes.c_int
        L.orc_scene_load.restype = vp
        L.orc_scene_load.argtypes = [ctypes.c_char_p] * 3 + [ctypes.c_uint]
        L.orc_scene_random.restype = vp
        L.orc_scene_random.argtypes = [ci, ctypes.c_uint]
        L.orc_scene_free.argtypes = [vp]
        L.orc_scene_ntris.argtypes = [vp]
        L.orc_scene_nlights.argtypes = [vp]
        L.orc_scene_triangles.restype = vp
        L.orc_scene_triangles.argtypes = [vp]
        L.orc_scene_lights.restype = vp
        L.orc_scene_lights.argtypes = [vp]
        L.orc_bvh_build.argtypes = [vp, ci]
        L.orc_bvh_export.argtypes = [vp, vp, vp]
        L.orc_set_use_bvh.argtypes = [vp, ci]
        L.orc_set_bounces.argtypes = [vp, ci]
        L.orc_camera.argtypes = [ci, ci, vp]
        L.orc_render.argtypes = [vp] + [ci] * 6 + [vp] * 5
        L.orc_render_spp.argtypes = [vp] + [ci] * 7 + [vp] * 2
        _libs[name] = L
    return _libs[name]


class OracleScene:
    def __init__(self, handle, flavour="strict"):
        if not handle:
            raise RuntimeError("oracle scene load failed")
        self.h = handle
        self.L = lib(flavour)

    @classmethod
    def load(cls, obj, mtl, lights, seed=1, flavour="strict"):
        L = lib(flavour)
        return cls(L.orc_scene_load(obj.encode(), mtl.encode(), lights.encode() if lights else None, seed), flavour)

    @classmethod
    def random(cls, n, seed=1, flavour="strict"):
        return cls(lib(flavour).orc_scene_random(n, seed), flavour)

    def __del__(self):
        try:
            self.L.orc_scene_free(self.h)
        except Exception:
            pass

    @property
    def ntris(self):
        return self.L.orc_scene_ntris(self.h)

    def triangles_bytes(self):
        return ctypes.string_at(self.L.orc_scene_triangles(self.h), 108 * self.ntris)

    def lights_bytes(self):
        n = self.L.orc_scene_nlights(self.h)
        return ctypes.string_at(self.L.orc_scene_lights(self.h), 24 * n) if n else b""

    def build_bvh(self, heuristic=3):
        n = self.L.orc_bvh_build(self.h, heuristic)
        if n < 0:
            raise RuntimeError("oracle bvh build failed")
        return n

    def bvh_export(self):
        n = self.L.orc_bvh_export(self.h, None, None)
        nodes = np.zeros(n * 32, np.uint8)
        idx = np.zeros(self.ntris, np.int32)
        self.L.orc_bvh_export(self.h, nodes.ctypes.data, idx.ctypes.data)
        return nodes.tobytes(), idx

    def set_use_bvh(self, on):
        self.L.orc_set_use_bvh(self.h, 1 if on else 0)

    def set_bounces(self, b):
        self.L.orc_set_bounces(self.h, b)

    def render(self, W, H, rows=None, threads=None, bounce_hits=False):
        ro, rs, nr = rows if rows is not None else (0, 1, H)
        N = W * H
        hit = np.full(N, -7, np.int32)
        t = np.zeros(N, np.float32)
        rgb = np.zeros(3 * N, np.float32)
        bh = np.full(4 * N, -7, np.int32) if bounce_hits else None
        c = np.zeros(NCOUNT, np.uint64)
        rc = self.L.orc_render(self.h, W, H, ro, rs, nr, threads or os.cpu_count() or 8, hit.ctypes.data,
                               t.ctypes.data, rgb.ctypes.data, bh.ctypes.data if bh is not None else None,
                               c.ctypes.data)
        if rc:
            raise RuntimeError(f"orc_render failed {rc}")
        out = {"hit": hit.reshape(H, W), "t": t.reshape(H, W), "rgb": rgb.reshape(H, W, 3),
               "counters": dict(zip(COUNTERS, (int(v) for v in c[:len(COUNTERS)])))}
        if bh is not None:
            out["bounce_hit"] = bh.reshape(H, W, 4)
        return out

    def render_spp(self, W, H, spp, rows=None, threads=None):
        ro, rs, nr = rows if rows is not None else (0, 1, H)
        rgb = np.zeros(3 * W * H, np.float32)
        c = np.zeros(NCOUNT, np.uint64)
        rc = self.L.orc_render_spp(self.h, W, H, spp, ro, rs, nr, threads or os.cpu_count() or 8,
                                   rgb.ctypes.data, c.ctypes.data)
        if rc:
            raise RuntimeError(f"orc_render_spp failed {rc}")
        return rgb.reshape(H, W, 3), dict(zip(COUNTERS, (int(v) for v in c[:len(COUNTERS)])))


def camera(W, H):
    out = np.zeros(12, np.float32)
    lib().orc_camera(W, H, out.ctypes.data)
    return out.reshape(4, 3)
