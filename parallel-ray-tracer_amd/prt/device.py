"""Device mirror of the render seam over librt_hip.so (include/rt_hip.h):
load_to_gpu -> Renderer.upload, render_frame -> Renderer.render, load_from_gpu -> Renderer.download.

No fallback: if librt_hip.so is missing or no GPU is visible, constructing a Renderer raises.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import BvhNode, Camera, Frame, Light, Opts, SceneDesc, Stats, Triangle, Vec3

P = ctypes.POINTER

KERNELS = {"auto": 0, "strict": 1, "fast": 2}
# rt_frame.variant (launch configurations of the fast kernel, include/rt_hip.h); a variant name is also
# accepted as `kernel` (kernel="coop4" == kernel="fast", variant="coop4")
VARIANTS = {"default": 0, "persist": 1, "persist4": 2, "coop2": 4, "coop4": 5, "hybrid": 11, "shpool": 13, "shdefer": 15}
VARIANT_NAMES = {v: k for k, v in VARIANTS.items()}
HOT_KERNELS = {"coop4": 0, "coop2": 1}  # rt_frame.hot_kernel (RT_HOT_*)
DEALING = {"default": 0, "global": 1, "rows": 2, "columns": 3, "blocks": 4, "row_major": 5}
ACCEL = {"auto": 0, "reference": 1, "gpu": 2, "host": 3}
ACCEL_NAMES = {v: k for k, v in ACCEL.items()}
FLAG_COUNTERS = 1
FLAG_UNPACKED_STACK = 2  # the builds scenes of more than 2^24 wide nodes run (rt_hip.h RT_FLAG_UNPACKED_STACK)
FLAG_UNPACKED_TRIS = 4   # the builds scenes of 2^26 or more triangles run (RT_FLAG_UNPACKED_TRIS)


class RtError(RuntimeError):
    pass


class Outputs(ctypes.Structure):
    _fields_ = [("rgb", ctypes.c_void_p), ("hit", ctypes.c_void_p), ("t", ctypes.c_void_p),
                ("bounce_hit", ctypes.c_void_p), ("bgra", ctypes.c_void_p)]


_lib.hip()  # fail loudly at import if the HIP library is absent
_L = _lib.hip()
_L.rt_render.argtypes = [ctypes.c_void_p, P(Camera), P(Frame), P(Outputs)]
_L.rt_gather.argtypes = [P(ctypes.c_void_p), ctypes.c_int, ctypes.c_int]
_L.rt_download_bmp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]


def lib_md5():
    """md5 of the librt_hip.so this process loaded"""
    return _lib.lib_md5("librt_hip.so")


def device_count():
    return _L.rt_device_count()


def gather(renderers, root=0, out=None):
    """rt_gather: the last renders of several Renderers (frames or frame batches whose rows partition each
    frame) -> renderers[root]'s device frames; afterwards renderers[root].download() / download_bmp() return
    the full frame. out: a contiguous device tensor for the full frames instead (rt_gather_to), e.g. a batch
    [frames, H, W, 3] f32 or [frames, H, W] int32 (BGRA8)."""
    arr = (ctypes.c_void_p * len(renderers))(*[r._ctx.value for r in renderers])
    if out is not None:
        rc = _L.rt_gather_to(arr, len(renderers), root, ctypes.c_void_p(_gather_out(renderers[root], out)))
    else:
        rc = _L.rt_gather(arr, len(renderers), root)
    r = renderers[root]
    r._chk(rc, "rt_gather")
    W, H = r._size
    r._last = (W, H)


def _gather_out(r, out):
    """device pointer of a gather's full-frame output tensor: contiguous, on the root's device, of the root's
    last render's pixel format (float32 for rgb, int32 for BGRA8: rt_gather_to / rt_comm_gather move the bgra
    pixels when the render wrote them) and holding every frame of that render (frames x H x W x words); a
    short or mistyped tensor is refused here rather than overrun on the device"""
    import torch
    if not hasattr(r, "_size"):
        raise RtError("gather out: the root renderer has not rendered")
    W, H = r._size
    words = r._words
    want = torch.int32 if words == 1 else torch.float32
    return _ptr(out, "gather out", r._frames * W * H * words, (want,), r.device)


COMM_ID_BYTES = 128  # RT_COMM_ID_BYTES


def comm_id():
    """rt_comm_get_id: a fresh RCCL unique id (bytes) for rt_comm_init_rank; rank 0 makes it, every rank gets it"""
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    if _L.rt_comm_get_id(buf) != 0:
        raise RtError("rt_comm_get_id failed")
    return buf.raw


class Comm:
    """rt_comm: an RCCL communicator over Renderers (SURVEY §8e's framebuffer gather over xGMI).
    Comm(renderers): one process, one Renderer per device (rt_comm_init); Comm([renderer], nranks, rank, id):
    one rank of a multi-process job (rt_comm_init_rank)."""

    def __init__(self, renderers, nranks=None, rank=None, uid=None):
        self._r = list(renderers)
        self._c = ctypes.c_void_p()
        if nranks is None:
            arr = (ctypes.c_void_p * len(self._r))(*[r._ctx.value for r in self._r])
            rc = _L.rt_comm_init(arr, len(self._r), ctypes.byref(self._c))
        else:
            assert len(self._r) == 1 and uid is not None and len(uid) == COMM_ID_BYTES
            rc = _L.rt_comm_init_rank(self._r[0]._ctx, nranks, rank, ctypes.create_string_buffer(uid, COMM_ID_BYTES),
                                      ctypes.byref(self._c))
        if rc != 0:
            raise RtError(f"rt_comm_init: {rc} ({_L.rt_last_error(self._r[0]._ctx).decode()})")
        self.rank0 = 0 if rank is None else rank

    def gather(self, root=0, out=None, src=None):
        """rt_comm_gather: every rank's last render -> the root's full frames; `out` (root only): a contiguous
        device tensor [frames, H, W, 3] f32 or [frames, H, W] int32 (BGRA8), else the root Renderer's own
        buffer (its download() / download_bmp() then read the full frame). src (multi-process communicators): the
        Renderer of this rank whose last render to send (rt_comm_gather_from; default: the one it was built with)."""
        ptr = None
        here = [src] if src is not None else self._r
        if out is not None:
            ptr = ctypes.c_void_p(_gather_out(here[root - self.rank0] if 0 <= root - self.rank0 < len(here)
                                              else here[0], out))
        if src is not None:
            if all(src is not x for x in self._r):
                self._r.append(src)  # (kept alive while the communicator may still use its stream)
            rc = _L.rt_comm_gather_from(self._c, src._ctx, root, ptr)
        else:
            rc = _L.rt_comm_gather(self._c, root, ptr)
        if rc != 0:
            raise RtError(f"rt_comm_gather: {rc} ({_L.rt_comm_last_error(self._c).decode()})")
        lr = root - self.rank0
        if 0 <= lr < len(here):
            r = here[lr]
            r._last = r._size

    def set_timeout(self, seconds):
        """rt_comm_set_timeout: the deadline of every host wait on a collective (a peer that never joins turns into
        RT_E_TIMEOUT and an aborted communicator instead of a hang)"""
        if _L.rt_comm_set_timeout(self._c, float(seconds)) != 0:
            raise RtError("rt_comm_set_timeout failed")

    def relayout(self):
        """rt_comm_relayout (collective): the next gather exchanges the ranks' row sets again"""
        if _L.rt_comm_relayout(self._c) != 0:
            raise RtError("rt_comm_relayout failed")

    def wait(self):
        """rt_comm_wait: bounded wait for the last gather; raises on a timeout (the communicator is aborted)"""
        rc = _L.rt_comm_wait(self._c)
        if rc != 0:
            raise RtError(f"rt_comm_wait: {rc} ({_L.rt_comm_last_error(self._c).decode()})")

    def info(self):
        """rt_comm_get_info: gathers, descriptor exchanges (one per layout), layouts checked pixel by pixel"""
        i = _lib.CommInfo()
        if _L.rt_comm_get_info(self._c, ctypes.byref(i)) != 0:
            raise RtError("rt_comm_get_info failed")
        return {f: getattr(i, f) for f, _ in _lib.CommInfo._fields_}

    def close(self):
        if self._c:
            _L.rt_comm_destroy(self._c)
            self._c = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _ptr(x, what="", n=0, dtypes=(), device=None):
    """device pointer of a torch tensor / raw int pointer / None. A tensor must be contiguous, of one of
    `dtypes`, on `device` and hold at least n elements (the kernel writes n of them); raw pointers are the
    caller's responsibility."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    import torch
    if not isinstance(x, torch.Tensor):
        raise RtError(f"{what}: expected a torch tensor, an int pointer or None, got {type(x).__name__}")
    if not x.is_contiguous():
        raise RtError(f"{what}: tensor is not contiguous")
    if dtypes and x.dtype not in dtypes:
        raise RtError(f"{what}: dtype {x.dtype}, expected {' or '.join(str(d) for d in dtypes)}")
    if x.numel() < n:
        raise RtError(f"{what}: {x.numel()} elements, the frame needs {n}")
    if x.device.type != "cuda" or (device is not None and x.device.index != device):
        raise RtError(f"{what}: tensor on {x.device}, expected cuda:{device}")
    return x.data_ptr()


def _rows(rows, height):
    """rows tuple (offset, stride, n[, block[, frame_shift]]) -> rt_frame fields; None = full frame"""
    if rows is None:
        return 0, 1, height, 1, 0
    r = tuple(rows)
    return r + (1, 0)[len(r) - 3:] if len(r) < 5 else r[:5]


class Renderer:
    """One rt_ctx on one device (gpu.cuh:23-26 seam, explicit instead of global)."""

    def __init__(self, device=0, counters=False, stream=None, flags=0):
        """flags: more rt_opts.flags (FLAG_UNPACKED_STACK / FLAG_UNPACKED_TRIS: the unpacked builds for any scene)"""
        self._ctx = ctypes.c_void_p()
        opts = Opts(device, (FLAG_COUNTERS if counters else 0) | flags, stream)
        rc = _L.rt_create(ctypes.byref(opts), ctypes.byref(self._ctx))
        if rc != 0:
            raise RtError(f"rt_create(device={device}) failed with status {rc}")
        self.device = device
        self.scene = None

    def _chk(self, rc, what):
        if rc != 0:
            raise RtError(f"{what}: status {rc}: {_L.rt_last_error(self._ctx).decode()}")

    def upload(self, scene, accel="auto", ploc_radius=0, collapse_node_cost=0.0):
        """load_to_gpu(): scene = prt.host.Scene with a built BVH (the reference's bvh_build output).
        accel="auto" / "gpu": the library builds the fast kernel's BVH on the GPU (PLOC, rt_build.hpp) and
        collapses it to the 8-wide layout ("host": a binned SAH on the host instead; "auto" falls back to it
        when the GPU tree is too deep for the wide walk); accel="reference": the fast kernel traverses the given
        BVH too."""
        if scene.nodes is None:
            raise RtError("upload: build the BVH first")
        tris = np.ascontiguousarray(scene.triangles)
        nodes = np.ascontiguousarray(scene.nodes)
        idx = np.ascontiguousarray(scene.tri_idx, dtype=np.int32)
        lights = np.ascontiguousarray(scene.lights)
        d = SceneDesc(tris.ctypes.data_as(P(Triangle)), len(tris), nodes.ctypes.data_as(P(BvhNode)), len(nodes),
                      idx.ctypes.data_as(P(ctypes.c_int)),
                      lights.ctypes.data_as(P(Light)) if len(lights) else None, len(lights), Vec3(*scene.amb),
                      ACCEL.get(accel, accel), ploc_radius, collapse_node_cost)
        self._chk(_L.rt_upload_scene(self._ctx, ctypes.byref(d)), "rt_upload_scene")
        self.scene = scene
        return self

    def _frame(self, width, height, rows, bounces, spp, kernel, variant, tune, waves_cap, dealing, regroup, hot_pct=0,
               hot_kernel="coop4"):
        ro, rs, nr, rb, sh = _rows(rows, height)
        if isinstance(kernel, str) and kernel in VARIANTS:
            kernel, variant = "fast", kernel
        v = VARIANTS.get(variant, variant) if variant is not None else 0
        return Frame(width, height, ro, rs, nr, bounces, spp, KERNELS.get(kernel, kernel), rb, sh, v,
                     1 if tune else 0, waves_cap, DEALING.get(dealing, dealing), regroup, hot_pct,
                     HOT_KERNELS.get(hot_kernel, hot_kernel)), nr

    def _outputs(self, nf, nr, width, bounces, rgb, hit, t, bounce_hit, bgra):
        import torch
        n = nf * nr * width
        i32 = (torch.int32,)
        return Outputs(_ptr(rgb, "rgb", 3 * n, (torch.float32,), self.device),
                       _ptr(hit, "hit", n, i32, self.device), _ptr(t, "t", n, (torch.float32,), self.device),
                       _ptr(bounce_hit, "bounce_hit", n * bounces, i32, self.device),
                       _ptr(bgra, "bgra", n, (torch.int32, getattr(torch, "uint32", torch.int32)), self.device))

    def render(self, cam, width, height, rows=None, bounces=4, spp=1, kernel="auto", rgb=None, hit=None, t=None,
               bounce_hit=None, bgra=None, variant=None, tune=False, waves_cap=0, dealing="default", regroup=0,
               hot_pct=0, hot_kernel="coop4"):
        """render_frame(): asynchronous. rows = (offset, stride, n[, block[, frame_shift]]) (rt_frame; prt.dist)
        or None for the full frame.
        rgb / hit / t / bounce_hit ([n, W, bounces] int32) / bgra ([n, W] int32: the BMP-quantised pixel in
        top-down rows, rt_outputs.bgra): optional device tensors (torch: checked for size, dtype, device and
        contiguity) or raw pointers. variant / tune / waves_cap / dealing / regroup / hot_pct / hot_kernel: the fast
        kernel's launch configuration (rt_frame; VARIANTS, DEALING, HOT_KERNELS)."""
        f, nr = self._frame(width, height, rows, bounces, spp, kernel, variant, tune, waves_cap, dealing, regroup,
                            hot_pct, hot_kernel)
        out = self._outputs(1, nr, width, bounces, rgb, hit, t, bounce_hit, bgra)
        self._chk(_L.rt_render(self._ctx, ctypes.byref(cam), ctypes.byref(f), ctypes.byref(out)), "rt_render")
        self._last = (width, nr)
        self._size = (width, height)
        self._frames = 1
        self._words = 1 if bgra is not None else 3  # the payload a gather moves (rt_hip.hip payload_of)

    def render_frames(self, cams, width, height, rows=None, bounces=4, spp=1, kernel="auto", rgb=None, hit=None,
                      t=None, bounce_hit=None, bgra=None, variant=None, tune=False, waves_cap=0, dealing="default",
                      regroup=0):
        """rt_render_frames(): a batch of len(cams) frames of one shape (one persistent launch on the fast
        kernel); outputs [n_frames, n_rows, W, ...]. Asynchronous."""
        f, nr = self._frame(width, height, rows, bounces, spp, kernel, variant, tune, waves_cap, dealing, regroup)
        out = self._outputs(len(cams), nr, width, bounces, rgb, hit, t, bounce_hit, bgra)
        arr = (Camera * len(cams))(*cams)
        self._chk(_L.rt_render_frames(self._ctx, arr, len(cams), ctypes.byref(f), ctypes.byref(out)),
                  "rt_render_frames")
        self._last = (width, nr)
        self._size = (width, height)
        self._frames = len(cams)
        self._words = 1 if bgra is not None else 3

    def sync(self):
        ms = ctypes.c_float()
        self._chk(_L.rt_sync(self._ctx, ctypes.byref(ms)), "rt_sync")
        return ms.value

    def kernel_times(self, n):
        """per-launch kernel ms of the last n renders (HIP events on the launch stream)"""
        buf = (ctypes.c_float * max(n, 1))()
        got = _L.rt_kernel_times(self._ctx, buf, n)
        if got < 0:
            self._chk(got, "rt_kernel_times")
        return [buf[i] for i in range(got)]

    def download(self, hit=False):
        """load_from_gpu(): the last frame's compact rows -> (rgb[n_rows, W, 3], hit or None)"""
        W, nr = self._last
        nf = getattr(self, "_frames", 1)
        shp = (nr, W) if nf == 1 else (nf, nr, W)
        rgb = np.zeros(shp + (3,), np.float32)
        h = np.zeros(shp, np.int32) if hit else None
        self._chk(_L.rt_download(self._ctx, rgb.ctypes.data, h.ctypes.data if hit else None), "rt_download")
        return rgb, h

    def download_bmp(self):
        """bmp_write_file's bytes of the last (full) frame, quantised on the device (rt_download_bmp)"""
        W, H = self._size
        buf = np.zeros(54 + 4 * W * H, np.uint8)
        self._chk(_L.rt_download_bmp(self._ctx, buf.ctypes.data, buf.size), "rt_download_bmp")
        return buf.tobytes()

    def scene_info(self):
        """rt_get_scene_info: what the last upload built (accel_built: "host" = host binned SAH, "gpu" = PLOC on
        the device, "reference" = the handed-over BVH), the wide BVH's size and depth, build times"""
        i = _lib.SceneInfo()
        self._chk(_L.rt_get_scene_info(self._ctx, ctypes.byref(i)), "rt_get_scene_info")
        d = {f: getattr(i, f) for f, _ in _lib.SceneInfo._fields_}
        d["accel_built"] = ACCEL_NAMES.get(d["accel_built"], d["accel_built"])
        return d

    def launch_info(self):
        """rt_get_launch_info: what the last render ran (variant name, hot tiles, cold kernel) and whether it was a
        measuring / trial frame of the default rule (`trial`) or the shape's decided configuration (`settled`);
        no synchronisation"""
        i = _lib.LaunchInfo()
        self._chk(_L.rt_get_launch_info(self._ctx, ctypes.byref(i)), "rt_get_launch_info")
        d = {f: getattr(i, f) for f, _ in _lib.LaunchInfo._fields_}
        d["variant"] = VARIANT_NAMES.get(d["variant"], d["variant"])
        d["cold_variant"] = VARIANT_NAMES.get(d["cold_variant"], d["cold_variant"])
        d["build_bits"] = sorted(k for k, v in _lib.BUILD_BITS.items() if d["build"] & v)
        return d

    def stats(self):
        s = Stats()
        self._chk(_L.rt_get_stats(self._ctx, ctypes.byref(s)), "rt_get_stats")
        d = {f: getattr(s, f) for f in _lib.STAT_FIELDS}
        d["rays"] = d["primary"] + d["reflection"] + d["shadow"]
        # wave steps [kind: closest, shadow][level 0, 1, 2, 3+][active lanes 1-16, 17-32, 33-48, 49-64]
        h = list(s.steps_hist)
        d["steps_hist"] = [[h[16 * k + 4 * l:16 * k + 4 * l + 4] for l in range(4)] for k in range(2)]
        return d

    def close(self):
        if self._ctx:
            _L.rt_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
