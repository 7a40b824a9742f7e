"""prt — MI355X-native drop-in for the per-pixel render path of deluf/parallel-ray-tracer.

Python mirror of the reference's host interface, over two C-ABI libraries built in-tree:
  librt_host.so (include/rt_host.h)  scene loader, camera, BVH builders, BMP writer (C++)
  librt_hip.so  (include/rt_hip.h)   the per-pixel hot path as HIP kernels for gfx950

`prt.host` needs no GPU; `prt.device` requires the HIP library and a GPU and raises otherwise.
"""
from . import host, scenes  # noqa: F401

__all__ = ["host", "scenes"]
