"""The C-ABI libraries load and export every symbol include/*.h declares (no GPU compute here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "parallel-ray-tracer_amd", "lib")


def declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(rth?_\w+)\s*\(", src, flags=re.M)))


def exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(LIB, lib)], capture_output=True, text=True,
                         check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


@pytest.mark.parametrize("header,lib", [("rt_host.h", "librt_host.so"), ("rt_hip.h", "librt_hip.so")])
def test_every_declared_symbol_is_exported(header, lib):
    names = declared(header)
    assert len(names) >= 8
    missing = [n for n in names if n not in exported(lib)]
    assert not missing, missing
    L = ctypes.CDLL(os.path.join(LIB, lib))
    for n in names:
        getattr(L, n)


def test_hip_library_loads_without_gpu_and_reports_no_device():
    L = ctypes.CDLL(os.path.join(LIB, "librt_hip.so"))
    L.rt_version.restype = ctypes.c_char_p
    assert b"gfx950" in L.rt_version()
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    ctx = ctypes.c_void_p()
    assert L.rt_create(None, ctypes.byref(ctx)) == -6  # RT_E_NODEVICE, no exit()


def test_code_object_targets_gfx950():
    data = open(os.path.join(LIB, "librt_hip.so"), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in data


def test_ctypes_mirrors_match_the_c_layouts(tmp_path):
    """prt/_lib.py and prt/device.py mirror the C structs field by field: sizes and offsets from the C
    compiler itself (gcc on include/*.h)"""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "parallel-ray-tracer_amd"))
    from prt import _lib
    Outputs = __import__("prt.device", fromlist=["Outputs"]).Outputs if _lib_has_hip() else None
    structs = {"rt_opts": _lib.Opts, "rt_scene": _lib.SceneDesc, "rt_frame": _lib.Frame, "rt_stats": _lib.Stats,
               "rt_camera": _lib.Camera, "rt_triangle": _lib.Triangle, "rt_bvh_node": _lib.BvhNode,
               "rt_light": _lib.Light, "rth_rng": _lib.Rng, "rth_bvh_stats": _lib.BvhStats,
               "rth_wbvh_info": _lib.WbvhInfo, "rt_scene_info": _lib.SceneInfo, "rt_launch_info": _lib.LaunchInfo,
               "rt_comm_info": _lib.CommInfo}
    if Outputs is not None:
        structs["rt_outputs"] = Outputs
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "rt_hip.h"', '#include "rt_host.h"',
             "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "layouts.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layouts"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                        check=True).stdout.split("\n") if l)
    for cname, py in structs.items():
        assert int(got[cname]) == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(py, f).offset, (cname, f)


def _lib_has_hip():
    return os.path.exists(os.path.join(LIB, "librt_hip.so"))
