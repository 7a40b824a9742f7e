"""The reference-side binding of INTEGRATION.md §1, compiled and linked (no GPU needed, nothing is run).

INTEGRATION.md §1 is the patch a maintainer applies to the reference's cpu/src/main.c: the prelude
(rt_hip.h, the BVH globals of bvh.c:16-18, gpu_init = load_to_gpu) goes to file scope, gpu_init() is
called after bvh_build (main.c:138), and its render_frame replaces main.c:214-226. This test applies
exactly that patch — the C text is taken from the INTEGRATION.md code block itself, so the document cannot
drift from what compiles — to a temporary copy of main.c, builds every cpu/src/*.c the way cpu/makefile
does (gcc, -Iinclude), and links the result with librt_hip.so / librt_host.so. The reference sources are
read where they lie under /root/reference (the test skips when that tree is absent, e.g. on the GPU box);
nothing of them is kept in the repository.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/cpu"
LIB = os.path.join(ROOT, "parallel-ray-tracer_amd", "lib")

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")), reason="reference tree absent")


def integration_snippet():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = doc.split("## 1.", 1)[1].split("## 2.", 1)[0]
    code = re.search(r"```c\n(.*?)```", sec, re.S).group(1)
    cut = code.index("void render_frame(void)")
    return code[:cut], code[cut:]


def patched_main(prelude, render):
    src = open(os.path.join(REF, "src", "main.c")).read()
    # main.c:214-226: the reference's render_frame definition, up to its closing brace at column 0
    m = re.search(r"\nvoid render_frame\(\)\s*\{.*?\n\}\n", src, re.S)
    assert m, "render_frame definition not found in main.c"
    src = src[:m.start()] + "\n" + render + src[m.end():]
    # the prelude at file scope, after main.c's forward declarations (main.c:44-45)
    anchor = "vec_t render_pixel(const vec_t* start, const vec_t* inc_x, const vec_t* inc_y, int x, int y);\n"
    assert anchor in src
    src = src.replace(anchor, anchor + prelude, 1)
    # gpu_init() right after the BVH is built (main.c:138)
    call = "bvh_build(triangles, triangles_len);\n"
    assert call in src
    return src.replace(call, call + "    gpu_init();\n", 1)


def test_integration_render_frame_compiles_and_links(tmp_path):
    if not os.path.exists(os.path.join(LIB, "librt_hip.so")):
        pytest.skip("librt_hip.so not built (make hip)")
    prelude, render = integration_snippet()
    assert "rt_render(" in render and "rt_download(" in render and "rt_upload_scene(" in prelude
    src = tmp_path / "src"
    src.mkdir()
    for f in os.listdir(os.path.join(REF, "src")):
        if f.endswith(".c") and f != "main.c":
            shutil.copy(os.path.join(REF, "src", f), src / f)
    (src / "main.c").write_text(patched_main(prelude, render))
    exe = tmp_path / "raytracer_gpu"
    cmd = ["gcc", "-std=gnu11", "-O2", "-Wall", "-Werror=implicit-function-declaration",
           "-Werror=incompatible-pointer-types", "-I" + os.path.join(REF, "include"), "-I" + os.path.join(ROOT, "include")]
    cmd += sorted(str(p) for p in src.glob("*.c"))
    cmd += ["-o", str(exe), "-L" + LIB, "-lrt_hip", "-lrt_host", "-Wl,-rpath," + LIB, "-Wl,-rpath,/opt/rocm/lib",
            "-Wl,-rpath-link,/opt/rocm/lib", "-lm", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    nm = subprocess.run(["nm", "-u", str(exe)], capture_output=True, text=True, check=True).stdout
    for sym in ("rt_create", "rt_upload_scene", "rt_render", "rt_download", "rt_last_error"):
        assert re.search(r"\b" + sym + r"\b", nm), sym  # bound to librt_hip.so, resolved at load time
