"""Treelet restructuring of the GPU-built binary BVH (rt_treelet.hpp), compiled with g++ and run on the CPU: random
trees over random boxes stay BVHs of the same leaves (every leaf once, every internal box the union of its
children's, the root's box unchanged) and their SAH cost never rises. The GPU parity suite then renders through the
restructured trees bit-exactly (tests/test_gpu_build.py, every kernel test)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_treelet(tmp_path):
    exe = tmp_path / "treelet_test"
    src = os.path.join(ROOT, "tests", "c", "treelet_test.cpp")
    inc = os.path.join(ROOT, "parallel-ray-tracer_amd", "csrc", "hip")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-Wall", "-Wextra", "-Werror", "-I", inc, "-o", str(exe), src],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "treelet: ok" in r.stdout
