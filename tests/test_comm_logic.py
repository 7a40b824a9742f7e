"""The multi-process gather's host-side decisions (rt_comm_logic.hpp), compiled with g++ and run on the CPU: the
deadline-bounded wait over a stub stream that never completes (RT_E_TIMEOUT + one abort instead of a hang), the
ranks' exchange decision with one rank toggling its hit output (no collective mismatch), row-set checks.
No GPU: this is the CPU-side cover of verdict r4 item 6 (the first 8-GPU run must fail loudly, not hang)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_comm_logic(tmp_path):
    exe = tmp_path / "comm_logic_test"
    src = os.path.join(ROOT, "tests", "c", "comm_logic_test.cpp")
    inc = os.path.join(ROOT, "parallel-ray-tracer_amd", "csrc", "hip")
    subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-I", inc, "-o", str(exe), src,
                    "-pthread"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout
