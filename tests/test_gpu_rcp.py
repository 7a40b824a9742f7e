"""The closest walks' fast reciprocal (rt_device.hpp rtd::rcp_ieee: v_rcp_f32 + one FMA correction, the division
above 2^125) equals the reference's correctly rounded `1.0f / det` (cpu/src/raytracer.c:35-59, hit_triangle) for
EVERY normal float of both signs: tools/rcp/rcp_exhaustive (built by the Makefile from the product header) checks
all 2^32 bit patterns on the GPU in well under a second. Without it the triangle tests would still be pinned by the
fixture tests, but only on the dets those scenes happen to produce.
"""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "rcp", "rcp_exhaustive")


def test_rcp_ieee_is_ieee_division_for_every_normal_float():
    assert os.path.exists(BIN), "tools/rcp/rcp_exhaustive missing: run `make` (build() does)"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "rcp_ieee (product) mismatches 0 " in r.stdout, r.stdout
    # the bare rcp + FMA differs only where the result is below 2^-126 (exponent fields 253, 254), which is why
    # rcp_ieee divides above 2^125
    fields = {int(l.split()[2][:-1]) for l in r.stdout.splitlines() if l.strip().startswith("exponent field")}
    assert fields <= {253, 254}, r.stdout
