"""prt.device's checks of the output tensors handed to the kernels (no GPU needed: every refusal happens
before any device call). The kernels write frames * n_rows * width * channels elements through raw
pointers, so a tensor that is too small, of the wrong dtype, strided or on another device must raise
RtError instead of becoming an out-of-bounds device write."""
import pytest
import torch

from prt import device


def test_output_tensors_are_checked_before_any_launch():
    f32, i32 = (torch.float32,), (torch.int32,)
    ok = torch.zeros(4 * 3, dtype=torch.float32)
    with pytest.raises(device.RtError, match="elements"):  # undersized: 11 < 12
        device._ptr(torch.zeros(11, dtype=torch.float32), "rgb", 12, f32, 0)
    with pytest.raises(device.RtError, match="dtype"):  # an rgb buffer passed as bgra
        device._ptr(ok, "bgra", 4, i32, 0)
    with pytest.raises(device.RtError, match="contiguous"):
        device._ptr(torch.zeros(8, 3, dtype=torch.float32)[::2], "rgb", 12, f32, 0)
    with pytest.raises(device.RtError, match="expected cuda:0"):  # a host tensor
        device._ptr(ok, "rgb", 12, f32, 0)
    with pytest.raises(device.RtError, match="torch tensor"):
        device._ptr([0.0] * 12, "rgb", 12, f32, 0)
    assert device._ptr(None, "rgb", 12, f32, 0) is None
    assert device._ptr(1234, "rgb", 12, f32, 0) == 1234  # a raw device pointer is the caller's responsibility


def test_variant_and_dealing_names_match_the_header():
    """prt.device's names for rt_frame.variant / rt_frame.dealing follow include/rt_hip.h's enums"""
    import os
    import re
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "rt_hip.h")).read()
    enum = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"RT_VARIANT_(\w+) = (\d+)", hdr)}
    assert enum == device.VARIANTS
    deal = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"RT_DEAL_(\w+) = (\d+)", hdr)}
    assert deal == device.DEALING
