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


def test_gather_output_tensor_is_checked():
    """rt_gather_to / rt_comm_gather's full-frame output: EVERY frame of the root's last render (frames x W x H),
    in that render's pixel format (rgb f32 x 3 or BGRA8 int32)"""
    class Root:  # the root Renderer's last render, as prt.device.Renderer keeps it
        _size, device, _frames, _words = (4, 2), 0, 1, 3

    with pytest.raises(device.RtError, match="elements"):
        device._gather_out(Root(), torch.zeros(4 * 2 * 3 - 1, dtype=torch.float32))
    with pytest.raises(device.RtError, match="dtype"):
        device._gather_out(Root(), torch.zeros(4 * 2 * 3, dtype=torch.int64))
    with pytest.raises(device.RtError, match="dtype"):  # an rgb render gathered into a BGRA8 tensor
        device._gather_out(Root(), torch.zeros(4 * 2 * 3, dtype=torch.int32))
    with pytest.raises(device.RtError, match="expected cuda:0"):
        device._gather_out(Root(), torch.zeros(4 * 2 * 3, dtype=torch.float32))

    class Batch(Root):  # a 16-frame BGRA8 batch: a one-frame tensor is refused
        _frames, _words = 16, 1

    with pytest.raises(device.RtError, match="elements"):
        device._gather_out(Batch(), torch.zeros(4 * 2, dtype=torch.int32))
    with pytest.raises(device.RtError, match="dtype"):
        device._gather_out(Batch(), torch.zeros(16 * 4 * 2, dtype=torch.float32))
    with pytest.raises(device.RtError, match="expected cuda:0"):
        device._gather_out(Batch(), torch.zeros(16 * 4 * 2, dtype=torch.int32))

    class Fresh:  # nothing rendered yet
        device = 0

    with pytest.raises(device.RtError, match="not rendered"):
        device._gather_out(Fresh(), torch.zeros(8, dtype=torch.int32))


def test_variant_and_dealing_names_match_the_header():
    """prt.device's names for rt_frame.variant / rt_frame.dealing follow include/rt_hip.h's enums"""
    import os
    import re
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "rt_hip.h")).read()
    enum = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"RT_VARIANT_(\w+) = (\d+)", hdr)}
    assert enum == device.VARIANTS
    deal = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"RT_DEAL_(\w+) = (\d+)", hdr)}
    assert deal == device.DEALING
