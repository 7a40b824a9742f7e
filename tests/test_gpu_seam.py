"""The drop-in seam under the reference's own loop (cpu/src/main.c:171-185, gpu/src/main.cu:110-115: one render_frame
per iteration) with the library's default launch rule, on a MOVING camera.

The rule for single 1-spp frames (RT_VARIANT_HYBRID) measures and tries its candidates on the first frames of a frame
shape; the rule for frame batches (PERSIST4 vs the shadow pool) does the same on the first launches. Both are keyed by
the shape, not the camera, and read their measurements by event queries: a walkthrough that moves the camera every
frame enqueues frame after frame without the host waiting for the GPU. Every frame is bit-exact to the strict
(reference-order) kernel whatever configuration the rule is trying or has chosen."""
import time

import numpy as np
import pytest
import torch

from prt import host

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from prt import device
    assert device.device_count() > 0
    return device


def walk(W, H, i, step=0.02):
    c = host.camera(W, H)
    c.pos.x += i * step
    c.ul.x += i * step
    c.pos.z += 0.5 * i * step
    c.ul.z += 0.5 * i * step
    return c


def same_bits(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.int32), np.asarray(b, np.float32).view(np.int32))


def strict_frames(dev, s, cams, W, H):
    r = dev.Renderer(0)
    r.upload(s)
    out = []
    for c in cams:
        rgb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        hit = torch.empty((H, W), dtype=torch.int32, device="cuda")
        r.render(c, W, H, kernel="strict", rgb=rgb, hit=hit)
        r.sync()
        out.append((rgb.cpu().numpy(), hit.cpu().numpy()))
    r.close()
    return out


@pytest.mark.parametrize("name", ["dragon", "car_boxed"])
def test_moving_camera_walkthrough_enqueues_without_waits(dev, name):
    """30 rt_render calls with the default rule and a camera moved every frame, enqueued back to back: the host's
    enqueue time stays well below the frames' GPU time (no call waits for an earlier frame), and every frame equals
    the strict kernel's frame of its camera"""
    W, H, n = 1920, 1080, 30
    s = host.Scene.named(name).build_bvh(3)
    cams = [walk(W, H, i) for i in range(n)]
    r = dev.Renderer(0)
    r.upload(s)
    # (filled with values no render writes: a tile the device-built lists left out would show)
    rgb = torch.full((n, H, W, 3), -1.0, dtype=torch.float32, device="cuda")
    hit = torch.full((n, H, W), -7, dtype=torch.int32, device="cuda")
    r.render(cams[0], W, H, rgb=rgb[0], hit=hit[0])  # (first call of the shape: its buffers and events)
    r.sync()
    t0 = time.perf_counter()
    for i in range(n):
        r.render(cams[i], W, H, rgb=rgb[i], hit=hit[i])
    enqueue_ms = (time.perf_counter() - t0) * 1e3
    r.sync()
    gpu_ms = sum(r.kernel_times(n))
    r.close()
    assert enqueue_ms < 0.5 * gpu_ms, (enqueue_ms, gpu_ms)
    ref = strict_frames(dev, s, cams, W, H)
    for i in range(n):
        np.testing.assert_array_equal(hit[i].cpu().numpy(), ref[i][1], err_msg=str(i))
        assert same_bits(rgb[i].cpu().numpy(), ref[i][0]), i


def test_single_frame_rule_settles_on_a_moving_camera(dev):
    """the single-frame rule keyed by shape: with a sync per frame (the reference's loop) it settles within its
    measuring frame + 4 trial frames per candidate (+ the frames that find the last trial still running), on a camera that
    never repeats, and stays settled; once settled every frame deals its tiles by the previous frame's per-tile times,
    its lists built on the device (rt_launch_info.build: feedback), so no measuring frame refreshes them any more (the
    hybrid candidates' trial frames build theirs the same way);
    rt_get_launch_info names what each frame ran"""
    W, H = 640, 360
    s = host.Scene.named("dragon").build_bvh(3)
    r = dev.Renderer(0)
    r.upload(s)
    px = torch.empty((H, W), dtype=torch.int32, device="cuda")
    infos = []
    for i in range(100):
        r.render(walk(W, H, i), W, H, bgra=px)
        r.sync()
        infos.append(r.launch_info())
    r.close()
    first = next(i for i, x in enumerate(infos) if x["settled"])
    assert first <= 1 + 4 * 5 + 2, (first, infos[:first + 1])
    assert len(infos) - first > 70
    assert all(x["settled"] and not x["trial"] for x in infos[first:]), infos
    assert not any(x["refresh"] for x in infos)
    # the first settled frame may still run the rule's host-built lists; every later one the device-built ones
    assert all("feedback" in x["build_bits"] for x in infos[first + 1:]), infos[first:first + 4]
    # the trials of hybrid candidates run device-built lists too (a candidate tried later is not priced with older
    # lists than one tried first); the measuring frame and the whole-frame kernels' trials never do
    assert "feedback" not in infos[0]["build_bits"]
    assert all("feedback" not in x["build_bits"] for x in infos[:first] if x["variant"] != "hybrid"), infos[:first]
    assert infos[0]["trial"] == 1 and infos[0]["variant"] == "persist"  # the measuring frame
    assert infos[-1]["variant"] in ("persist", "shpool", "shdefer", "hybrid")


@pytest.mark.parametrize("name", ["dragon", "car_boxed"])
def test_frame_batches_with_changing_cameras(dev, name):
    """12 rt_render_frames batches of 4 frames, every batch a new camera set (more sets than the pinned camera
    slots, so slots are reused), enqueued back to back under the default rule (its PERSIST4 / shadow-pool trials
    included): every frame equals its single-frame render"""
    W, H, n, nb = 160, 90, 4, 12
    s = host.Scene.named(name).build_bvh(3)
    r = dev.Renderer(0)
    r.upload(s)
    outs = [torch.empty((n, H, W, 3), dtype=torch.float32, device="cuda") for _ in range(nb)]
    sets = [[walk(W, H, 4 * b + i, 0.05) for i in range(n)] for b in range(nb)]
    for b in range(nb):
        r.render_frames(sets[b], W, H, rgb=outs[b])
    r.sync()
    r.close()
    ref = strict_frames(dev, s, [c for cs in sets for c in cs], W, H)
    for b in range(nb):
        got = outs[b].cpu().numpy()
        for i in range(n):
            assert same_bits(got[i], ref[4 * b + i][0]), (b, i)


@pytest.mark.parametrize("name", ["dragon", "two_cars"])
def test_batch_rule_settles_on_the_faster_kernel(dev, name):
    """frame batches under the default rule: PERSIST4 and the shadow pool (the all-levels pool where its path buffer
    fits, as on dragon) are tried three times each on the first launches of the shape, then the faster renders;
    launch_info reports the trials and the choice; every launch's frames are the same bits"""
    W, H, n = 320, 180, 8
    s = host.Scene.named(name).build_bvh(3)
    cams = [walk(W, H, i) for i in range(n)]
    r = dev.Renderer(0)
    r.upload(s)
    ref = None
    seen = []
    for k in range(10):
        px = torch.empty((n, H, W), dtype=torch.int32, device="cuda")
        r.render_frames(cams, W, H, bgra=px)
        r.sync()
        seen.append(r.launch_info())
        got = px.cpu().numpy()
        if ref is None:
            ref = got
        np.testing.assert_array_equal(got, ref, err_msg=str(k))
    r.close()
    tried = [x["variant"] for x in seen[:6]]
    pool = "shdefer" if name == "dragon" else tried[1]
    assert tried == ["persist4", pool] * 3 and pool in ("shpool", "shdefer") and all(x["trial"] for x in seen[:6]), seen
    assert seen[6]["settled"] and all(x["settled"] and x["variant"] == seen[6]["variant"] for x in seen[6:]), seen
