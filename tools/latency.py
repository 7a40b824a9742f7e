#!/usr/bin/env python3
"""Single-frame latency as the reference's loop sees it (cpu/src/main.c:171-185, gpu/src/main.cu:110-115: one
render_frame() per iteration, each waited for): per launch configuration, `--iters` frames through rt_render,
each followed by rt_sync; median HIP-event kernel ms and median host wall ms per frame over the frames after the
library's rule has settled (rt_get_launch_info), bit-exactness of the last frame against the first configuration.
usage: python tools/latency.py [--scene dragon] [--iters 20] persist hybrid hybrid:hot_pct=50 ..."""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-ray-tracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="dragon")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--walk", type=float, default=0.0, help="camera moved by i * WALK along x in frame i (a walkthrough)")
    ap.add_argument("--frames", action="store_true", help="also print every settled frame's kernel ms")
    ap.add_argument("--start", type=int, default=0, help="walk: the first frame's camera index")
    ap.add_argument("--hold", action="store_true", help="walk: every frame at the --start camera (a fixed camera there)")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import numpy as np
    import torch
    from prt import device, host
    s = host.Scene.named(a.scene).build_bvh(3)
    W, H = a.width, a.height
    cam = host.camera(W, H)
    ref = None
    for spec in a.variants:
        name, _, opts = spec.partition(":")
        kw = {k: (int(v) if v.lstrip("-").isdigit() else v) for k, v in (o.split("=") for o in opts.split(",") if o)}
        r = device.Renderer(0)
        r.upload(s)
        rgb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        ks, ws, settled, info = [], [], None, {}
        for i in range(a.iters):
            t0 = time.perf_counter()
            c = cam
            if a.walk:
                c = host.camera(W, H)
                j = a.start + (0 if a.hold else i)
                c.pos.x += j * a.walk
                c.ul.x += j * a.walk
            r.render(c, W, H, kernel=name, rgb=rgb, **kw)
            ms = r.sync()
            info = r.launch_info()
            if info["settled"]:  # only the frames after the rule's measuring / trial frames
                settled = i if settled is None else settled
                ks.append(ms)
                ws.append((time.perf_counter() - t0) * 1e3)
        got = rgb.cpu().numpy()
        r.close()
        if ref is None:
            ref = got
        same = np.array_equal(got.view(np.int32), ref.view(np.int32))
        print(f"{a.scene:10s} {spec:22s} bit-exact {same!s:5s} kernel ms median {statistics.median(ks):.3f} "
              f"min {min(ks):.3f} max {max(ks):.3f} ({len(ks)} frames after settling at frame {settled})  wall ms median "
              f"{statistics.median(ws):.3f}  ran {info}", flush=True)
        if a.frames:
            print("   frames (settled, kernel ms):", " ".join(f"{k:.3f}" for k in ks), flush=True)


if __name__ == "__main__":
    main()
