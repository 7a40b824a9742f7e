#!/usr/bin/env python3
"""Per camera of the bench's walkthrough path: the strict fallbacks (exact ties + degenerate directions) of a frame,
its wave steps, and the single-frame kernel ms of a fixed kernel (no rule) -- does a walk frame's cost follow its
fallbacks?  usage: python tools/walk_fallbacks.py [--scene dragon] [--first 20] [--last 40] [--variant shdefer]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-ray-tracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="dragon")
    ap.add_argument("--first", type=int, default=20)
    ap.add_argument("--last", type=int, default=40)
    ap.add_argument("--orbit", type=float, default=0.02)
    ap.add_argument("--variant", default="shdefer")
    a = ap.parse_args()
    import torch
    from prt import device, host
    s = host.Scene.named(a.scene).build_bvh(3)
    W, H = 1920, 1080
    rc = device.Renderer(0, counters=True)
    rc.upload(s)
    rt = device.Renderer(0)
    rt.upload(s)
    rgb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    for i in range(a.first, a.last + 1):
        c = host.camera(W, H)
        c.pos.x += i * a.orbit
        c.ul.x += i * a.orbit
        rc.render(c, W, H, kernel="fast", variant=a.variant, rgb=rgb)
        rc.sync()
        st = rc.stats()
        ms = []
        for _ in range(3):
            rt.render(c, W, H, kernel="fast", variant=a.variant, rgb=rgb)
            ms.append(rt.sync())
        print(f"camera {i:3d}  fallbacks {st['fallbacks']:7d}  wave_steps {st['wave_steps']:9d}  ch_inner {st['ch_inner']:10d}  "
              f"kernel ms {sorted(ms)[1]:.3f}", flush=True)
    rc.close()
    rt.close()


if __name__ == "__main__":
    main()
