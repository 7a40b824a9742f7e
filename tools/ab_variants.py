#!/usr/bin/env python3
"""Same-box A/B of the fast kernel's launch configurations (rt_frame.variant): bit-exactness against the
first variant, ray counts, and ms per frame (single frames and frame batches, HIP-event kernel times).

usage: python tools/ab_variants.py [--scene dragon] [--frames 16] [--rounds 3] persist persist4 pool pool:regroup=8 ...
       persist4:up_accel=host persist4:up_ploc_radius=32 (up_*: upload options: the fast walk's BVH)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-ray-tracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="dragon")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--spp", type=int, default=1)
    ap.add_argument("--accel", default="auto")
    ap.add_argument("--ploc-radius", type=int, default=0)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import numpy as np
    import torch
    from prt import device, host
    s = host.Scene.named(a.scene).build_bvh(3)
    W, H, F = a.width, a.height, a.frames
    cam = host.camera(W, H)
    ref = None
    for spec in a.variants:
        name, _, opts = spec.partition(":")
        kw = {k: (int(v) if v.lstrip("-").isdigit() else v) for k, v in (o.split("=") for o in opts.split(",") if o)}
        kw_up = {k[3:]: v for k, v in kw.items() if k.startswith("up_")}  # e.g. persist4:up_ploc_radius=32
        kw = {k: v for k, v in kw.items() if not k.startswith("up_")}
        up = dict(accel=kw_up.pop("accel", a.accel), ploc_radius=kw_up.pop("ploc_radius", a.ploc_radius),
                  collapse_node_cost=float(kw_up.pop("cnode", 0)) / 10.0)  # up_cnode=15: c_node 1.5
        r = device.Renderer(0, counters=True)
        r.upload(s, **up)
        info = r.scene_info()
        rgb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        r.render(cam, W, H, kernel=name, rgb=rgb, spp=a.spp, **kw)
        st = r.stats()
        r.close()
        got = rgb.cpu().numpy()
        if ref is None:
            ref = (got, st)
        same = np.array_equal(got.view(np.int32), ref[0].view(np.int32))
        eff = (st["ch_inner"] + st["sh_inner"]) / max(1, 64 * st["wave_steps"])
        r = device.Renderer(0)
        r.upload(s, **up)
        bg = torch.empty((F, H, W), dtype=torch.int32, device="cuda")
        one, bat = [], []
        for _ in range(a.rounds):
            for _ in range(3):
                r.render(cam, W, H, kernel=name, bgra=bg[0], spp=a.spp, **kw)
            one.append(min(r.kernel_times(3)))
            for _ in range(3):
                r.render_frames([cam] * F, W, H, kernel=name, bgra=bg, spp=a.spp, **kw)
            bat.append(min(r.kernel_times(3)) / F)
        r.close()
        print(f"{a.scene:10s} {spec:24s} bit-exact {same!s:5s} rays {st['rays']} (ref {ref[1]['rays']}) "
              f"simd-eff {eff:.3f} wave-steps {st['wave_steps']}  single {min(one):.3f} ms  "
              f"batch{F} {min(bat):.3f} ms/frame  accel {info['accel_built']} wide {info['wide_nodes']}/{info['wide_depth']} "
              f"build {info['build_ms']:.1f} ms", flush=True)


if __name__ == "__main__":
    main()
