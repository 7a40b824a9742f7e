#!/usr/bin/env python3
"""SIMD efficiency of the walks' triangle loops (a PRT_DIAG_TRI build, PRT_LIB_DIR=<its dir>): wave iterations of
the closest / shadow triangle loops against the lane tests they ran, per variant, on one 20-frame batch.
usage: PRT_LIB_DIR=ab_diag python tools/diag_tri.py [--scene dragon] variants..."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "parallel-ray-tracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="dragon")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import torch
    from prt import device, host
    s = host.Scene.named(a.scene).build_bvh(3)
    W, H = 1920, 1080
    cams = [host.camera(W, H) for _ in range(a.frames)]
    for v in a.variants:
        r = device.Renderer(0, counters=True)
        r.upload(s)
        px = torch.empty((a.frames, H, W), dtype=torch.int32, device="cuda")
        r.render_frames(cams, W, H, bgra=px, kernel="fast", variant=v)
        r.sync()
        st = r.stats()
        r.close()
        ws, wsh = st["wave_steps"], st["shadow_wave_steps"]
        q1, q2 = st["steps_lanes_16"], st["steps_lanes_32"]
        print(f"{a.scene:10s} {v:9s} wave steps {ws} (shadow {wsh})  closest tri: {st['ch_tri']} lane tests in {q1} "
              f"wave iterations (eff {st['ch_tri'] / max(1, 64 * q1):.3f}, {q1 / max(1, ws - wsh):.2f} per step)  "
              f"shadow tri: {st['sh_tri']} in {q2} (eff {st['sh_tri'] / max(1, 64 * q2):.3f}, "
              f"{q2 / max(1, wsh):.2f} per step)", flush=True)


if __name__ == "__main__":
    main()
