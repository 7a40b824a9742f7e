#!/usr/bin/env python3
"""A/B timing of kernel variants in ONE process (interleaved rounds, §5.4 rule 24 of the HIP guide).
usage: python tools/ab.py [--scene dragon] [--W 1920 --H 1080] [--rounds 5] [--frames 5] variant...
variant = "<kernel>[:ENV=VAL,ENV=VAL]", e.g. fast wavefront wavefront:PRT_REFILL_BELOW=16 strict
Prints median/min kernel ms per variant and Mrays/s (rays from the kernel counters)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-ray-tracer_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="dragon")
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--reupload", action="store_true", help="rebuild the scene per variant (knobs read at upload)")
    ap.add_argument("--world", type=int, default=1, help="render rank --rank's cyclic rows of a --world split")
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--batch", type=int, default=1, help="frames per launch (rt_render_frames); times are per frame")
    ap.add_argument("--orbit", type=float, default=0.0,
                    help="batch frames from a camera path: frame i's camera moved by i * ORBIT along x "
                         "(0: the reference's fixed camera)")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import torch
    from prt import device, host
    s = host.Scene.named(a.scene).build_bvh(3)
    r = device.Renderer(0)
    r.upload(s)
    cam = host.camera(a.W, a.H)
    cams = []
    for i in range(a.batch):
        c = host.camera(a.W, a.H)
        for v in (c.pos, c.ul):
            v.x += i * a.orbit
        cams.append(c)
    from prt.dist import cyclic_rows
    rows = cyclic_rows(a.H, a.rank, a.world)
    rgb = torch.empty((a.batch, rows[2], a.W, 3), dtype=torch.float32, device="cuda")
    res = {v: [] for v in a.variants}
    rays = {}
    pixels = {}

    base_env = {k: v for k, v in os.environ.items() if k.startswith("PRT_")}  # the caller's knobs persist

    def setenv(v):
        parts = v.split(":")
        for k in [k for k in os.environ if k.startswith("PRT_") and k not in base_env]:
            os.environ.pop(k)
        for k, val in base_env.items():
            os.environ[k] = val
        if len(parts) > 1:
            for kv in parts[1].split(","):
                k, val = kv.split("=")
                os.environ[k] = val
        return parts[0]

    ref, same = None, {}
    for rnd in range(a.rounds + 1):
        for v in a.variants:
            kern = setenv(v)
            if a.reupload:
                r.upload(s)
            for _ in range(a.frames):
                r.render_frames(cams, a.W, a.H, rows=rows, kernel=kern, rgb=rgb)
            ts = [t / a.batch for t in r.kernel_times(a.frames)]
            if rnd > 0:  # round 0 = warm-up
                res[v] += ts
            st = r.stats()
            rays[v] = st["rays"] // a.batch
            pixels[v] = st["pixels"] // a.batch
            if rnd == 0:  # every variant must render the first variant's frame bit for bit
                frame = rgb.view(torch.int32).clone()
                if ref is None:
                    ref = frame
                else:
                    same[v] = bool(torch.equal(frame, ref))
    out = {}
    for v in a.variants:
        t = sorted(res[v])
        med = t[len(t) // 2]
        out[v] = {"median_ms": med, "min_ms": t[0], "Mrays_s": rays[v] / med / 1e3, "rays": rays[v],
                  "bit_exact_vs_first": same.get(v, True)}
        print(f"{v:40s} median {med:8.3f} ms  min {t[0]:8.3f} ms  {rays[v] / med / 1e3:9.1f} Mrays/s  rays {rays[v]} "
              f"px {pixels[v]}  same={same.get(v, True)}")
    print(json.dumps({"scene": a.scene, "W": a.W, "H": a.H, "results": out}))


if __name__ == "__main__":
    main()
