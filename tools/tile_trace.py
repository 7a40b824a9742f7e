#!/usr/bin/env python3
"""Tile timeline of one k_persist frame (PRT_TILE_TRACE diagnostics): launch ramp, per-wave busy time,
tail, and the spread of tile costs. usage: python tools/tile_trace.py [--scene dragon] [--W 1920 --H 1080]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-ray-tracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="dragon")
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--out", default=None)
    ap.add_argument("--counters", action="store_true", help="COUNT kernel: per-tile wave steps and node visits")
    ap.add_argument("--world", type=int, default=1, help="render rank --rank's cyclic rows of a --world split")
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--variant", default="auto", help="persist (default rule under a trace) or relay (k_relay's trace: "
                    "per tile the path wave's steps and the light waves' steps in place of node visits)")
    a = ap.parse_args()
    import torch
    from prt import device, host
    s = host.Scene.named(a.scene).build_bvh(3)
    r = device.Renderer(0, counters=a.counters)
    r.upload(s)
    cam = host.camera(a.W, a.H)
    from prt.dist import cyclic_rows
    rows = cyclic_rows(a.H, a.rank, a.world)
    rgb = torch.empty((rows[2], a.W, 3), dtype=torch.float32, device="cuda")
    for _ in range(5):
        r.render(cam, a.W, a.H, rows=rows, rgb=rgb, kernel=a.variant)
    r.sync()
    a.out = a.out or os.path.join(ROOT, "gpurun_out", f"tile_trace_{a.scene}.bin")
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    os.environ["PRT_TILE_TRACE"] = a.out
    r.render(cam, a.W, a.H, rows=rows, rgb=rgb, kernel=a.variant)
    r.sync()
    del os.environ["PRT_TILE_TRACE"]
    ms = r.kernel_times(1)[0]
    tr = np.fromfile(a.out, dtype=np.uint64).reshape(-1, 4).astype(np.int64)
    t0 = tr[:, 0].min()
    b, e = (tr[:, 0] - t0) * 10e-3, (tr[:, 1] - t0) * 10e-3  # 100 MHz ticks -> us
    w, fb = tr[:, 2] & 0xFFFFFFFF, tr[:, 2] >> 32
    ws, nv = tr[:, 3] & 0xFFFFFFFF, tr[:, 3] >> 32
    span = e.max()
    dur = e - b
    waves = np.unique(w)
    first = np.array([b[w == x].min() for x in waves])
    last = np.array([e[w == x].max() for x in waves])
    busy = np.array([dur[w == x].sum() for x in waves])
    # k_coop<4> and k_fan<4> (2-3 lights) deal 4x4 tiles
    tw, tht = (8, 8)  # (PRT_TILE_TRACE records the 8x8 tiles of k_persist, the configuration it forces)
    tx = (a.W + tw - 1) // tw
    rows = dur.reshape(-1, tx).mean(1) if len(dur) % tx == 0 else None
    res = {
        "kernel_ms_event": ms, "tile_span_us": float(span), "tiles": int(len(tr)), "waves": int(len(waves)),
        "tiles_per_wave": float(len(tr) / len(waves)),
        "wave_first_start_us_p50_p99_max": [float(np.percentile(first, 50)), float(np.percentile(first, 99)),
                                            float(first.max())],
        "wave_last_end_us_min_p10_p50": [float(last.min()), float(np.percentile(last, 10)),
                                         float(np.percentile(last, 50))],
        "busy_fraction_of_span": float(busy.sum() / (len(waves) * span)),
        "tile_us_mean_p50_p90_p99_max": [float(dur.mean()), float(np.percentile(dur, 50)),
                                         float(np.percentile(dur, 90)), float(np.percentile(dur, 99)),
                                         float(dur.max())],
        "tail_us_after_first_idle_wave": float(span - last.min()),
    }
    top = np.argsort(-dur)[:12]
    res["slowest_tiles"] = [{"x": int(i % tx) * tw, "y_compact": int(i // tx) * tht, "us": round(float(dur[i]), 1),
                             "fallback_rays": int(fb[i]), "start_us": round(float(b[i]), 1),
                             "wave_steps": int(ws[i]), "lane_node_visits": int(nv[i])} for i in top]
    if a.counters:
        m = ws > 0
        res["us_per_wave_step_all_tiles"] = float(dur[m].sum() / ws[m].sum())
        res["us_per_wave_step_slowest_1pct"] = float(dur[np.argsort(-dur)[:len(dur) // 100]].sum()
                                                     / ws[np.argsort(-dur)[:len(dur) // 100]].sum())
        res["simd_eff_all"] = float(nv.sum() / (64 * ws.sum()))
        res["wave_steps_p50_p99_max"] = [float(np.percentile(ws, 50)), float(np.percentile(ws, 99)), float(ws.max())]
    res["tiles_with_fallbacks"] = int((fb > 0).sum())
    res["mean_us_tiles_with_without_fallbacks"] = [float(dur[fb > 0].mean()) if (fb > 0).any() else None,
                                                  float(dur[fb == 0].mean())]
    if rows is not None:
        res["tile_row_mean_us_every_10th_row"] = [round(float(x), 1) for x in rows[::10]]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
