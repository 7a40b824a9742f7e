"""Single-frame kernel times with a fixed camera vs a camera moved every frame (the bench's walkthrough step), one
kernel per run, no hybrid rule: does a moving camera itself cost time? usage: tools/walk_probe.py [scene] [variants]"""
import sys
import torch
sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "parallel-ray-tracer_amd"))
from prt import device, host


def cam_at(W, H, i, step=0.02):
    c = host.camera(W, H)
    c.pos.x += i * step
    c.ul.x += i * step
    return c


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "dragon"
    variants = sys.argv[2:] or ["shdefer", "persist"]
    W, H = 1920, 1080
    s = host.Scene.named(scene).build_bvh(3)
    px = torch.empty((H, W), dtype=torch.int32, device="cuda")
    for v in variants:
        r = device.Renderer(0)
        r.upload(s)
        res = {}
        for mode in ("fixed", "walk", "fixed_mid", "alternate"):
            ts = []
            for i in range(40):
                k = {"fixed": 0, "walk": i, "fixed_mid": 20, "alternate": 20 + (i & 1)}[mode]
                r.render(cam_at(W, H, k), W, H, bgra=px, kernel=v)
                ts.append(r.sync())
            ts = sorted(ts[8:])
            res[mode] = ts[len(ts) // 2]
        r.close()
        print(scene, v, " ".join(f"{m} {t:.3f}" for m, t in res.items()), flush=True)


def stale(scene):
    """the default rule settled on one camera (its lists measured there), then frames of cameras d walk steps away:
    how fast the rule's per-tile knowledge goes stale (the lists refresh only every 64 frames of a decided shape)"""
    W, H = 1920, 1080
    s = host.Scene.named(scene).build_bvh(3)
    px = torch.empty((H, W), dtype=torch.int32, device="cuda")
    r = device.Renderer(0)
    r.upload(s)
    n = 0
    while True:
        r.render(cam_at(W, H, 20), W, H, bgra=px)
        r.sync()
        n += 1
        if r.launch_info()["settled"] or n > 60:
            break
    out = []
    for d in (0, 1, 2, 4, 8, 16):
        ts = []
        for _ in range(3):
            r.render(cam_at(W, H, 20 + d), W, H, bgra=px)
            ts.append(r.sync())
        out.append(f"d{d} {sorted(ts)[1]:.3f}")
    info = r.launch_info()
    r.close()
    print(scene, "stale:", " ".join(out), info, flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "stale":
        stale(sys.argv[1])
        sys.exit(0)
    main()
