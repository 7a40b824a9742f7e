import sys, os, numpy as np
sys.path.insert(0,'.'); sys.path.insert(0,'parallel-ray-tracer_amd')
import torch
from prt import host, device
from tests.oracle_bind import OracleScene
from tests.scenes import scene_paths
W,H=96,54; N=W*H
raw = open('dbg/dragon_ref_96x54.bin','rb').read()
refhit = np.frombuffer(raw[:4*N], np.int32).reshape(H,W)
s = host.Scene.named("dragon").build_bvh(3)
o = OracleScene.load(*scene_paths("dragon")); o.build_bvh(3)
port = o.render(W,H)
ob = OracleScene.load(*scene_paths("dragon")); ob.set_use_bvh(False); bf = ob.render(W,H)
for k in ("strict","fast"):
    r = device.Renderer(0, counters=True); r.upload(s)
    hit = torch.empty((H,W), dtype=torch.int32, device="cuda"); t = torch.empty((H,W), dtype=torch.float32, device="cuda")
    rgb = torch.empty((H,W,3), dtype=torch.float32, device="cuda")
    r.render(host.camera(W,H), W, H, kernel=k, rgb=rgb, hit=hit, t=t); r.sync()
    g = hit.cpu().numpy(); gt = t.cpu().numpy()
    print(k, "gpu vs port", (g!=port["hit"]).sum(), "gpu vs ref", (g!=refhit).sum(), "stats", r.stats())
    for (y,x) in np.argwhere(g!=port["hit"]):
        print("  ", y, x, "gpu", g[y,x], gt[y,x], "port", port["hit"][y,x], port["t"][y,x], "ref", refhit[y,x], "brute", bf["hit"][y,x])
# NaN semantics probe on the device
a = torch.tensor([float('nan'), 1.0, -float('inf'), 0.0], device="cuda")
b = torch.tensor([float('inf'), float('nan'), float('nan'), -0.0], device="cuda")
print("torch fmin", torch.fmin(a,b).cpu().tolist(), "fmax", torch.fmax(a,b).cpu().tolist())
