import sys, torch, numpy as np
sys.path.insert(0, "parallel-ray-tracer_amd"); sys.path.insert(0, ".")
from prt import device as dev, host
s = host.Scene.named("car_boxed").build_bvh(3)
W, H = 200, 113
for kind in ("rgb", "bgra"):
    r = dev.Renderer(0); r.upload(s)
    shp = (1, H, W) if kind == "bgra" else (1, H, W, 3)
    dt = torch.int32 if kind == "bgra" else torch.float32
    t = torch.empty(shp, dtype=dt, device="cuda")
    r.render_frames([host.camera(W, H)], W, H, **{kind: t}); r.sync()
    comm = dev.Comm([r], nranks=1, rank=0, uid=dev.comm_id())
    out = torch.zeros(shp, dtype=dt, device="cuda"); torch.cuda.synchronize()
    try:
        comm.gather(0, out)
        print(kind, "gather ok")
    except Exception as e:
        print(kind, "ERR", e)
    r.sync(); torch.cuda.synchronize()
    a = out.cpu().view(torch.int32).numpy(); b = t.cpu().view(torch.int32).numpy()
    print(kind, "equal", np.array_equal(a, b), "ff count", int((a == -1).sum()), "sample", a.reshape(-1)[:6], b.reshape(-1)[:6])
    print(comm.info())
    comm.close(); r.close()
