"""probe: can gloo gather CUDA tensors (two ranks on one GPU)? exercises prt.dist.FrameGather's CUDA path"""
import os, sys
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(rank, world, port):
    sys.path.insert(0, os.path.join(ROOT, "parallel-ray-tracer_amd"))
    from prt.dist import FrameGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    H, W = 36, 8
    g = FrameGather(H, W, 3, rank, world, dist, torch.empty(0, device="cuda"), frames=2, buffers=2)
    ro, rs, nr = g.rows()
    for b in range(2):
        for f in range(2):
            g.blocks[b][f, :nr] = torch.arange(nr, device="cuda", dtype=torch.float32)[:, None, None] * world + ro + 100 * f
        g.start(b)
    out = [g.finish(0), g.finish(1)]
    torch.cuda.synchronize()
    if rank == 0:
        for fr in out:
            for f in range(2):
                ok = torch.equal(fr[f, :, 0, 0].cpu(), torch.arange(H, dtype=torch.float32) + 100 * f)
                print("frame ok", ok, flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.start_processes(worker, args=(2, 29517), nprocs=2, join=True, start_method="spawn")
