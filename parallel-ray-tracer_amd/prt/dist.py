"""Multi-GPU framebuffer partition and gather.

Rows are dealt cyclically: rank r renders image rows y = r, r + N, r + 2N, ... (rt_frame row_offset = r,
row_stride = N). SURVEY §8e measured this at 7.83x (car_boxed) / 7.88x (car_only) of 8 GPUs against
5.0x / 2.7x for equal contiguous blocks: per-row cost varies a lot (sky rows vs car rows) and cyclic
dealing averages it out without a cost model. Every rank's compact block is padded to ceil(H/N) rows,
gathered to rank 0 with ONE collective (torch.distributed gather; backend "nccl" = RCCL over xGMI on
MI355X, "gloo" on CPU for tests) and un-interleaved on rank 0's device.
"""


def cyclic_rows(H, rank, world):
    """(row_offset, row_stride, n_rows) of this rank's rows."""
    if not (0 <= rank < world) or H <= 0:
        raise ValueError("bad rank/world/height")
    return rank, world, (H - rank + world - 1) // world


def padded_rows(H, world):
    return (H + world - 1) // world


class FrameGather:
    """Gather per-rank compact row blocks [padded_rows, W, C] into the full frame on rank 0."""

    def __init__(self, H, W, C, rank, world, dist, like):
        import torch
        self.H, self.W, self.rank, self.world, self.dist = H, W, rank, world, dist
        self.n_max = padded_rows(H, world)
        self.block = torch.zeros((self.n_max, W, C), dtype=like.dtype, device=like.device)
        self.frame = torch.zeros((H, W, C), dtype=like.dtype, device=like.device) if rank == 0 else None
        self.parts = [torch.empty_like(self.block) for _ in range(world)] if (rank == 0 and world > 1) else None

    def rows(self):
        return cyclic_rows(self.H, self.rank, self.world)

    def gather(self):
        """collective: every rank calls it after rendering into self.block"""
        if self.world == 1:
            self.frame.copy_(self.block)
            return self.frame
        self.dist.gather(self.block, self.parts if self.rank == 0 else None, dst=0)
        if self.rank == 0:
            for q in range(self.world):
                nq = cyclic_rows(self.H, q, self.world)[2]
                self.frame[q::self.world] = self.parts[q][:nq]
        return self.frame
