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


def padded_rows(H, world, block=1):
    """rows of the largest rank block (every rank's block is padded to it for the gather)"""
    return max(rank_rows(H, q, world, block)[2] for q in range(world)) if block > 1 else (H + world - 1) // world


def rank_rows(H, rank, world, block=1):
    """rt_frame rows of rank `rank`: (row_offset, row_stride, n_rows, row_block). block = 1: cyclic rows
    (y = rank + k * world); block = B: blocks of B consecutive rows dealt cyclically (block j on rank
    j % world), so an 8x8 pixel tile of a rank's compact rows is an 8x8 tile of the image (B = 8) while
    the ranks' costs still average out over the ~H / (B * world) blocks each."""
    if block <= 1:
        return cyclic_rows(H, rank, world) + (1,)
    if not (0 <= rank < world) or H <= 0:
        raise ValueError("bad rank/world/height")
    nb = (H + block - 1) // block
    n = sum(min(block, H - j * block) for j in range(rank, nb, world))
    return rank * block, world * block, n, block


def image_rows(H, rank, world, block=1):
    """image row of each of rank `rank`'s compact rows (rt_frame: off + (k // B) * stride + k % B)"""
    off, stride, n, b = rank_rows(H, rank, world, block)
    return [off + (k // b) * stride + k % b for k in range(n)]


class FrameGather:
    """Gather per-rank compact row blocks [padded_rows, W, C] into the full frame on rank 0.

    frames > 1: a frame batch (rt_render_frames) — every rank's frames are compact ([frames, n_rows, W, C]
    with its OWN n_rows, as rt_render_frames writes them: frame f at f * n_rows * W), at the start of a
    block of frames * padded_rows rows (equal on every rank, as the collective needs) -> frames
    [frames, H, W, C], one collective for the whole batch. Render into target(i), not blocks[i].
    rotate (frame batches of row blocks): frame f of rank q renders the block residue (q + f) % world
    (rt_frame.frame_shift = block), so over a batch every rank renders every residue and the ranks' costs
    even out whatever the image's cost per residue; every rank then renders padded_rows compact rows per
    frame (rows past the image are skipped by the kernel) and rank 0 unpacks with one index copy. buffers > 1: ping-pong blocks, so that the
    gather of batch k (start(k % buffers), asynchronous on the collective's stream) overlaps the render of
    batch k + 1 into the other block; finish(i) makes the current stream wait for it and un-interleaves.
    World 1: the block IS the frame (no collective, no copy). On a GPU, rank 0 un-interleaves on a side
    stream, so the copy (F frames of H x W x C) does not delay rank 0's next render — which every rank's
    next gather would wait for."""

    def __init__(self, H, W, C, rank, world, dist, like, frames=1, buffers=1, block=1, rotate=False):
        import torch
        self.H, self.W, self.C, self.rank, self.world, self.dist = H, W, C, rank, world, dist
        self.frames = frames
        self.bk = max(1, block)
        self.rotate = bool(rotate) and frames > 1 and self.bk > 1 and world > 1
        self._flat = None  # rotate: (source rows, frame rows) of the one index copy
        self.n_max = padded_rows(H, world, self.bk)
        shape = (self.n_max, W, C) if frames == 1 else (frames, self.n_max, W, C)
        self.blocks = [torch.zeros(shape, dtype=like.dtype, device=like.device) for _ in range(buffers)]
        self.block = self.blocks[0]
        many = rank == 0 and world > 1
        fshape = (H, W, C) if frames == 1 else (frames, H, W, C)
        self.frame = torch.zeros(fshape, dtype=like.dtype, device=like.device) if many else None
        self.parts = [torch.empty((world,) + shape, dtype=like.dtype, device=like.device) for _ in range(buffers)] \
            if many else None
        self._work = [None] * buffers
        cuda = like.device.type == "cuda" and many
        self._side = torch.cuda.Stream(device=like.device) if cuda else None
        self._copied = [None] * buffers  # side-stream event: parts[i] read by the un-interleave
        self._idx = None
        if many and self.bk > 1 and H % (world * self.bk) != 0:  # general block layout: index copies
            self._idx = [torch.tensor(image_rows(H, q, world, self.bk), dtype=torch.long, device=like.device)
                         for q in range(world)]

    def target(self, i=0):
        """blocks[i] as this rank's render output: [frames, n_rows, W, C] compact frames (or [n_rows, W, C])"""
        n = self.n_max if self.rotate else rank_rows(self.H, self.rank, self.world, self.bk)[2]
        b = self.blocks[i]
        if self.frames == 1:
            return b[:n]
        return b.view(-1)[:self.frames * n * self.W * self.C].view(self.frames, n, self.W, self.C)

    def _part(self, P, q):
        """rank q's compact frames inside its gathered block P[q]: [frames, n_q, W, C]"""
        n = rank_rows(self.H, q, self.world, self.bk)[2]
        return P[q].reshape(-1)[:P.shape[1] * n * self.W * self.C].view(P.shape[1], n, self.W, self.C)

    def rows(self):
        """this rank's rt_frame rows: (offset, stride, n) for single rows, (offset, stride, n, block)"""
        r = rank_rows(self.H, self.rank, self.world, self.bk)
        if self.rotate:  # (offset, stride, padded rows, block, frame_shift = block)
            return r[0], r[1], self.n_max, self.bk, self.bk
        return r if self.bk > 1 else r[:3]

    def start(self, i=0):
        """collective (every rank): begin gathering blocks[i] to rank 0"""
        if self.world == 1:
            return
        if self._copied[i] is not None:  # parts[i] is still being read by the last un-interleave
            import torch
            torch.cuda.current_stream().wait_event(self._copied[i])
            self._copied[i] = None
        dst = list(self.parts[i]) if self.rank == 0 else None
        self._work[i] = self.dist.gather(self.blocks[i], dst, dst=0, async_op=True)

    def pending(self, i=0):
        return self._work[i] is not None

    def finish(self, i=0):
        """wait for start(i)'s gather; rank 0: un-interleave it into self.frame and return it"""
        if self.world == 1:
            return self.blocks[i]
        w, self._work[i] = self._work[i], None
        if w is not None:
            w.wait()  # the current stream waits for the gather (blocks[i] may be rendered into again)
        if self.rank != 0:
            return None
        if self._side is not None:
            import torch
            self._side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self._side):
                self._uninterleave(i)
            self._copied[i] = self._side.record_event()
        else:
            self._uninterleave(i)
        return self.frame

    def _uninterleave(self, i):
        if self.rotate:
            self._unrotate(i)
            return
        P = self.parts[i]
        frame = self.frame
        if self.frames == 1:
            P, frame = P.unsqueeze(1), frame.unsqueeze(0)
        F, n = P.shape[1], self.n_max
        if self.bk > 1:
            if self._idx is None:  # one copy: frame row (m * world + q) * B + r <- rank q's row m * B + r
                M, B = self.H // (self.world * self.bk), self.bk
                frame.view(F, M, self.world, B, self.W, self.C).copy_(
                    P.view(self.world, F, M, B, self.W, self.C).permute(1, 2, 0, 3, 4, 5))
            else:
                for q in range(self.world):
                    frame.index_copy_(1, self._idx[q], self._part(P, q))
        elif self.H % self.world == 0:  # one copy: frame row k * world + q <- rank q's compact row k
            frame.view(F, n, self.world, self.W, self.C).copy_(P.permute(1, 2, 0, 3, 4))
        else:
            for q in range(self.world):
                frame[:, q::self.world] = self._part(P, q)

    def _unrotate(self, i):
        import torch
        if self._flat is None:
            N, B, F, n = self.world, self.bk, self.frames, self.n_max
            src, dst = [], []
            for q in range(N):
                for f in range(F):
                    res = (q + f) % N  # rt_frame: (row_offset + f * frame_shift) % row_stride, in blocks
                    for k in range(n):
                        y = res * B + (k // B) * N * B + k % B
                        if y < self.H:
                            src.append((q * F + f) * n + k)
                            dst.append(f * self.H + y)
            dev = self.frame.device
            self._flat = (torch.tensor(src, dtype=torch.long, device=dev),
                          torch.tensor(dst, dtype=torch.long, device=dev))
        src, dst = self._flat
        rows = self.parts[i].view(-1, self.W, self.C).index_select(0, src)
        self.frame.view(-1, self.W, self.C).index_copy_(0, dst, rows)

    def gather(self, i=0):
        """collective: every rank calls it after rendering into blocks[i]; the returned frame is ready on
        the current stream"""
        self.start(i)
        out = self.finish(i)
        if self._side is not None:
            import torch
            torch.cuda.current_stream().wait_event(self._copied[i])
        return out


class NativeGather:
    """The N > 1 frame gather through the boundary's own RCCL code (include/rt_hip.h rt_comm_init_rank /
    rt_comm_gather_from, replacing gpu/src/gpu.cu:203-228's load_from_gpu): one communicator per rank, shared by its
    contexts (bench.py alternates contexts on their own streams), torch.distributed only hands the RCCL id out; the
    row-set descriptors are exchanged once per layout, and the layout's first gather is checked pixel by pixel. Each context
    renders its rows of a frame batch into target(c) (compact rows, as rt_render_frames writes them); gather(c),
    called on every rank right after that render, enqueues the send (or, on rank 0, the receives and the
    un-interleaving into frames(c)) on the context's stream, so the gather of one context's batch overlaps the
    next render of the other. Same row layout as FrameGather (8-row blocks, residues rotated per frame)."""

    def __init__(self, renderers, H, W, C, rank, world, dist, like, frames=1, block=1, rotate=False, timeout=120.0):
        import torch
        from . import device
        self.H, self.W, self.C, self.rank, self.world = H, W, C, rank, world
        self.frames, self.bk = frames, max(1, block)
        self.rotate = bool(rotate) and frames > 1 and self.bk > 1 and world > 1
        self.n_max = padded_rows(H, world, self.bk)
        n = self.n_max if self.rotate else rank_rows(H, rank, world, self.bk)[2]
        self.blocks = [torch.zeros((frames, n, W, C), dtype=like.dtype, device=like.device) for _ in renderers]
        self.full = [torch.zeros((frames, H, W, C), dtype=like.dtype, device=like.device) for _ in renderers] \
            if rank == 0 else None
        ids = [device.comm_id()] if rank == 0 else [None]
        if dist is not None:
            dist.broadcast_object_list(ids, src=0)
        # one communicator for the rank, shared by its contexts (rt_comm_gather_from)
        self.comm = device.Comm([renderers[0]], world, rank, ids[0])
        self.comm.set_timeout(timeout)  # every host wait on a collective bounded (rt_comm_set_timeout)
        self.renderers = list(renderers)

    def rows(self):
        r = rank_rows(self.H, self.rank, self.world, self.bk)
        if self.rotate:
            return r[0], r[1], self.n_max, self.bk, self.bk
        return r if self.bk > 1 else r[:3]

    def target(self, c):
        """context c's render output: [frames, n_rows, W, C] compact rows (render nf <= frames into [:nf])"""
        return self.blocks[c]

    def gather(self, c, nf=None):
        """collective (every rank, after context c's render of nf frames): its frames -> rank 0's frames_of(c)"""
        out = self.full[c][:nf or self.frames] if self.rank == 0 else None
        self.comm.gather(root=0, out=out, src=self.renderers[c])

    def wait(self):
        """bounded wait for the last gather (rt_comm_wait): raises, with the communicator aborted, when a peer never
        joined, instead of leaving the caller's device synchronisation to hang"""
        self.comm.wait()

    def frames_of(self, c):
        return self.full[c] if self.rank == 0 else None

    def info(self):
        return self.comm.info()

    def close(self):
        self.comm.close()
