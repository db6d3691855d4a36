"""1-D row sharding of a level-synchronous BFS across ranks.

The vertex set is cut into equal slots of 64-bit bitmap words, one per rank
(the last may be short).  Rank r owns rows [lo, hi) of A^T and computes the
next-frontier bits of those rows (`GrB_mxv` on its shard, or any local step);
the per-rank bitmap slices are then all-gathered so every rank holds the whole
frontier -- the path's only exchange step (RCCL over xGMI on GPUs, gloo in the
CPU tests).  Every rank sees the same gathered bitmap, so the termination test
(empty frontier) needs no extra collective.
"""
import numpy as np


def partition(n, world, rank):
    """Bitmap-word slot of `rank`: dict(words, slot, lo_w, hi_w, lo, hi)."""
    words = (n + 63) // 64
    slot = (words + world - 1) // world
    lo_w, hi_w = min(words, rank * slot), min(words, (rank + 1) * slot)
    return {"words": words, "slot": slot, "lo_w": lo_w, "hi_w": hi_w, "lo": lo_w * 64,
            "hi": min(n, hi_w * 64)}


class BitmapAllGather:
    """All-gather of equal-size int64 bitmap slices into one frontier bitmap.

    `send` (slot words) is filled by the local step (e.g. GxB_Vector_bitmap_export);
    after `run()`, `gathered[:words]` is the full bitmap (GxB_Vector_bitmap_import).
    Uses all_gather_into_tensor where the backend has it (NCCL/RCCL), else all_gather."""

    def __init__(self, dist, part, world, device):
        import torch

        self.dist = dist
        self.part = part
        self.world = world
        self.send = torch.zeros(part["slot"], dtype=torch.int64, device=device)
        self.gathered = torch.zeros(part["slot"] * world, dtype=torch.int64, device=device)
        self._fused = dist.get_backend() == "nccl"

    def run(self, out=None):
        """Gather into `out` (e.g. a vector's device bitmap, slot*world words) or the
        internal buffer; returns the tensor gathered into."""
        out = self.gathered if out is None else out
        if self._fused:
            self.dist.all_gather_into_tensor(out, self.send)
        elif self.send.is_cuda:  # gloo rehearsal of the GPU path: stage through host memory
            host = torch_empty_like_cpu(out)
            self.dist.all_gather(list(host.chunk(self.world)), self.send.cpu())
            out.copy_(host)
        else:
            self.dist.all_gather(list(out.chunk(self.world)), self.send)
        return out


def torch_empty_like_cpu(t):
    import torch

    return torch.empty(t.shape, dtype=t.dtype)


def pack_bits(mask_bool, nwords):
    """bool[k] -> int64[nwords] little-endian bitmap words (numpy)."""
    b = np.zeros(nwords * 64, dtype=bool)
    b[:mask_bool.size] = mask_bool
    return np.packbits(b, bitorder="little").view(np.int64)


def unpack_bits(words, n):
    """int64[*] bitmap words -> bool[n] (numpy)."""
    return np.unpackbits(np.ascontiguousarray(words).view(np.uint8), bitorder="little")[:n].astype(bool)
