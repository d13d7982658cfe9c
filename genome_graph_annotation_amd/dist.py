"""Multi-GPU sharding of a get_rows batch.

The BRWT image is replicated on every GPU (each rank builds or loads its own
copy; nothing of the structure crosses xGMI).  A batch of query rows is cut
into contiguous per-rank slices; every rank runs the HIP traversal on its
slice and the per-row label sets are reassembled into one global CSR by an
all-gatherv over RCCL (backend "nccl" on ROCm).  RCCL has no all-gatherv, so
the label arrays are padded to the largest rank's count and gathered with one
all_gather_into_tensor; the padding is <1% for equal-sized random slices.
The same code runs on gloo (CPU tensors) for the multi-process CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(n: int, world: int, rank: int):
    """Contiguous slice [lo, hi) of an n-row batch owned by `rank`."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _all_gather(out: torch.Tensor, inp: torch.Tensor, group=None):
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, inp, group=group)
    else:
        world = dist.get_world_size(group)
        parts = list(out.chunk(world))
        dist.all_gather(parts, inp, group=group)


def allgatherv_csr(offsets: torch.Tensor, cols: torch.Tensor, group=None):
    """Reassemble per-rank CSR slices (offsets: int64 [n_r + 1] starting at 0;
    cols: int32 [>= offsets[-1]]) into the global CSR of the concatenated
    batch, on every rank.  Returns (offsets [N + 1] int64, cols [L] int32)."""
    world = dist.get_world_size(group)
    dev = offsets.device
    n_r = offsets.numel() - 1
    l_r = int(offsets[-1].item())
    sizes = torch.tensor([n_r, l_r], dtype=torch.int64, device=dev)
    all_sizes = torch.empty(world * 2, dtype=torch.int64, device=dev)
    _all_gather(all_sizes, sizes, group)
    all_sizes = all_sizes.view(world, 2).cpu()
    max_n = int(all_sizes[:, 0].max())
    max_l = int(all_sizes[:, 1].max())
    # rows: gather per-row counts (offsets deltas), padded
    cnt = torch.zeros(max_n, dtype=torch.int64, device=dev)
    cnt[:n_r] = offsets[1:] - offsets[:-1]
    all_cnt = torch.empty(world * max_n, dtype=torch.int64, device=dev)
    _all_gather(all_cnt, cnt, group)
    # labels, padded to the largest slice
    lab = torch.zeros(max(1, max_l), dtype=torch.int32, device=dev)
    lab[:l_r] = cols[:l_r]
    all_lab = torch.empty(world * max(1, max_l), dtype=torch.int32, device=dev)
    _all_gather(all_lab, lab, group)
    # compact: drop the padding of every slice
    keep_rows = torch.cat([torch.arange(int(all_sizes[r, 0]), device=dev) + r * max_n for r in range(world)])
    keep_lab = torch.cat([torch.arange(int(all_sizes[r, 1]), device=dev) + r * max(1, max_l) for r in range(world)])
    g_cnt = all_cnt[keep_rows]
    g_off = torch.zeros(g_cnt.numel() + 1, dtype=torch.int64, device=dev)
    torch.cumsum(g_cnt, 0, out=g_off[1:])
    return g_off, all_lab[keep_lab]
