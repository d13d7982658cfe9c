"""Multi-GPU sharding of a get_rows batch.

The BRWT image is replicated on every GPU (each rank builds or loads its own
copy; nothing of the structure crosses xGMI).  A batch of query rows is cut
into contiguous per-rank slices; every rank runs the HIP traversal on its
slice and the per-row label sets are reassembled into one global CSR by an
all-gatherv over RCCL (backend "nccl" on ROCm).

RCCL has no all-gatherv, so the exchange is:
  1. one tiny all-gather of every rank's (rows, labels) sizes (the only host
     synchronisation);
  2. ONE all_gather_into_tensor of a packed byte buffer per rank, padded to
     the largest rank: [per-row label counts | labels].  The wire types are
     u16 when the matrix has < 2^16 columns (a count is <= num_columns, a
     label < num_columns) and u32 otherwise -- the Kingsford shape (2,652
     columns) ships 2 bytes per label and per row instead of 4 + 8, i.e.
     ~2.2x fewer bytes over xGMI than u32 labels + u64 offsets;
  3. unpacking with contiguous slice copies: one scan of the gathered counts
     gives the global offsets, each rank's label slice is widened into its
     place of the global label array.
AllGatherV splits 1-2 from 3 so that a batch's exchange overlaps the next
batch's traversal (bench.py pipelines its steps this way); on GPUs the
unpacking is queued behind the all-gather on a side stream and overlaps too.
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


def _round16(x: int) -> int:
    return (x + 15) // 16 * 16


def wire_is_narrow(num_columns) -> bool:
    """u16 wire types are exact when every count (<= num_columns) and every
    label (< num_columns) fits 16 bits."""
    return num_columns is not None and num_columns < (1 << 16)


class AllGatherV:
    """One all-gatherv of per-rank CSR slices, split so that the exchange can
    overlap the next batch's traversal: start() exchanges the sizes (the only
    host synchronisation), packs the wire buffer and launches the all-gather
    asynchronously; finish() waits for it and unpacks.  Between the two the
    caller may run other GPU work on the current stream (RCCL runs the
    all-gather on its own stream)."""

    def __init__(self, offsets: torch.Tensor, cols: torch.Tensor, n_labels=None, num_columns=None, group=None):
        self.group = group
        world = dist.get_world_size(group)
        dev = offsets.device
        n_r = offsets.numel() - 1
        l_r = int(offsets[-1].item()) if n_labels is None else int(n_labels)
        sizes = torch.tensor([n_r, l_r], dtype=torch.int64, device=dev)
        all_sizes = torch.empty(world * 2, dtype=torch.int64, device=dev)
        _all_gather(all_sizes, sizes, group)
        table = all_sizes.view(world, 2).cpu().tolist()
        self.ns, self.ls = [t[0] for t in table], [t[1] for t in table]
        max_n, max_l = max(self.ns), max(self.ls)
        self.num_columns = num_columns
        self.narrow = wire_is_narrow(num_columns)
        self.wdt = torch.int16 if self.narrow else torch.int32
        wb = 2 if self.narrow else 4
        self.cnt_bytes = _round16(max(1, max_n) * wb)
        self.per = self.cnt_bytes + _round16(max(1, max_l) * wb)
        # pack: counts (offsets deltas) then labels, in the wire type (int64 ->
        # int16 keeps the low 16 bits: exact for values < 2^16, read back & 0xFFFF)
        send = torch.empty(self.per, dtype=torch.uint8, device=dev)
        if n_r:
            send[:self.cnt_bytes].view(self.wdt)[:n_r].copy_(offsets[1:] - offsets[:-1])
        if l_r:
            send[self.cnt_bytes:].view(self.wdt)[:l_r].copy_(cols[:l_r])
        self.recv = torch.empty(world * self.per, dtype=torch.uint8, device=dev)
        self.send = send  # kept alive until the exchange is done
        if dist.get_backend(group) == "nccl":
            self.work = dist.all_gather_into_tensor(self.recv, send, group=group, async_op=True)
        else:
            self.work = dist.all_gather(list(self.recv.chunk(world)), send, group=group, async_op=True)
        self.result = None
        self.done = None
        if dev.type == "cuda":
            # the unpacking is queued right behind the all-gather on a side
            # stream, so it too overlaps whatever the caller runs next
            side = _side_stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                self.work.wait()
                self.result = self._unpack()
                self.done = torch.cuda.Event()
                self.done.record(side)
            for t in (self.send, self.recv):
                t.record_stream(side)

    def finish(self):
        """Wait for the exchange and return the global CSR (offsets [N + 1]
        int64, cols [L] int32)."""
        if self.done is not None:
            torch.cuda.current_stream(self.recv.device).wait_event(self.done)
            g_off, g_cols = self.result
            for t in (g_off, g_cols):
                t.record_stream(torch.cuda.current_stream(self.recv.device))
        else:
            self.work.wait()
            g_off, g_cols = self._unpack()
        self.send = self.recv = self.result = None
        return g_off, g_cols

    def _unpack(self):
        world = len(self.ns)
        dev = self.recv.device
        R = self.recv.view(world, self.per)
        # unpack: global offsets by one scan over the ranks' counts in rank order
        N, L = sum(self.ns), sum(self.ls)
        g_cnt = torch.empty(N, dtype=torch.int64, device=dev)
        g_cols = torch.empty(L, dtype=torch.int32, device=dev)
        rb = lb = 0
        for r in range(world):
            if self.ns[r]:
                g_cnt[rb:rb + self.ns[r]].copy_(R[r, :self.cnt_bytes].view(self.wdt)[:self.ns[r]])
            if self.ls[r]:
                g_cols[lb:lb + self.ls[r]].copy_(R[r, self.cnt_bytes:].view(self.wdt)[:self.ls[r]])
            rb += self.ns[r]
            lb += self.ls[r]
        if self.narrow:  # int16 sign-extended on the way back: restore the u16 values
            g_cnt.bitwise_and_(0xFFFF)
            if self.num_columns > (1 << 15):
                g_cols.bitwise_and_(0xFFFF)
        g_off = torch.zeros(N + 1, dtype=torch.int64, device=dev)
        if N:
            torch.cumsum(g_cnt, 0, out=g_off[1:])
        return g_off, g_cols


_SIDE = {}


def _side_stream(dev):
    if dev not in _SIDE:
        _SIDE[dev] = torch.cuda.Stream(dev)
    return _SIDE[dev]


def allgatherv_csr(offsets: torch.Tensor, cols: torch.Tensor, n_labels=None, num_columns=None, group=None):
    """Reassemble per-rank CSR slices (offsets: int64 [n_r + 1] starting at 0;
    cols: int32 [>= offsets[-1]]) into the global CSR of the concatenated
    batch, on every rank.  `n_labels` (= offsets[-1], if the caller already
    has it on the host) saves a device read; `num_columns` (the same on every
    rank) enables the u16 wire format.  Returns (offsets [N + 1] int64,
    cols [L] int32)."""
    return AllGatherV(offsets, cols, n_labels, num_columns, group).finish()
