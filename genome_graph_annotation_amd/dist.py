"""Multi-GPU sharding of a get_rows batch.

The BRWT image is replicated on every GPU (each rank builds or loads its own
copy; nothing of the structure crosses xGMI).  A batch of query rows is cut
into contiguous per-rank slices; every rank runs the HIP traversal on its
slice and the per-row label sets are reassembled into one global CSR by an
all-gatherv over RCCL (backend "nccl" on ROCm).

RCCL has no all-gatherv, so the exchange is:
  1. one tiny all-gather of every rank's (rows, labels) sizes -- host
     integers over a CPU (gloo) group, so no device read-back;
  2. ONE all_gather_into_tensor of a packed byte buffer per rank, padded to
     the largest rank: [per-row label counts | labels], both bit-packed at
     ceil(log2(num_columns)) bits (mbrwt_pack_ids_device) -- the Kingsford
     shape (2,652 columns) ships 12 bits per label and per row instead of
     32 + 64, i.e. ~2.9x fewer bytes over xGMI than u32 labels + u64 offsets;
  3. unpacking every rank's segment in ONE launch per array
     (mbrwt_unpack_segments_device: counts, then labels widened to int32 in
     their global places) and one scan of the counts for the global offsets.
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


def wire_bits(num_columns):
    """Bits per label and per row count on the wire: labels < num_columns,
    counts <= num_columns; 32 each when num_columns is unknown."""
    if num_columns is None:
        return 32, 32
    return max(1, int(num_columns - 1).bit_length()), max(1, int(num_columns).bit_length())


def _words(n: int, bits: int) -> int:
    return (n * bits + 31) // 32


def _pack(values: torch.Tensor, n: int, bits: int, out_words: torch.Tensor):
    """values (int32, >= n entries) -> out_words (int32 view of the wire):
    value i at bits [i*bits, (i+1)*bits), LSB-first (include/mbrwt.h
    mbrwt_pack_ids_device; numpy on CPU tensors)."""
    if not n:
        return
    if values.is_cuda:
        from . import _lib as L
        s = torch.cuda.current_stream(values.device).cuda_stream
        L.check(L.lib().mbrwt_pack_ids_device(values.data_ptr(), n, bits, out_words.data_ptr(), s),
                "mbrwt_pack_ids_device")
        return
    import numpy as np
    v = values[:n].numpy().view(np.uint32).astype(np.uint64)
    bitm = ((v[:, None] >> np.arange(bits, dtype=np.uint64)) & 1).astype(np.uint8).ravel()
    nw = _words(n, bits)
    bitm = np.concatenate([bitm, np.zeros(nw * 32 - len(bitm), dtype=np.uint8)])
    out_words[:nw].copy_(torch.from_numpy(np.packbits(bitm, bitorder="little").view(np.int32).copy()))


def _unpack(words: torch.Tensor, n: int, bits: int, out_values: torch.Tensor):
    """Inverse of _pack into out_values (int32, n entries)."""
    if not n:
        return
    if words.is_cuda:
        from . import _lib as L
        s = torch.cuda.current_stream(words.device).cuda_stream
        L.check(L.lib().mbrwt_unpack_ids_device(words.data_ptr(), n, bits, out_values.data_ptr(), s),
                "mbrwt_unpack_ids_device")
        return
    import numpy as np
    b = np.unpackbits(words.contiguous().numpy().view(np.uint8), bitorder="little")[: n * bits].reshape(n, bits)
    v = (b.astype(np.uint64) << np.arange(bits, dtype=np.uint64)).sum(axis=1).astype(np.uint32)
    out_values[:n].copy_(torch.from_numpy(v.view(np.int32)))


class AllGatherV:
    """One all-gatherv of per-rank CSR slices, split so that the exchange can
    overlap the next batch's traversal: start() exchanges the sizes, packs the
    wire buffer and launches the all-gather asynchronously; finish() waits for
    it and unpacks.  Between the two the caller may run other GPU work on the
    current stream (RCCL runs the all-gather on its own stream).

    size_group: a CPU (gloo) process group for the sizes exchange -- host
    integers the caller already has (get_rows_device returns the label count),
    so a GPU step synchronises the host once (inside get_rows) instead of
    also reading the sizes back from the device.  timing: HIP events around
    the pack, the all-gather and the unpack (phases())."""

    def __init__(self, offsets: torch.Tensor, cols: torch.Tensor, n_labels=None, num_columns=None, group=None,
                 size_group=None, timing=False):
        import time
        self.group = group
        world = dist.get_world_size(group)
        dev = offsets.device
        n_r = offsets.numel() - 1
        l_r = int(offsets[-1].item()) if n_labels is None else int(n_labels)
        h0 = time.perf_counter()
        if size_group is not None or dev.type != "cuda":
            sizes = torch.tensor([n_r, l_r], dtype=torch.int64)
            parts = [torch.empty(2, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(parts, sizes, group=size_group if size_group is not None else group)
            table = [p.tolist() for p in parts]
        else:
            sizes = torch.tensor([n_r, l_r], dtype=torch.int64, device=dev)
            all_sizes = torch.empty(world * 2, dtype=torch.int64, device=dev)
            _all_gather(all_sizes, sizes, group)
            table = all_sizes.view(world, 2).cpu().tolist()
        self.sizes_ms = (time.perf_counter() - h0) * 1e3
        self.ns, self.ls = [t[0] for t in table], [t[1] for t in table]
        max_n, max_l = max(self.ns), max(self.ls)
        self.bits_l, self.bits_c = wire_bits(num_columns)
        self.cnt_bytes = _round16(max(1, _words(max_n, self.bits_c)) * 4)
        self.per = self.cnt_bytes + _round16(max(1, _words(max_l, self.bits_l)) * 4)
        self.wire_bytes = self.per  # sent by this rank (received: (world - 1) x per)
        cuda = dev.type == "cuda"
        self.ev = {}
        if cuda and timing:
            for k in ("t0", "packed", "gathered", "done"):
                self.ev[k] = torch.cuda.Event(enable_timing=True)
            self.ev["t0"].record(torch.cuda.current_stream(dev))
        # pack: row counts (offsets deltas), then labels, bit-packed
        send = torch.empty(self.per, dtype=torch.uint8, device=dev)
        if n_r:
            cnt = (offsets[1:] - offsets[:-1]).to(torch.int32)
            _pack(cnt, n_r, self.bits_c, send[:self.cnt_bytes].view(torch.int32))
        if l_r:
            _pack(cols, l_r, self.bits_l, send[self.cnt_bytes:].view(torch.int32))
        if self.ev:
            self.ev["packed"].record(torch.cuda.current_stream(dev))
        self.recv = torch.empty(world * self.per, dtype=torch.uint8, device=dev)
        self.send = send  # kept alive until the exchange is done
        if dist.get_backend(group) == "nccl":
            self.work = dist.all_gather_into_tensor(self.recv, send, group=group, async_op=True)
        else:
            self.work = dist.all_gather(list(self.recv.chunk(world)), send, group=group, async_op=True)
        self.result = None
        self.done = None
        if cuda:
            # the unpacking is queued right behind the all-gather on a side
            # stream, so it too overlaps whatever the caller runs next
            side = _side_stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                self.work.wait()
                if self.ev:
                    self.ev["gathered"].record(side)
                self.result = self._unpack()
                self.done = self.ev["done"] if self.ev else torch.cuda.Event()
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

    def phases(self):
        """Device times (ms) of the exchange's phases -- pack, all-gather
        (from the packed buffer to the gathered one: RCCL's time plus any
        wait for the stream), unpack -- and the host time of the sizes
        exchange; valid once the exchange has completed (timing=True)."""
        out = {"sizes_host_ms": self.sizes_ms}
        if self.ev:
            self.ev["done"].synchronize()
            out["pack_ms"] = self.ev["t0"].elapsed_time(self.ev["packed"])
            out["all_gather_ms"] = self.ev["packed"].elapsed_time(self.ev["gathered"])
            out["unpack_ms"] = self.ev["gathered"].elapsed_time(self.ev["done"])
        return out

    def _unpack(self):
        world = len(self.ns)
        dev = self.recv.device
        N, L = sum(self.ns), sum(self.ls)
        g_cnt = torch.empty(max(1, N), dtype=torch.int32, device=dev)
        g_cols = torch.empty(L, dtype=torch.int32, device=dev)
        if dev.type == "cuda":
            # every rank's segment in one launch each (include/mbrwt.h
            # mbrwt_unpack_segments_device): counts, then labels
            import ctypes as C
            from . import _lib as LB
            s = torch.cuda.current_stream(dev).cuda_stream
            base = self.recv.data_ptr()
            for off, counts, bits, out in ((0, self.ns, self.bits_c, g_cnt),
                                           (self.cnt_bytes, self.ls, self.bits_l, g_cols)):
                arr = (C.c_uint64 * world)(*counts)
                LB.check(LB.lib().mbrwt_unpack_segments_device(base + off, world, self.per, arr, bits,
                                                               out.data_ptr(), s), "mbrwt_unpack_segments_device")
        else:
            R = self.recv.view(world, self.per)
            rb = lb = 0
            for r in range(world):
                _unpack(R[r, :self.cnt_bytes].view(torch.int32), self.ns[r], self.bits_c, g_cnt[rb:])
                _unpack(R[r, self.cnt_bytes:].view(torch.int32), self.ls[r], self.bits_l, g_cols[lb:])
                rb += self.ns[r]
                lb += self.ls[r]
        # global offsets: one scan of the gathered counts in rank order
        g_off = torch.zeros(N + 1, dtype=torch.int64, device=dev)
        if N:
            torch.cumsum(g_cnt[:N], 0, dtype=torch.int64, out=g_off[1:])
        return g_off, g_cols


class DeviceAllGatherV:
    """The all-gatherv with DEVICE-side sizes: no host synchronisation per
    exchange, so a GPU step (asynchronous get_rows + this exchange) never
    waits on the host.  Every rank's wire segment has a fixed size, agreed
    once (outside the timed region): [u64 label count][row counts at
    bits_count][labels at bits_label, up to labels_cap] (include/mbrwt.h
    mbrwt_pack_csr_device).  The label count is read from the device (the
    status block of mbrwt_get_rows_device_async), the row counts of every
    rank are static (the batch split), and the segments' label prefix is
    computed on the device by the unpacking (mbrwt_unpack_labels_device).  A
    label count above labels_cap sets status[1]; the caller reads the status
    after its timed region.  GPU tensors and RCCL (or gloo) only.

    rows_per_rank: every rank's slice length (host ints; every rank must pass
    the same list); labels_cap: this rank's label capacity -- the ranks AGREE
    on the largest one here, so callers may pass their own sizing; slots:
    output double-buffering for pipelined steps.

    The wire segments of all ranks must have one size, or the all-gather
    mismatches (gloo aborts, RCCL hangs or reads past a segment), so the
    constructor is collective: it agrees on labels_cap (MAX over the group)
    and checks that every rank passed the same rows_per_rank and
    num_columns, raising the same ValueError on every rank otherwise."""

    def __init__(self, rows_per_rank, labels_cap, num_columns, device, group=None, timing=False, slots=2):
        from . import _lib as L
        self.L = L
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.ns = [int(x) for x in rows_per_rank]
        # (the entry count is checked inside the collective: a local raise
        # here would leave the other ranks blocked in its all-reduce)
        self.cap = _agree_wire(self.ns, int(labels_cap), int(num_columns), group, device)
        self.bits_l, self.bits_c = wire_bits(num_columns)
        n_max = max(self.ns)
        self.lab_off = int(L.lib().mbrwt_wire_labels_offset(n_max, self.bits_c))
        self.per = _round16(self.lab_off + max(1, (self.cap + 31) // 32 * self.bits_l) * 4)  # (whole 32-value chunks)
        self.wire_bytes = self.per
        self.device = device
        self.timing = timing
        N = sum(self.ns)
        self.N = N
        # the global offsets straight from the packed counts: one scan whose
        # input unpacks them (mbrwt_unpack_offsets_device), its scratch sized
        # once (every unpack runs on the one side stream, so one scratch)
        import ctypes as C
        self._counts = (C.c_uint64 * self.world)(*self.ns)
        self.fused_offsets = self.world <= 8  # (beyond one node: counts unpacked, then scanned)
        tb = C.c_uint64(0)
        if self.fused_offsets:
            L.check(L.lib().mbrwt_unpack_offsets_device(C.c_void_p(16), self.world, self.per, self._counts,
                                                        self.bits_c, None, None, C.byref(tb), None),
                    "mbrwt_unpack_offsets_device")
        self.scan_tmp = torch.empty(max(16, int(tb.value)), dtype=torch.uint8, device=device)
        self.slots = []
        for _ in range(slots):
            self.slots.append({
                "send": torch.empty(self.per, dtype=torch.uint8, device=device),
                "recv": torch.empty(self.world * self.per, dtype=torch.uint8, device=device),
                "off": torch.zeros(N + 1, dtype=torch.int64, device=device),
                "cnt": None if self.fused_offsets else torch.empty(max(1, N), dtype=torch.int32, device=device),
                "cols": torch.empty(max(1, self.world * self.cap) + 32, dtype=torch.int32, device=device),
                "status": torch.zeros(2, dtype=torch.int64, device=device),
                "done": torch.cuda.Event(),
                "ev": {k: torch.cuda.Event(enable_timing=True) for k in ("t0", "packed", "gathered", "done")}
                if timing else {},
            })
        self.k = 0
        self.side = _side_stream(device)
        self.last_phases = []

    def start(self, offsets, cols, d_num_labels):
        """Queue the exchange of this rank's slice (offsets [n_r + 1] int64,
        cols int32, d_num_labels: a device u64/int64 holding offsets[-1]);
        returns the slot handle for finish()."""
        L = self.L
        sl = self.slots[self.k % len(self.slots)]
        self.k += 1
        cur = torch.cuda.current_stream(self.device)
        s = cur.cuda_stream
        if sl.get("used"):
            # the slot's previous exchange (queued from any stream: callers may
            # alternate query streams) has read its send buffer and written its
            # outputs before this one packs
            cur.wait_event(sl["done"])
        sl["used"] = True
        if sl["ev"]:
            sl["ev"]["t0"].record(cur)
        L.check(L.lib().mbrwt_pack_csr_device(offsets.data_ptr(), self.ns[self.rank], cols.data_ptr(),
                                              cols.numel(), d_num_labels.data_ptr(), self.cap, self.bits_c, self.bits_l,
                                              self.lab_off, sl["send"].data_ptr(), self.per, s),
                "mbrwt_pack_csr_device")
        if sl["ev"]:
            sl["ev"]["packed"].record(cur)
        if dist.get_backend(self.group) == "nccl":
            work = dist.all_gather_into_tensor(sl["recv"], sl["send"], group=self.group, async_op=True)
        else:  # (gloo: the rehearsal of several ranks on one GPU)
            work = dist.all_gather(list(sl["recv"].chunk(self.world)), sl["send"], group=self.group, async_op=True)
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            work.wait()
            if sl["ev"]:
                sl["ev"]["gathered"].record(self.side)
            ss = self.side.cuda_stream
            import ctypes as C
            base = sl["recv"].data_ptr()
            # the labels with their device-side prefix, then the global offsets
            # from the row counts (static per rank) at byte 8 of every segment
            L.check(L.lib().mbrwt_unpack_labels_device(base, self.world, self.per, self.lab_off, self.cap,
                                                       self.bits_l, sl["cols"].data_ptr(), sl["cols"].numel(),
                                                       sl["status"].data_ptr(), ss), "mbrwt_unpack_labels_device")
            if self.fused_offsets:
                tb = C.c_uint64(self.scan_tmp.numel())
                L.check(L.lib().mbrwt_unpack_offsets_device(base, self.world, self.per, self._counts, self.bits_c,
                                                            sl["off"].data_ptr(), self.scan_tmp.data_ptr(),
                                                            C.byref(tb), ss), "mbrwt_unpack_offsets_device")
            else:
                L.check(L.lib().mbrwt_unpack_segments_device(base + 8, self.world, self.per, self._counts,
                                                             self.bits_c, sl["cnt"].data_ptr(), ss),
                        "mbrwt_unpack_segments_device")
                if self.N:
                    torch.cumsum(sl["cnt"][:self.N], 0, dtype=torch.int64, out=sl["off"][1:])
            if sl["ev"]:
                sl["ev"]["done"].record(self.side)
            sl["done"].record(self.side)
        return sl

    def finish(self, sl):
        """Make the current stream wait for the slot's exchange; returns the
        global CSR (offsets [N + 1] int64, cols int32 with offsets[-1] valid
        entries) and the exchange's status (device int64 [2]: total labels,
        capacity overflow flag)."""
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(sl["done"])
        if sl["ev"]:
            self.last_phases.append(sl)
        return sl["off"], sl["cols"], sl["status"]

    def phases(self):
        """Mean device times (ms) of the timed exchanges' phases."""
        out = {}
        if not self.last_phases:
            return out
        acc = {"pack_ms": [], "all_gather_ms": [], "unpack_ms": []}
        for sl in self.last_phases:
            e = sl["ev"]
            e["done"].synchronize()
            acc["pack_ms"].append(e["t0"].elapsed_time(e["packed"]))
            acc["all_gather_ms"].append(e["packed"].elapsed_time(e["gathered"]))
            acc["unpack_ms"].append(e["gathered"].elapsed_time(e["done"]))
        return {k: float(sum(v) / len(v)) for k, v in acc.items()}


_SIDE = {}


def _agree_wire(ns, labels_cap, num_columns, group, device):
    """Collective precondition of the fixed-size wire: every rank's segment
    layout is a function of (rows_per_rank, labels_cap, num_columns), so all
    three must be equal on every rank.  Returns the group's largest
    labels_cap; raises ValueError on EVERY rank (they all see the same
    reduced values) when rows_per_rank or num_columns differ."""
    on = device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    world = dist.get_world_size(group)
    # first the entry counts, in a reduction of fixed size (ranks with lists
    # of different lengths would otherwise enter all-reduces of different
    # sizes: RCCL hangs, gloo times out), so every rank raises alike
    k = torch.tensor([len(ns), -len(ns)], dtype=torch.int64, device=on)
    dist.all_reduce(k, op=dist.ReduceOp.MAX, group=group)
    k_hi, k_lo = int(k[0].item()), -int(k[1].item())
    if k_hi != k_lo or k_hi != world:
        raise ValueError(f"DeviceAllGatherV: rows_per_rank has {k_lo}..{k_hi} entries over the ranks "
                         f"for a group of {world} ranks")
    v = [labels_cap, num_columns, len(ns)] + list(ns)
    mx = torch.tensor(v, dtype=torch.int64, device=on)
    mn = -mx  # MIN as the MAX of the negation: one reduction op for both backends
    both = torch.cat([mx, mn])
    dist.all_reduce(both, op=dist.ReduceOp.MAX, group=group)
    both = both.cpu().tolist()
    hi, lo = both[:len(v)], [-x for x in both[len(v):]]
    if hi[1:] != lo[1:]:
        what = "num_columns" if hi[1] != lo[1] else "rows_per_rank"
        raise ValueError(f"DeviceAllGatherV: the ranks passed different {what} "
                         f"(max {hi[1] if what == 'num_columns' else hi[3:]}, "
                         f"min {lo[1] if what == 'num_columns' else lo[3:]}); the wire segments would differ")
    return int(hi[0])


def _side_stream(dev):
    if dev not in _SIDE:
        _SIDE[dev] = torch.cuda.Stream(dev)
    return _SIDE[dev]


def allgatherv_csr(offsets: torch.Tensor, cols: torch.Tensor, n_labels=None, num_columns=None, group=None,
                   size_group=None):
    """Reassemble per-rank CSR slices (offsets: int64 [n_r + 1] starting at 0;
    cols: int32 [>= offsets[-1]]) into the global CSR of the concatenated
    batch, on every rank.  `n_labels` (= offsets[-1], if the caller already
    has it on the host) saves a device read; `num_columns` (the same on every
    rank) sets the wire's bit width.  Returns (offsets [N + 1] int64,
    cols [L] int32)."""
    return AllGatherV(offsets, cols, n_labels, num_columns, group, size_group).finish()
