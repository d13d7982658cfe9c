"""bench_wire.py -- the device-sized all-gatherv's per-rank costs at the
bench's global batch (8 M rows of the C4 law), on one GPU: a one-rank RCCL
group, the rank's slice = the whole batch, so pack, all-gather (a local copy
here) and unpack see exactly the bytes one rank of an N-GPU step handles
(every rank unpacks the GLOBAL CSR).  Prints one JSON line with the mean
device times of each phase and the unpacked CSR checked against the slice.

    python tools/bench_wire.py [--rows 1000000000] [--batch 8000000]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genome_graph_annotation_amd import BRWTDevice  # noqa: E402
from genome_graph_annotation_amd.dist import DeviceAllGatherV  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=1_000_000_000)
ap.add_argument("--batch", type=int, default=8_000_000)
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()

dev = torch.device("cuda", 0)
dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
m = BRWTDevice.synthetic(a.rows, 2652, 0.003, 8, 42, layout="rows")
rows = torch.from_numpy(np.random.default_rng(42).integers(0, a.rows, a.batch, dtype=np.uint64).view(np.int64)).cuda()
off = torch.empty(a.batch + 1, dtype=torch.int64, device=dev)
cols = torch.empty(a.batch * 12, dtype=torch.int32, device=dev)
st = torch.zeros(3, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream().cuda_stream
m.get_rows_device_async(rows, off, cols, st, s)
torch.cuda.synchronize()
nl = int(st[0].item())
wire = DeviceAllGatherV([a.batch], int(nl * 1.02) + 1024, 2652, dev, timing=True)
for _ in range(3):
    g = wire.finish(wire.start(off, cols, st))
torch.cuda.synchronize()
wire.last_phases = []
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(a.steps):
    g = wire.finish(wire.start(off, cols, st))
ev1.record()
torch.cuda.synchronize()
g_off, g_cols, g_st = g
ok = bool(torch.equal(g_off, off) and torch.equal(g_cols[:nl], cols[:nl]) and g_st.tolist() == [nl, 0])
ph = wire.phases()
print(json.dumps({"rows": a.batch, "labels": nl, "wire_bytes": wire.wire_bytes, "exact": ok,
                  "exchange_ms": ev0.elapsed_time(ev1) / a.steps, **ph}), flush=True)
dist.destroy_process_group()
