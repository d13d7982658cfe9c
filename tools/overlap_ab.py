"""overlap_ab.py -- does batch k+1's traversal overlap batch k's output pass?
One row-record image and a clone of its context (mbrwt_ctx_clone: the same
image, separate workspaces), each driven on its own stream; batches
alternate between them (async get_rows).  Compared with one context on one
stream.
Experiment tool (not the bench); every batch's CSR hash is checked equal.

    python tools/overlap_ab.py --rows 3700000000 --batch 8000000 --steps 40
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genome_graph_annotation_amd import BRWTDevice  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=3_700_000_000)
ap.add_argument("--cols", type=int, default=2652)
ap.add_argument("--density", type=float, default=0.003)
ap.add_argument("--batch", type=int, default=8_000_000)
ap.add_argument("--steps", type=int, default=40)
a = ap.parse_args()

rows_np = np.random.default_rng(42).integers(0, a.rows, a.batch, dtype=np.uint64)
rows = torch.from_numpy(rows_np.view(np.int64)).cuda()
mats = [BRWTDevice.synthetic(a.rows, a.cols, a.density, 8, 42)]
mats.append(mats[0].clone())  # the same image, its own workspaces (mbrwt_ctx_clone)
mats.append(mats[0].clone())
torch.cuda.synchronize()
pool = [torch.cuda.Stream(), torch.cuda.Stream()]
null = torch.cuda.default_stream()
hi = torch.cuda.Stream(priority=-1)
STREAMS = {"pool": pool, "null+pool": [null, pool[1]], "null+hi": [null, hi], "null+pool+hi": [null, pool[1], hi],
           "null+pool+pool": [null, pool[0], pool[1]]}
streams = pool
need = mats[0].get_rows_device(rows, torch.empty(a.batch + 1, dtype=torch.int64, device="cuda"),
                               torch.empty(80_000_000, dtype=torch.int32, device="cuda"),
                               torch.cuda.current_stream().cuda_stream)
bufs = [(torch.empty(a.batch + 1, dtype=torch.int64, device="cuda"),
         torch.empty(int(need) + 1024, dtype=torch.int32, device="cuda"),
         torch.zeros(3, dtype=torch.int64, device="cuda")) for _ in range(3)]
torch.cuda.synchronize()


def run(k, dual):
    q = len(streams) if dual else 1
    for i in range(k):
        j = i % q
        off, cols, st = bufs[j]
        mats[j].get_rows_device_async(rows, off, cols, st, streams[j].cuda_stream)


def digest(j):
    off, cols, st = bufs[j]
    h = hashlib.blake2b(digest_size=8)
    h.update(off.cpu().numpy().tobytes())
    h.update(cols[:int(off[-1].item())].cpu().numpy().tobytes())
    return h.hexdigest()


out = {"rows": a.rows, "batch": a.batch, "steps": a.steps, "device_gb": mats[0].device_bytes() / 1e9}
for sk in ("pool", "null+pool", "null+hi", "null+pool+hi", "null+pool+pool", "null+pool"):
    streams = STREAMS[sk]
    for mode in ("single", "dual"):
        dual = mode == "dual"
        run(6, dual)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(a.steps, dual)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        out.setdefault(f"{mode}/{sk}", []).append({"ms_per_step": ms, "rows_per_s": a.batch / ms * 1e3})
        print(f"{mode} on {sk}: {ms:.4f} ms/step, {a.batch / ms / 1e6:.2f} G rows/s", file=sys.stderr, flush=True)
hs = [digest(0), digest(1)]
out["hashes"] = hs
out["same"] = hs[0] == hs[1]
for j in range(2):
    out[f"status{j}"] = bufs[j][2].cpu().tolist()
print(json.dumps(out), flush=True)
