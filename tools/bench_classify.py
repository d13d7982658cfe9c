"""bench_classify.py -- batched get_labels(indices, presence_ratio)
(include/mbrwt.h mbrwt_get_labels_batch_device; annotate_static.cpp:71-94),
the `classify` consumer of get_rows, on the
Kingsford-shaped Multi-BRWT of bench.py (3.7 B x 2,652, d = 0.3 %, device
generated).  Synthetic reads of --read-len k-mer rows drawn uniformly at random
(rows of a real read are correlated; i.i.d. rows are the label-richest case for
ratio 0).  One step = one call over --reads reads, device-resident in and out.
Parity: every read of the batch against the reference semantics applied to
the batch's own get_rows output (np.bincount + the std::ceil threshold)."""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=3_700_000_000)
ap.add_argument("--cols", type=int, default=2652)
ap.add_argument("--density", type=float, default=0.003)
ap.add_argument("--reads", type=int, default=100_000)
ap.add_argument("--read-len", type=int, default=80)
ap.add_argument("--ratio", type=float, default=0.0)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--top", type=int, default=-1, help="get_top_labels(indices, TOP) instead (classify --count-labels)")
a = ap.parse_args()

from genome_graph_annotation_amd import BRWTDevice, _lib as L  # noqa: E402

dev = torch.device("cuda", 0)
mat = BRWTDevice.synthetic(a.rows, a.cols, a.density, 8, 42)
rng = np.random.default_rng(3)
n = a.reads * a.read_len
rows_np = rng.integers(0, a.rows, n, dtype=np.uint64)
read_off = np.arange(a.reads + 1, dtype=np.uint64) * a.read_len
rt = torch.from_numpy(rows_np.view(np.int64)).to(dev)
ot = torch.from_numpy(read_off.view(np.int64)).to(dev)
lo = torch.empty(a.reads + 1, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream(dev).cuda_stream
top = a.top >= 0


def call(lt, ct):
    if top:
        return mat.get_top_labels_batch_device(rt, ot, a.top, lo, lt, ct, s)
    return mat.get_labels_batch_device(rt, ot, a.ratio, lo, lt, s)


try:
    need = call(None, None)
except L.MBRWTError as e:
    need = e.needed
lt = torch.empty(need + 1024, dtype=torch.int32, device=dev)
ct = torch.empty(need + 1024, dtype=torch.int64, device=dev)
call(lt, ct)  # warm-up
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.steps):
    got = call(lt, ct)
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / a.steps

# parity: the reference's get_labels / get_top_labels over this batch's own rows (get_rows)
off_r, cols_r = mat.get_rows(rows_np)
lo_h = lo.cpu().numpy().view(np.uint64)
lt_h = lt[:got].cpu().numpy().view(np.uint32)
ct_h = ct[:got].cpu().numpy().view(np.uint64)
ok = True
for r in range(a.reads):
    x, y = int(read_off[r]), int(read_off[r + 1])
    cnt = np.bincount(cols_r[off_r[x]:off_r[y]], minlength=a.cols)
    sl = slice(int(lo_h[r]), int(lo_h[r + 1]))
    if top:
        nz = np.nonzero(cnt)[0]
        want = nz[np.lexsort((nz, -cnt[nz].astype(np.int64)))][:a.top]
        good = np.array_equal(lt_h[sl], want) and np.array_equal(ct_h[sl], cnt[want])
    else:
        thr = 1 if a.ratio == 0 else math.ceil((y - x) * a.ratio)
        good = np.array_equal(lt_h[sl], np.nonzero((cnt > 0) & (cnt >= thr))[0])
    if not good:
        ok = False
        break
what = ("get_top_labels(indices, num_top)" if top else "get_labels(indices, presence_ratio)")
print(json.dumps({
    "metric": f"batched {what} on Multi-BRWT (classify), reads/s",
    "value": a.reads / el, "unit": "reads/s", "rows_per_s": n / el, "ms_per_step": el * 1e3,
    "config": {"rows": a.rows, "columns": a.cols, "density": a.density, "reads": a.reads,
               "read_len": a.read_len, "presence_ratio": None if top else a.ratio,
               "num_top": a.top if top else None, "labels_out": int(got)},
    "parity": (f"every read identical to {'annotate.cpp:57-83' if top else 'annotate_static.cpp:71-94'} "
               "applied to the batch's get_rows"
               if ok else "MISMATCH"),
}))
