"""A/B sweep of traversal-kernel variants on one structure, in one process
(interleaved repetitions, HIP-event kernel times).  Calibration tool, not the
bench: python tools/sweep.py --rows 3700000000 --batch 8000000"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genome_graph_annotation_amd import BRWTDevice, _lib as L  # noqa: E402
from genome_graph_annotation_amd.brwt import build_option  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=3_700_000_000)
ap.add_argument("--cols", type=int, default=2652)
ap.add_argument("--density", type=float, default=0.003)
ap.add_argument("--arity", type=int, default=8)
ap.add_argument("--batch", type=int, default=8_000_000)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--variants", default="1,2,3,4")
ap.add_argument("--presort", action="store_true", help="sort the batch on the host (locality experiment)")
ap.add_argument("--fold", default="1", help="root folding settings to build, e.g. 0,1")
a = ap.parse_args()
ap2 = a
mats = {}
for fold in a.fold.split(","):
    t0 = time.time()
    kinds = L.MBRWT_KIND_ALL if fold != "0" else L.MBRWT_KIND_ALL & ~L.MBRWT_KIND_FOLD_ROOT
    with build_option(L.MBRWT_BUILD_NODE_KINDS, kinds):
        mats[fold] = BRWTDevice.synthetic(a.rows, a.cols, a.density, a.arity, 42)
    print(f"built fold={fold} {mats[fold].device_bytes() / 1e9:.1f} GB in {time.time() - t0:.1f}s", flush=True)
m = next(iter(mats.values()))
rows_np = np.random.default_rng(42).integers(0, a.rows, a.batch, dtype=np.uint64)
if a.presort:
    rows_np = np.sort(rows_np)
rows = torch.from_numpy(rows_np.view(np.int64)).cuda()
off = torch.empty(a.batch + 1, dtype=torch.int64, device="cuda")
s = torch.cuda.current_stream().cuda_stream
v, lab = m.count_work_device(rows, s)
cols = torch.empty(2 * lab + 1024, dtype=torch.int32, device="cuda")  # diagnostic variants may emit more
alg = 64 * v + 16 * a.batch + 4 * lab
variants = [int(x) for x in a.variants.split(",")]
sorts = [0]
res = {}
ref = None  # every variant's CSR must equal the first one's (bit-exact)
for rep in range(a.reps):
  for fold, m in mats.items():
    for var in variants:
        for so in [fold]:
            m.set_option(L.MBRWT_OPT_KERNEL, var)
            nl = m.get_rows_device(rows, off, cols, s)
            if rep == 0:
                torch.cuda.synchronize()
                got = (off.clone(), cols[:nl].clone())
                if ref is None:
                    ref = got
                elif not (torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1])):
                    print(f"MISMATCH: variant {var} differs from variant {variants[0]}", flush=True)
                    sys.exit(1)
            m.take_timing()
            m.set_option(L.MBRWT_OPT_TIMING, 1)
            torch.cuda.synchronize()
            w0 = time.perf_counter()
            for _ in range(3):
                m.get_rows_device(rows, off, cols, s)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - w0) / 3
            m.set_option(L.MBRWT_OPT_TIMING, 0)
            ms, k = m.take_timing()
            res.setdefault((var, so), []).append((ms / k, wall * 1e3))
for (var, so), xs in sorted(res.items()):
    kms = np.median([x[0] for x in xs])
    wms = np.median([x[1] for x in xs])
    print(f"variant {var} fold {so}: kernel {kms:.3f} ms  step {wms:.3f} ms  -> {a.batch / wms * 1e3 / 1e6:.1f} M rows/s, "
          f"alg {alg / kms / 1e6:.0f} GB/s")
