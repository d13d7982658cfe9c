"""Traversal A/B on one synthetic structure (measurement tool, not the bench).

Builds the BASELINE C4 structure (or the given shape) with the library named
by MBRWT_LIB (tools/ab_build.sh variants; default the release library), runs
the asynchronous get_rows on one stream and prints one JSON line: the
traversal kernel's HIP-event time, the step time, and -- for a build with
MBRWT_AB_STAMPS -- the per-phase shader-clock cycles of k_traverse_rows summed
over every wave of the last launch (load, parse + scan, walk, output, loop).

    MBRWT_LIB=tools/_ab/libmbrwt_stamps.so python tools/trav_ab.py --steps 20
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genome_graph_annotation_amd import BRWTDevice, _lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=3_700_000_000)
ap.add_argument("--cols", type=int, default=2652)
ap.add_argument("--density", type=float, default=0.003)
ap.add_argument("--arity", type=int, default=8)
ap.add_argument("--batch", type=int, default=8_000_000)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--seed", type=int, default=42)
ap.add_argument("--shape", default="", help="npz (num_children/first_child/leaf_column): synthetic_shaped")
ap.add_argument("--tag", default="")
ap.add_argument("--stamps-out", default="", help="save the per-wave stamp words (npy) here")
ap.add_argument("--probe", action="store_true", help="also measure the random-request ceiling (tools/probe.hip)")
ap.add_argument("--var-lanes", type=int, default=0, help="MBRWT_BUILD_VAR_LANES of the build (0: auto)")
ap.add_argument("--wgs-per-cu", type=int, default=0, help="MBRWT_BUILD_ROWS_WGS_PER_CU of the build (0: auto)")
ap.add_argument("--rows-block", default="", help="B,S: MBRWT_BUILD_ROWS_BLOCK of the build (default: auto)")
a = ap.parse_args()

dev = torch.device("cuda:0")
t0 = time.time()
from genome_graph_annotation_amd.brwt import build_option  # noqa: E402
_lanes = build_option(L.MBRWT_BUILD_VAR_LANES, a.var_lanes)
_lanes.__enter__()
_wgs = build_option(L.MBRWT_BUILD_ROWS_WGS_PER_CU, a.wgs_per_cu)
_wgs.__enter__()
if a.rows_block:
    _bb, _ss = (int(x) for x in a.rows_block.split(","))
    _blk = build_option(L.MBRWT_BUILD_ROWS_BLOCK, _bb << 8 | _ss)  # (kept referenced: scoped to the script)
    _blk.__enter__()
if a.shape:
    mat = BRWTDevice.synthetic_shaped(a.rows, dict(np.load(a.shape)), a.density, a.seed, device=0, layout="rows")
else:
    mat = BRWTDevice.synthetic(a.rows, a.cols, a.density, a.arity, a.seed, device=0, layout="rows")
build_s = time.time() - t0
batches = [torch.from_numpy(np.random.default_rng(a.seed + k).integers(0, a.rows, a.batch, dtype=np.uint64)
                            .view(np.int64)).to(dev) for k in range(4)]
off = torch.empty(a.batch + 1, dtype=torch.int64, device=dev)
cols = torch.empty(int(a.batch * max(16.0, 3.0 * a.cols * a.density)) + 4096, dtype=torch.int32, device=dev)
status = torch.zeros(3, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream().cuda_stream
for i in range(a.warmup):
    mat.get_rows_device_async(batches[i % 4], off, cols, status, s)
torch.cuda.synchronize()
mat.take_timing()
mat.set_option(L.MBRWT_OPT_TIMING, 1)
t1 = time.perf_counter()
for i in range(a.steps):
    mat.get_rows_device_async(batches[i % 4], off, cols, status, s)
torch.cuda.synchronize()
step_ms = (time.perf_counter() - t1) / a.steps * 1e3
mat.set_option(L.MBRWT_OPT_TIMING, 0)
km, kl = mat.take_timing()
out = {"tag": a.tag, "lib": os.environ.get("MBRWT_LIB", "release"), "kernel": mat.traverse_kernel(),
       "kernel_ms": km / max(1, kl), "step_ms": step_ms, "build_s": round(build_s, 1),
       "status": status.cpu().tolist(), "rows_stats": mat.rows_stats()}
lib = L.lib()
if hasattr(lib, "mbrwt_ab_stamps"):
    # one more launch, then its per-wave phase cycles
    lib.mbrwt_ab_stamps.argtypes = [C.c_void_p, C.c_uint64]
    words = 16384 * 8
    buf = np.zeros(words, dtype=np.uint64)
    lib.mbrwt_ab_stamps(buf.ctypes.data, words)  # (clears)
    mat.get_rows_device_async(batches[0], off, cols, status, s)
    torch.cuda.synchronize()
    lib.mbrwt_ab_stamps(buf.ctypes.data, words)
    w = buf.reshape(-1, 8)
    if a.stamps_out:
        np.save(a.stamps_out, w)
    w = w[w[:, 7] == 1]
    names = ["load", "parse_scan", "walk", "output", "loop"]
    tot = w[:, 6].astype(np.float64)
    ph = {n: float(w[:, k].sum()) for k, n in enumerate(names)}
    all_c = sum(ph.values())
    out["stamps"] = {"waves": int(len(w)), "tiles": int(w[:, 5].sum()),
                     "cycles_per_tile": {n: v / max(1, w[:, 5].sum()) for n, v in ph.items()},
                     "share": {n: v / max(1.0, all_c) for n, v in ph.items()},
                     "wave_cycles_mean": float(tot.mean()), "wave_cycles_max": float(tot.max()),
                     "wave_cycles_min": float(tot.min())}
if a.probe:
    # the request ceiling on this box beside the structure: random 64-byte
    # segments over a buffer of the image's size (tools/probe.hip)
    sys.path.insert(0, ROOT)
    import bench
    free, _ = torch.cuda.mem_get_info(dev)
    sg, rnd = bench.probe_ceilings(dev, s, free, mat.device_bytes())
    out["probe"] = {"stream_read_GBs": sg, "random": rnd}
print(json.dumps(out), flush=True)
