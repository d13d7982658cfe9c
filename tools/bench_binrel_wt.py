"""bench_binrel_wt.py -- get_rows()/s of the BinRel-WT engine on BASELINE
configs[4]: BinRel-WT(sdsl) get_row on a 1 B x 3,173, d = 3.8 % matrix
(RefSeq shape), 1 x MI355X.  Prints ONE JSON line like bench.py.

One step = one batched get_row over 10 M uniform random rows (device-resident
ids -> device-resident CSR).  roofline: algorithmic bytes of the decode
kernel per launch = sum over rows of (16 + 4 L + 64 B x w x L) -- one 64-byte
line per symbol per wavelet level, w = 12 bits for 3,173 columns
(DESIGN.md "BinRel-WT"; the reference's levelwise tree, not this build's
4-ary wavelet matrix of ceil(w/2) levels) -- over its HIP-event time.  cpu_baseline: the
oracle's restatement of BinRelWT_sdsl::get_row (sdsl-style levelwise wavelet
tree, interval_symbols) over the first --cpu-rows rows of the SAME matrix,
timed on random rows of that prefix on the host cores.  Parity: the device
rows of the batch that fall in that prefix against the oracle element-wise,
and --check-rows batch rows against the row generator spec.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

METRIC = "get_rows()/s on BinRel-WT(sdsl), 1B×3,173 d=3.8% (BASELINE configs[4]), 1×MI355X"
HBM_PEAK_GBS = 8000.0


def committed_traffic(cfg):
    """Per-launch HBM traffic of k_wt_decode from the committed PMC summary of
    this workload (profiles/*/traffic_k_wt_decode*.json, tools/pmc_traffic.py),
    or None."""
    import glob
    hit = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic_k_wt_decode*.json"))):
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        if {k: str(v) for k, v in cfg.items()} == {k: str(v) for k, v in t.get("config", {}).items()}:
            hit = (t["traffic_bytes"], os.path.relpath(path, ROOT))
    return hit


def log(msg):
    print(f"[bench_wt] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000_000)
    ap.add_argument("--cols", type=int, default=3173)
    ap.add_argument("--density", type=float, default=0.038)
    ap.add_argument("--batch", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=2_000_000, help="prefix of rows the CPU oracle structure holds")
    ap.add_argument("--cpu-sample", type=int, default=200_000)
    ap.add_argument("--check-rows", type=int, default=200_000)
    a = ap.parse_args()

    from genome_graph_annotation_amd import BinRelWTDevice, _lib as L

    dev_t = torch.device("cuda", 0)
    t0 = time.time()
    mat = BinRelWTDevice.synthetic(a.rows, a.cols, a.density, a.seed)
    setup_s = time.time() - t0
    log(f"device structure built in {setup_s:.1f} s ({mat.device_bytes() / 1e9:.1f} GB, "
        f"{mat.num_relations():,} relations)")
    rows_np = np.random.default_rng(a.seed + 1).integers(0, a.rows, a.batch, dtype=np.uint64)
    rows_t = torch.from_numpy(rows_np.view(np.int64)).to(dev_t)
    off_t = torch.empty(a.batch + 1, dtype=torch.int64, device=dev_t)
    sptr = torch.cuda.current_stream(dev_t).cuda_stream
    probe = torch.empty(1, dtype=torch.int32, device=dev_t)
    try:
        need = mat.get_rows_device(rows_t, off_t, probe, sptr)
    except L.MBRWTError as e:
        if e.status != L.MBRWT_ERR_CAPACITY:
            raise
        need = e.needed
    cols_t = torch.empty(need + 1024, dtype=torch.int32, device=dev_t)
    for _ in range(a.warmup):
        mat.get_rows_device(rows_t, off_t, cols_t, sptr)
    torch.cuda.synchronize()
    mat.take_timing()
    mat.set_option(L.MBRWT_OPT_TIMING, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        n_lab = mat.get_rows_device(rows_t, off_t, cols_t, sptr)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    mat.set_option(L.MBRWT_OPT_TIMING, 0)
    kern_ms_total, launches = mat.take_timing()
    kern_ms = kern_ms_total / max(1, launches)
    w = max(1, int(np.ceil(np.log2(a.cols))))
    alg_bytes = 16 * a.batch + (4 + 64 * w) * n_lab
    achieved = alg_bytes / (kern_ms / 1e3) / 1e9
    log(f"timed {a.steps} steps: {elapsed / a.steps * 1e3:.2f} ms/step, decode kernel {kern_ms:.2f} ms")

    # parity against the generator spec on a sample of the batch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # checker / CPU-baseline leg only

    off_h = off_t.cpu().numpy().view(np.uint64)
    chk = min(a.check_rows, a.batch)
    cols_h = cols_t[: int(off_h[chk])].cpu().numpy().view(np.uint32)
    ok = True
    buf = np.zeros(a.cols, dtype=np.uint32)
    T = O.lib().wt_synth_threshold(a.density)
    for i in range(chk):
        cnt = O.lib().wt_synth_row(int(rows_np[i]), a.cols, T, a.seed, O._p32(buf), a.cols)
        if cnt != off_h[i + 1] - off_h[i] or not np.array_equal(buf[:cnt], cols_h[off_h[i]:off_h[i + 1]]):
            ok = False
            break
    parity = f"{'bit-exact' if ok else 'MISMATCH'} on {chk:,} batch rows vs the row generator spec"

    cpu = None
    if not a.no_cpu:
        threads = min(16, len(os.sched_getaffinity(0)))
        g0 = time.time()
        off_p, cols_p = O.wt_synth_rows(0, a.cpu_rows, a.cols, a.density, a.seed, threads)
        ref = O.OracleWT.from_csr(off_p, cols_p, a.cols)
        gen_s = time.time() - g0
        # device vs the oracle's own BinRel-WT on the batch rows inside the prefix
        inside = rows_np[rows_np < a.cpu_rows][:50_000]
        o_o, c_o = ref.get_rows(inside, threads)
        o_d, c_d = mat.get_rows(inside)
        same = np.array_equal(o_o, o_d) and np.array_equal(c_o, c_d)
        parity += f"; {'bit-exact' if same else 'MISMATCH'} on {len(inside):,} rows vs the BinRel-WT oracle"
        sample = np.random.default_rng(a.seed + 2).integers(0, a.cpu_rows, a.cpu_sample, dtype=np.uint64)
        cpu_s = ref.time_rows(sample, threads)
        cpu = {"value": len(sample) / cpu_s, "unit": "rows/s", "cores": threads, "kind": "port",
               "sample": f"{len(sample):,} random rows of the first {a.cpu_rows:,} rows of the same matrix, held in "
                         f"the oracle's levelwise wavelet tree (BinRelWT_sdsl::get_row restated, plain rank/select; "
                         f"host build {gen_s:.0f} s)"}
        del ref

    traffic = committed_traffic({"rows": a.rows, "cols": a.cols, "density": a.density, "batch": a.batch,
                                 "kernel_name": "k_wt_decode"})
    line = {
        "metric": METRIC, "value": a.batch * a.steps / elapsed, "unit": "rows/s", "n_gpus": 1,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32/u64",
        "data": "synthetic (i.i.d. Bernoulli rows from a counter hash, seed 42; uniform random query rows)",
        "config": {"workload": f"BinRel-WT {a.rows:,} x {a.cols:,}, d={a.density}; batch {a.batch:,} rows",
                   "num_rows": a.rows, "num_columns": a.cols, "density": a.density, "batch": a.batch,
                   "structure_bytes": mat.device_bytes(), "relations": mat.num_relations(),
                   "setup_s": round(setup_s, 1)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None if traffic is None else traffic[0],
                     "traffic_source": None if traffic is None else traffic[1] + " (rocprofv3 PMC; per launch)",
                     "kernel": "k_wt_decode",
                     "kernel_ms": kern_ms, "alg_bytes_per_launch": alg_bytes,
                     "labels_per_row": n_lab / a.batch, "levels": w, "digit_levels": (w + 1) // 2},
        "cpu_baseline": cpu,
        "parity": parity,
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
