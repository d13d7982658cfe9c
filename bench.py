"""bench.py -- get_rows()/s on a Kingsford-shaped Multi-BRWT (BASELINE.json).

Workload (config.workload): BASELINE.json configs[3] -- a 3.7 B x 2,652
Multi-BRWT (i.i.d. d = 0.3 % columns, basic arity-8 partitioner, generated
top-down on the device: DESIGN.md "Synthetic matrices"), replicated on every
GPU, queried with a GLOBAL batch of 8 M uniform random rows (seed 42) cut into
contiguous per-rank slices (strong scaling, SURVEY.md §8(d) C4: 8 M / N rows
per GPU; --scaling weak keeps 8 M rows per GPU instead).  One step = one
batched get_rows over the rank's slice, device-resident row ids -> CSR in HBM,
plus (N > 1) the RCCL all-gatherv that reassembles the global CSR on every
rank (pipelined: step k's exchange overlaps step k+1's traversal).

Prints ONE JSON line (rank 0).
  roofline  -- the dominant kernel's layout-true algorithmic bytes per launch
               (what its layout must read and write: alg_basis) / its
               HIP-event-timed average duration (achieved) / the 8 TB/s spec
               (frac); beside it the measured HBM traffic (rocprofv3 --pmc
               FETCH_SIZE and WRITE_SIZE, one child pass each over this same
               workload, at N = 1 before the timed run: traffic,
               traffic_frac), SURVEY §8(d)'s probe-equivalent bytes
               (64 B x V + 16 + 4 B x L per row, V and L counted exactly on
               the device), and the measured ceilings: a streaming read and
               random 64-byte requests (tools/probe.hip).
  cpu_baseline -- the oracle's restatement of BRWT::get_row on the same
               structure (built on the host from the same spec), on a bounded
               row sample, on the job's host cores and single-threaded.
  parity    -- the whole global batch's CSR against the oracle, element-wise
               and by a 64-bit hash (N = 1 and, on rank 0, N > 1).
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "get_rows()/s on Multi-BRWT, 3.7B×2,652 Kingsford-shape @1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip-level table (spec)
# FETCH_SIZE per random 64-byte segment read, calibrated on a known count of
# exactly that access shape (profiles/r01/calib_gather_probe*: factor 1.000;
# the guide's 1/2 under-count applies to wide streaming reads)
FETCH_CALIB = 1.0


# BASELINE.json configs: (rows, columns, density, batch, layout).  Row records
# (layout rows): fixed blocks at the Kingsford shape (k_traverse_rows); the
# RefSeq shape's records (~160 bytes, 120 labels per row) are longer than a
# block, so they take the variable-length records (k_var_decode).
WORKLOADS = {
    "c4": dict(rows=3_700_000_000, cols=2652, density=0.003, batch=8_000_000, layout="rows"),
    "c3": dict(rows=1_000_000_000, cols=3173, density=0.038, batch=10_000_000, layout="rows"),
    "c2": dict(rows=1_000_000, cols=2652, density=0.003, batch=1_000_000, layout="rows"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # (a step is ~0.36 ms: 50 timed steps after 10 warm-up steps keep the
    # timed region clear of the first steps' ramp, profiles/r04/v13_query_streams/)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c4",
                    help="BASELINE config preset (c4 = configs[3], the driver's default; c3 = configs[2]; "
                         "c2 = configs[1]); --rows/--cols/--density/--batch/--layout override it")
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--cols", type=int, default=None)
    ap.add_argument("--density", type=float, default=None)
    ap.add_argument("--arity", type=int, default=8)
    ap.add_argument("--batch", type=int, default=None,
                    help="query rows: the global batch (strong) or rows per GPU (weak)")
    ap.add_argument("--batches", type=int, default=4,
                    help="distinct seeded batches; timed step i queries batch i mod this (no replayed batch)")
    ap.add_argument("--layout", choices=["rows", "nodes", "both"], default=None,
                    help="device layout (include/mbrwt.h): row records or per-node images")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the all-gatherv reassembly")
    ap.add_argument("--host-sizes", action="store_true",
                    help="N>1: the all-gatherv with host-side sizes (a gloo exchange and a host sync per step) "
                         "instead of the device-sized wire (dist.DeviceAllGatherV)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the host oracle (CPU baseline and parity)")
    ap.add_argument("--cpu-sample", type=int, default=400_000, help="rows timed on the CPU (job's cores)")
    ap.add_argument("--cpu-sample-1t", type=int, default=40_000, help="rows timed on one CPU thread")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = the job's CPU share")
    ap.add_argument("--check-rows", type=int, default=0,
                    help="rows checked element-wise against the oracle (0 = the whole global batch)")
    ap.add_argument("--kernel", type=int, default=0, help="MBRWT_OPT_KERNEL variant (0 = library default)")
    ap.add_argument("--rows-code", type=int, default=0, choices=[0, 1, 2, 3],
                    help="row records (MBRWT_BUILD_ROWS_CODE): 0 the library default (AUTO: terminal records where "
                         "smaller, DESIGN §4h), 1 nibble codes (§4g), 2 terminal records, 3 byte masks")
    ap.add_argument("--rows-block", default="",
                    help="row records: force the block shape B:S (MBRWT_BUILD_ROWS_BLOCK; default: the cost model)")
    ap.add_argument("--compact-cus", type=int, default=0,
                    help="row records: run each query stream's compaction on a stream masked to K of every 32 "
                         "CUs (MBRWT_OPT_COMPACT_CUS, VERDICT r05 #1a; 0 = the library default, same stream)")
    ap.add_argument("--query-streams", type=int, default=2, choices=[1, 2, 3, 4],
                    help="N = 1: consecutive batches alternate between the context and a clone of it "
                         "(mbrwt_ctx_clone: the same image, separate workspaces) on the default stream and "
                         "a second stream, so batch k+1's traversal overlaps batch k's output pass "
                         "(DESIGN.md §6); 1 = one context, one stream")
    ap.add_argument("--kernel-timing", choices=["all", "first", "off"], default="all",
                    help="HIP events around the dominant kernel in the timed region: every query context, the "
                         "first only, or none (diagnosis: the events' own cost)")
    ap.add_argument("--sync", action="store_true",
                    help="N = 1: time the synchronous mbrwt_get_rows_device (default: the asynchronous call, "
                         "status checked after the timed region)")
    ap.add_argument("--dist-backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--traffic", choices=["live", "committed", "off"], default="live",
                    help="roofline traffic: rocprofv3 PMC child passes (N = 1), a committed summary of the "
                         "same kernel sources, or none")
    ap.add_argument("--traffic-out", default="", help="write the live traffic summary (JSON) here")
    ap.add_argument("--no-probe", action="store_true", help="skip the measured ceilings")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (host buffers) leg")
    ap.add_argument("--pmc-pass", action="store_true", help=argparse.SUPPRESS)  # child under rocprofv3
    a = ap.parse_args()
    w = WORKLOADS[a.workload]
    for k in ("rows", "cols", "density", "batch", "layout"):
        if getattr(a, k) is None:
            setattr(a, k, w[k])
    return a


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def kernel_source_hash():
    """sha256 (16 hex) of the product's HIP/C++ sources: a traffic summary is
    only valid for the kernels it was measured on."""
    h = hashlib.sha256()
    for p in sorted(glob.glob(os.path.join(ROOT, "genome_graph_annotation_amd", "csrc", "*"))):
        if p.endswith((".hip", ".hpp", ".cpp", ".h")):
            h.update(os.path.basename(p).encode())
            with open(p, "rb") as f:
                h.update(f.read())
    return h.hexdigest()[:16]


def rows_block_opt(a):
    """--rows-block B:S as MBRWT_BUILD_ROWS_BLOCK (B << 8 | S; 0 = the cost model)."""
    if not a.rows_block:
        return 0
    b, s_ = (int(x) for x in a.rows_block.split(":"))
    return b << 8 | s_


def workload_args(a):
    return ["--rows", str(a.rows), "--cols", str(a.cols), "--density", repr(a.density), "--arity", str(a.arity),
            "--batch", str(a.batch), "--seed", str(a.seed), "--kernel", str(a.kernel), "--layout", a.layout,
            "--rows-code", str(a.rows_code)] + (["--rows-block", a.rows_block] if a.rows_block else [])


def pmc_pass(a):
    """Child under rocprofv3 --pmc: the structure and the rank-0 batch of an
    N = 1 run, 2 warm-up + 3 counted launches of the traversal."""
    from genome_graph_annotation_amd import BRWTDevice, _lib as L
    from genome_graph_annotation_amd.brwt import build_option
    torch.cuda.set_device(0)
    with build_option(L.MBRWT_BUILD_ROWS_CODE, a.rows_code), build_option(L.MBRWT_BUILD_ROWS_BLOCK, rows_block_opt(a)):
        mat = BRWTDevice.synthetic(a.rows, a.cols, a.density, a.arity, a.seed, device=0, layout=a.layout)
    if a.kernel:
        mat.set_option(L.MBRWT_OPT_KERNEL, a.kernel)
    rows_np = np.random.default_rng(a.seed).integers(0, a.rows, a.batch, dtype=np.uint64)
    rows_t = torch.from_numpy(rows_np.view(np.int64)).cuda()
    off_t = torch.empty(a.batch + 1, dtype=torch.int64, device="cuda")
    cols_t = torch.empty(int(a.batch * max(16.0, 3.0 * a.cols * a.density)) + 1024, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(5):
        mat.get_rows_device(rows_t, off_t, cols_t, s)
    torch.cuda.synchronize()
    print(json.dumps({"kernel_name": mat.traverse_kernel()}), flush=True)


def per_dispatch(csv_path, kernel_re, counter):
    import csv
    import re
    vals = {}
    with open(csv_path, newline="") as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter or not re.search(kernel_re, r.get("Kernel_Name", "")):
                continue
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals, key=int)]


def live_traffic(a, kernel_re):
    """Per-launch FETCH_SIZE / WRITE_SIZE of the traversal kernel from two
    rocprofv3 --pmc child passes (separate passes: FETCH_SIZE takes 3 of the 4
    TCC slots, WRITE_SIZE 2; MI355X_MICROARCH.md).  KiB -> bytes; the first
    two dispatches are warm-up."""
    out = {"counters": {}, "source_hash": kernel_source_hash(), "kernel_regex": kernel_re,
           "config": {"rows": a.rows, "cols": a.cols, "density": a.density, "arity": a.arity, "batch": a.batch,
                      "kernel": a.kernel, "layout": a.layout, "rows_code": a.rows_code}}
    env = dict(os.environ, TMPDIR="/tmp")
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="bench_pmc_", dir="/tmp")
        cmd = ["rocprofv3", "--pmc", counter, "--kernel-include-regex", kernel_re, "-d", d, "-o", "run",
               "--output-format", "csv", "--", sys.executable, os.path.join(ROOT, "bench.py"), "--pmc-pass",
               *workload_args(a)]
        t0 = time.time()
        try:
            r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=240)
        except (OSError, subprocess.TimeoutExpired) as e:
            log(f"PMC pass {counter} failed: {e!r}")
            return None
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if r.returncode != 0 or not files:
            log(f"PMC pass {counter} failed (rc {r.returncode}): {r.stderr[-600:]}")
            return None
        vals = per_dispatch(files[0], kernel_re, counter)
        if len(vals) < 3:
            log(f"PMC pass {counter}: {len(vals)} dispatches of {kernel_re!r}")
            return None
        kib = float(np.median(vals[2:]))
        out["counters"][counter] = {"per_dispatch_kib": vals, "median_kib": kib, "pass_s": round(time.time() - t0, 1)}
        log(f"PMC {counter}: {kib * 1024 / 1e9:.3f} GB per launch ({len(vals)} dispatches, {time.time() - t0:.0f} s)")
    out["read_bytes"] = out["counters"]["FETCH_SIZE"]["median_kib"] * 1024 * FETCH_CALIB
    out["write_bytes"] = out["counters"]["WRITE_SIZE"]["median_kib"] * 1024
    out["traffic_bytes"] = out["read_bytes"] + out["write_bytes"]
    out["fetch_calibration"] = FETCH_CALIB
    return out


def committed_traffic(a, kernel_re):
    """A committed live-traffic summary (profiles/*/traffic_*.json) of this
    workload measured on the CURRENT kernel sources, or None."""
    want_cfg = {"rows": a.rows, "cols": a.cols, "density": a.density, "arity": a.arity, "batch": a.batch,
                "kernel": a.kernel, "layout": a.layout, "rows_code": a.rows_code}
    h = kernel_source_hash()
    hit = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic_*.json"))):
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        if t.get("source_hash") == h and t.get("kernel_regex") == kernel_re and t.get("config") == want_cfg:
            hit = dict(t, source=os.path.relpath(path, ROOT))
    return hit


def csr_hash(off: np.ndarray, cols: np.ndarray) -> str:
    h = hashlib.blake2b(digest_size=8)
    h.update(np.ascontiguousarray(off, dtype=np.uint64).tobytes())
    h.update(np.ascontiguousarray(cols, dtype=np.uint32).tobytes())
    return h.hexdigest()


def probe_ceilings(dev_t, stream_ptr, free_bytes, struct_bytes=64 << 30):
    """Measured ceilings of this GPU (tools/probe.hip): streaming-read GB/s,
    and random-segment requests/s -- the MAXIMUM over a sweep of requests in
    flight and resident waves (the full sweep:
    tools/probe_sweep.py, profiles/r03/v01_probe_sweep.json) for 64-byte and
    128-byte segments (the row-record blocks); None where the probe library is
    missing."""
    import ctypes as C
    path = os.path.join(ROOT, "tools", "_build", "libprobe.so")
    if not os.path.exists(path):
        log("tools/_build/libprobe.so missing: no measured ceilings")
        return None, None
    lib = C.CDLL(path)
    lib.probe_stream_read.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_void_p, C.POINTER(C.c_double)]
    lib.probe_random_seg.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                     C.POINTER(C.c_double)]
    stream_gbs = rnd = None
    buf = torch.empty(4 << 30, dtype=torch.uint8, device=dev_t)
    v = C.c_double(0)
    if lib.probe_stream_read(buf.data_ptr(), buf.numel(), 5, stream_ptr, C.byref(v)) == 0:
        stream_gbs = v.value
    del buf
    # random segments over a buffer far past the 256 MiB Infinity Cache, as
    # large as the structure where memory allows: the request rate falls with
    # the buffer's span (address translation; 54.2 G/s over 4 GiB, 49.4 G/s
    # over 118 GiB: profiles/r03/v05_probe_random64_*gib.json)
    big = min(max(struct_bytes, 8 << 30), int(free_bytes * 0.8)) // (1 << 30) << 30
    if big >= (8 << 30):
        cus = torch.cuda.get_device_properties(dev_t).multi_processor_count
        buf = torch.empty(big, dtype=torch.uint8, device=dev_t)
        rnd = {"buffer_gib": big >> 30}
        for seg, sweep in ((64, [(2, 16), (4, 16), (8, 16), (4, 32), (16, 32)]), (128, [(8, 32), (16, 32), (8, 16)])):
            best = None
            for inflight, wpc in sweep:
                if lib.probe_random_seg(buf.data_ptr(), buf.numel(), seg, inflight, cus * wpc // 4, 256, stream_ptr,
                                        C.byref(v)) == 0 and (best is None or v.value > best[0]):
                    best = (v.value, inflight, wpc)
            if best is not None:
                rnd[f"seg{seg}_per_s"] = best[0]
                rnd[f"seg{seg}_best"] = {"inflight": best[1], "waves_per_cu": best[2]}
        rnd["segments_per_s"] = rnd.get("seg64_per_s")
        del buf
    torch.cuda.empty_cache()
    return stream_gbs, rnd


def pcie_rates(dev_t, mib=256):
    """Pinned H2D / D2H GB/s of this box (torch copies of `mib` MiB, best of 3):
    the PCIe bound of the end-to-end leg."""
    nb = mib << 20
    d = torch.empty(nb, dtype=torch.uint8, device=dev_t)
    h = torch.empty(nb, dtype=torch.uint8).pin_memory()
    out = {}
    for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        best = 0.0
        for _ in range(3):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = max(best, nb / (time.perf_counter() - t0) / 1e9)
        out[name + "_GBs"] = best
    del d, h
    return out


def end_to_end(mat, rows_np, n_labels, dev_t, ref_hash, reps=3):
    """The drop-in path (SURVEY §8(d) 'also'): host row ids -> host CSR through
    mbrwt_get_rows (csrc/hostpipe.cpp: chunks of 2^20 rows, upload / query /
    download overlapped), on the bench's own batch, with caller buffers that
    are pageable (numpy: staged through pinned slots) and page-locked (torch
    pin_memory: DMA straight into them).  Best of `reps` calls after one
    warm-up; the CSR is hashed against the device-resident result."""
    import ctypes as C
    from genome_graph_annotation_amd import _lib as L
    n = len(rows_np)
    lib = L.lib()
    rates = pcie_rates(dev_t)
    bytes_in, bytes_out = 8 * n, 8 * (n + 1) + 4 * n_labels
    bound_s = max(bytes_in / (rates["h2d_GBs"] * 1e9), bytes_out / (rates["d2h_GBs"] * 1e9))
    out = {"rows": n, "labels": n_labels, "bytes_in": bytes_in, "bytes_out": bytes_out, "pcie": rates,
           "pcie_bound_ms": bound_s * 1e3, "pcie_bound_rows_per_s": n / bound_s}
    kinds = {
        "pageable": (rows_np, np.empty(n + 1, dtype=np.uint64), np.empty(n_labels, dtype=np.uint32)),
        "pinned": (torch.from_numpy(rows_np.view(np.int64)).pin_memory(),
                   torch.empty(n + 1, dtype=torch.int64).pin_memory(),
                   torch.empty(max(1, n_labels), dtype=torch.int32).pin_memory()),
    }
    for kind, (r, o, c) in kinds.items():
        def ptr(x, t):
            return C.cast(C.c_void_p(x.data_ptr() if kind == "pinned" else x.ctypes.data), C.POINTER(t))
        need = C.c_uint64(0)
        times = []
        for i in range(reps + 1):
            t0 = time.perf_counter()
            st = lib.mbrwt_get_rows(mat._h, ptr(r, C.c_uint64), n, ptr(o, C.c_uint64), ptr(c, C.c_uint32), n_labels,
                                    C.byref(need))
            dt = time.perf_counter() - t0
            if st != L.MBRWT_OK or need.value != n_labels:
                raise RuntimeError(f"end-to-end mbrwt_get_rows ({kind}): status {st}, labels {need.value}")
            if i:
                times.append(dt)
        oh = o.numpy().view(np.uint64) if kind == "pinned" else o
        ch = c.numpy().view(np.uint32)[:n_labels] if kind == "pinned" else c
        best = min(times)
        h = csr_hash(oh, ch)
        out[kind] = {"ms": best * 1e3, "rows_per_s": n / best, "d2h_GBs": bytes_out / best / 1e9,
                     "vs_pcie_bound": best / bound_s, "csr_hash": h, "bit_exact_vs_device": h == ref_hash,
                     "ms_all": [t * 1e3 for t in times]}
    del kinds
    return out


def main():
    a = parse()
    if a.pmc_pass:
        pmc_pass(a)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    local = local % max(1, ndev)  # (rehearsal only: several ranks may share one GPU under gloo)

    from genome_graph_annotation_amd import BRWTDevice, _lib as L
    from genome_graph_annotation_amd.brwt import build_option
    from genome_graph_annotation_amd.dist import AllGatherV, DeviceAllGatherV, shard_bounds

    # roofline traffic first: the PMC child passes need the GPU's memory for
    # their own copy of the structure
    kernel_re = None
    traffic = None
    if rank == 0 and world == 1 and a.traffic != "off":
        if a.layout in ("rows", "both") and a.kernel == 0:
            kernel_re = "k_traverse_rows|k_var_decode"
        else:
            kernel_re = "k_traverse_(p2w|fast2)" if a.kernel == 0 or 17 <= a.kernel <= 23 else "k_traverse"
        if a.traffic == "live":
            traffic = live_traffic(a, kernel_re)
            if traffic is not None and a.traffic_out:
                with open(a.traffic_out, "w") as f:
                    json.dump(traffic, f, indent=1)
        if traffic is None:
            traffic = committed_traffic(a, kernel_re)

    size_group = None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            # the all-gatherv's sizes travel as host integers over gloo (no
            # device read-back in the step: dist.AllGatherV)
            size_group = dist.new_group(backend="gloo")
        else:
            dist.init_process_group(a.dist_backend)
    else:
        torch.cuda.set_device(local)

    dev_t = torch.device("cuda", local)
    t0 = time.time()
    with build_option(L.MBRWT_BUILD_ROWS_CODE, a.rows_code), build_option(L.MBRWT_BUILD_ROWS_BLOCK, rows_block_opt(a)):
        mat = BRWTDevice.synthetic(a.rows, a.cols, a.density, a.arity, a.seed, device=local, layout=a.layout)
    setup_s = time.time() - t0
    struct_bytes = mat.device_bytes()
    log(f"device structure built in {setup_s:.1f} s ({mat.device_bytes() / 1e9:.1f} GB, layout {mat.layout()}, "
        f"{mat.rows_stats()})")
    if a.kernel:
        mat.set_option(L.MBRWT_OPT_KERNEL, a.kernel)

    # K distinct global batches (batch k: seed + k; batch 0 is the r01/r02
    # batch) and this rank's contiguous slice of each; timed step i queries
    # batch i mod K, so no timed step replays the previous step's rows
    G = a.batch if a.scaling == "strong" else a.batch * world
    K = max(1, a.batches)
    lo, hi = shard_bounds(G, world, rank)
    nb = hi - lo
    globals_np = [np.random.default_rng(a.seed + k).integers(0, a.rows, G, dtype=np.uint64) for k in range(K)]
    rows_ts = [torch.from_numpy(np.ascontiguousarray(g[lo:hi]).view(np.int64)).to(dev_t) for g in globals_np]
    off_t = torch.empty(nb + 1, dtype=torch.int64, device=dev_t)
    stream = torch.cuda.current_stream(dev_t)
    sptr = stream.cuda_stream
    # size the label buffer once (capacity protocol), outside the timed region
    probe = torch.empty(1, dtype=torch.int32, device=dev_t)
    need = 0
    for rt in rows_ts:
        try:
            nk = mat.get_rows_device(rt, off_t, probe, sptr)
        except L.MBRWTError as e:
            if e.status != L.MBRWT_ERR_CAPACITY:
                raise
            nk = e.needed
        need = max(need, nk)
    cols_t = torch.empty(int(need * 1.02) + 1024, dtype=torch.int32, device=dev_t)
    wire = None
    if world > 1 and not a.no_gather and not a.host_sizes:
        # the device-sized all-gatherv: every rank's wire segment holds up to
        # labels_cap labels -- this rank's sizing (max over its batches); the
        # constructor agrees on the largest over the ranks and checks that
        # every rank passed the same slices (dist._agree_wire)
        rows_per_rank = [shard_bounds(G, world, r)[1] - shard_bounds(G, world, r)[0] for r in range(world)]
        # 3 slots: up to 2 exchanges in flight behind the current step, so
        # step k's pack + all-gather (RCCL stream) and step k-1's unpack (side
        # stream) overlap instead of chaining through the main stream
        wire = DeviceAllGatherV(rows_per_rank, int(need * 1.02) + 1024, a.cols, dev_t, timing=True, slots=3)

    # N > 1: steps are pipelined -- batch k's all-gatherv (RCCL stream) runs
    # while batch k+1 is traversed, so the outputs are double-buffered; drain()
    # completes the last exchange inside the timed region
    gather = world > 1 and not a.no_gather
    state = {"i": 0, "pending": None, "inflight": [], "global": None, "timed": False, "exchanges": [],
             "get_rows_host": []}

    # N = 1: the asynchronous call (include/mbrwt.h mbrwt_get_rows_device_async:
    # no host synchronisation per step; the status block -- labels, status,
    # sticky status bits -- is read once after the timed region)
    use_async = (world == 1 or wire is not None) and not a.sync
    status_t = torch.zeros(3, dtype=torch.int64, device=dev_t)
    # two query streams (N = 1 and, since r05, N > 1): batch i runs on query
    # context i mod 2 (the context, or a clone over the same image) on its own
    # stream, into its own output buffers and status block, so batch i+1's
    # traversal runs beside batch i's compaction (and, at N > 1, beside its
    # pack; the all-gather and the unpack run on RCCL's and a side stream)
    Q = a.query_streams if use_async else 1
    qmats, qstreams, qstatus = [mat], [stream], [status_t]
    for _ in range(Q - 1):
        qmats.append(mat.clone())
        qstreams.append(torch.cuda.Stream(dev_t))
        qstatus.append(torch.zeros(3, dtype=torch.int64, device=dev_t))
    if a.compact_cus:
        for qm in qmats:
            qm.set_option(L.MBRWT_OPT_COMPACT_CUS, a.compact_cus)
    # outputs: step i writes bufs[i mod len]; with two buffers a buffer's next
    # writer is two steps later on the SAME stream, behind this step's readers
    # (its compaction, its pack) -- double-buffered whenever steps overlap
    # (Q streams: buffer i mod Q is written only by stream i mod Q)
    bufs = [(off_t, cols_t)]
    for _ in range(max(Q, 2 if gather else 1) - 1):
        bufs.append((torch.empty_like(off_t), torch.empty_like(cols_t)))

    def step():
        i = state["i"]
        o, cb = bufs[i % len(bufs)]
        state["i"] += 1
        h0 = time.perf_counter()
        if use_async:
            q = i % Q
            with torch.cuda.stream(qstreams[q]):
                qmats[q].get_rows_device_async(rows_ts[i % K], o, cb, qstatus[q], qstreams[q].cuda_stream)
                if state["timed"]:
                    state["get_rows_host"].append((time.perf_counter() - h0) * 1e3)
                if wire is not None:
                    # no host synchronisation: the label count travels from the
                    # status block on the device into the wire header; the
                    # pack runs on this query's stream.  The oldest exchange is
                    # finished only when its slot comes round again
                    if len(state["inflight"]) == len(wire.slots) - 1:
                        state["global"] = wire.finish(state["inflight"].pop(0))
                    state["inflight"].append(wire.start(o, cb, qstatus[q]))
            return None
        n_lab = mat.get_rows_device(rows_ts[i % K], o, cb, sptr)
        if state["timed"]:
            state["get_rows_host"].append((time.perf_counter() - h0) * 1e3)
        if gather:
            if state["pending"] is not None:
                state["global"] = state["pending"].finish()
            state["pending"] = AllGatherV(o, cb, n_labels=n_lab, num_columns=a.cols, size_group=size_group,
                                          timing=state["timed"])
            if state["timed"]:
                state["exchanges"].append(state["pending"])
        return n_lab

    def drain():
        while state["inflight"]:
            state["global"] = wire.finish(state["inflight"].pop(0))
        if state["pending"] is not None:
            state["global"] = state["pending"].finish()
            state["pending"] = None

    for _ in range(a.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    if wire is not None:
        wire.last_phases = []
    for qi, qm in enumerate(qmats):
        qm.take_timing()
        if a.kernel_timing == "all" or (a.kernel_timing == "first" and qi == 0):
            qm.set_option(L.MBRWT_OPT_TIMING, 1)
    state["timed"] = True
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        n_lab = step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    state["timed"] = False
    if use_async:
        for q, st in enumerate(qstatus):
            need_l, st_l, sticky = st.cpu().tolist()
            if sticky != 1 << L.MBRWT_OK:
                raise RuntimeError(f"asynchronous get_rows reported status bits {sticky:#x} (last status {st_l})")
            if q == (state["i"] - 1) % Q:  # the last step's context
                n_lab = int(need_l)
    log(f"timed {a.steps} steps: {elapsed / a.steps * 1e3:.3f} ms/step")

    kern_ms_total, launches = 0.0, 0
    for qm in qmats:
        qm.set_option(L.MBRWT_OPT_TIMING, 0)
        km, kl = qm.take_timing()
        kern_ms_total += km
        launches += kl
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev_t)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    last_k = (state["i"] - 1) % K
    rows_global = globals_np[last_k]
    rows_t = rows_ts[last_k]

    # per-phase times of the multi-GPU step (this rank; max over ranks below)
    phases = None
    if world > 1:
        ph = {"traverse_kernel_ms": kern_ms_total / max(1, launches),
              "get_rows_host_ms": float(np.mean(state["get_rows_host"])) if state["get_rows_host"] else None}
        if state["exchanges"]:
            ex = [x.phases() for x in state["exchanges"]]
            for k in ex[0]:
                ph[k] = float(np.mean([e[k] for e in ex]))
            ph["wire_bytes_sent_per_rank"] = int(state["exchanges"][-1].wire_bytes)
            ph["wire_bytes_received_per_rank"] = int(state["exchanges"][-1].wire_bytes) * (world - 1)
        if wire is not None:
            ph.update(wire.phases())
            ph["sizes_host_ms"] = 0.0  # (device-side sizes: no host exchange)
            ph["wire_bytes_sent_per_rank"] = int(wire.wire_bytes)
            ph["wire_bytes_received_per_rank"] = int(wire.wire_bytes) * (world - 1)
        keys = sorted(k for k, v in ph.items() if v is not None)
        t = torch.tensor([float(ph[k]) for k in keys], dtype=torch.float64, device=dev_t)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        phases = {k: float(v) for k, v in zip(keys, t.tolist())}
        phases["note"] = ("max over ranks of each rank's mean over the timed steps; device times from HIP events "
                          "on the streams that run them; host_ms are wall times of the host calls")
        state["exchanges"] = []

    last_off, last_cols = bufs[(state["i"] - 1) % len(bufs)]
    # the global CSR of the last timed step: this rank's slice (N = 1) or the
    # all-gathered CSR every rank holds (N > 1)
    reassembly = None
    if gather:
        if wire is not None:
            g_off, g_cols, g_st = state["global"]
            tot, bad = g_st.tolist()
            if bad or tot != int(g_off[-1].item()):
                raise RuntimeError(f"device all-gatherv status: total {tot}, overflow flag {bad}, "
                                   f"offsets end {int(g_off[-1].item())}")
            g_cols = g_cols[:tot]
        else:
            g_off, g_cols = state["global"]
        b0 = int(g_off[lo].item())
        ok = bool(torch.equal(g_off[lo:hi + 1] - b0, last_off) and
                  torch.equal(g_cols[b0:b0 + n_lab], last_cols[:n_lab]) and g_off.numel() == G + 1)
        flag = torch.tensor([0 if ok else 1], dtype=torch.int64, device=dev_t)
        dist.all_reduce(flag, op=dist.ReduceOp.SUM)
        reassembly = (f"all-gatherv CSR ({g_off.numel() - 1:,} rows, {g_cols.numel():,} labels) holds every "
                      f"rank's slice verbatim" if int(flag.item()) == 0 else f"MISMATCH on {int(flag.item())} ranks")
        glob_off, glob_cols = g_off, g_cols
    else:
        glob_off, glob_cols = last_off, last_cols[:n_lab]
    chk = min(a.check_rows, G) if a.check_rows > 0 else G
    have_global = world == 1 or gather
    if rank == 0 and have_global:
        off_h = glob_off[: chk + 1].cpu().numpy().view(np.uint64)
        cols_h = glob_cols[: int(off_h[-1])].cpu().numpy().view(np.uint32)
    if gather:
        del g_off, g_cols, glob_off, glob_cols
        state["global"] = None

    # two query streams: the traversal's HIP-event time above includes the
    # other stream's compaction running beside it; the same kernel timed
    # alone (one context, one stream, untimed for `value`) is reported
    # beside the roofline as `isolated`
    iso = None
    if Q >= 2:
        for _ in range(3):
            mat.get_rows_device_async(rows_ts[0], off_t, cols_t, status_t, sptr)
        torch.cuda.synchronize()
        mat.take_timing()
        mat.set_option(L.MBRWT_OPT_TIMING, 1)
        iso_steps = 20
        t1 = time.perf_counter()
        for i in range(iso_steps):
            mat.get_rows_device_async(rows_ts[i % K], off_t, cols_t, status_t, sptr)
        torch.cuda.synchronize()
        iso_wall = (time.perf_counter() - t1) / iso_steps * 1e3
        mat.set_option(L.MBRWT_OPT_TIMING, 0)
        ikm, ikl = mat.take_timing()
        iso = {"kernel_ms": ikm / max(1, ikl), "ms_per_step": iso_wall, "steps": iso_steps}

    # N > 1: the same steps WITHOUT the all-gatherv (each rank keeps its
    # slice: the traversal alone, no data-path collective), timed the same way
    # right after, so the driver's SCALE lines carry both curves (VERDICT r05
    # #4); `value` stays the gathered figure (SURVEY §8(e)'s contract)
    no_gather = None
    if world > 1 and gather:
        for q in range(Q):
            qstatus[q].zero_()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(a.steps):
            o, cb = bufs[i % len(bufs)]
            if use_async:
                q = i % Q
                with torch.cuda.stream(qstreams[q]):
                    qmats[q].get_rows_device_async(rows_ts[i % K], o, cb, qstatus[q], qstreams[q].cuda_stream)
            else:
                mat.get_rows_device(rows_ts[i % K], o, cb, sptr)
        torch.cuda.synchronize()
        dist.barrier()
        ng = time.perf_counter() - t1
        tt = torch.tensor([ng], dtype=torch.float64, device=dev_t)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        ng = float(tt.item())
        no_gather = {"value": G * a.steps / ng, "unit": "rows/s", "ms_per_step": ng / a.steps * 1e3,
                     "steps": a.steps,
                     "note": "the same global batches and steps without the all-gatherv (every rank keeps its own "
                             "slice's CSR), timed after the gathered steps and their parity read-back: barrier + synchronize on both "
                             "sides, max over ranks; not `value` (the contract reassembles every row on every rank)"}
        if use_async:
            for q in range(Q):
                if qstatus[q][2].item() != 1 << L.MBRWT_OK:
                    raise RuntimeError(f"no-gather steps reported status bits {int(qstatus[q][2].item()):#x}")
        log(f"no-gather: {no_gather['ms_per_step']:.3f} ms/step")

    # measured ceilings of this GPU (streaming read; random 64-/128-B requests)
    stream_gbs = rnd = None
    if rank == 0 and not a.no_probe:
        free, _ = torch.cuda.mem_get_info(dev_t)
        stream_gbs, rnd = probe_ceilings(dev_t, sptr, free, struct_bytes)

    # exact work accounting for the algorithmic roofline (untimed diagnostic pass)
    try:
        visits, labels = mat.count_work_device(rows_t, sptr)
    except L.MBRWTError:  # terminal records (--rows-code 2) store no internal masks: no V accounting
        visits, labels = None, n_lab
    assert labels == n_lab, (labels, n_lab)
    # SURVEY §8(d)'s per-row figure: 64 B per index-bit probe of the
    # reference recursion (BRWT.cpp:30) + row id + offset + 4 B per label --
    # "probe-equivalent": the layouts answer a row without those probes
    probe_bytes = 64 * visits + 16 * nb + 4 * labels if visits is not None else None
    kern_ms = kern_ms_total / max(1, launches)
    # the roofline's kernel time must fit inside the step:
    # with two query streams the HIP events around one traversal also span
    # the other stream's compaction running beside it, so the kernel timed
    # alone on one stream (the isolated pass) is the roofline's time and the
    # overlapped event time is reported beside it
    kern_ms_overlapped = kern_ms if Q >= 2 else None
    if iso is not None:
        kern_ms = iso["kernel_ms"]
    kname = mat.traverse_kernel()
    rstats = mat.rows_stats()

    cpu = None
    parity = None
    if rank == 0 and have_global and not a.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU baseline and parity legs only

        nproc = os.cpu_count()
        share = len(os.sched_getaffinity(0))
        omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
        threads = a.cpu_threads or (min(share, omp) if omp > 0 else share)
        # the RefSeq shape's plain index bits (158 GB) are not built on the
        # host: its parity streams the same tree (oracle.topdown_get_rows,
        # tests/test_full_size.py) and it has no CPU-baseline structure
        streamed = a.rows * a.cols * a.density > 6e10
        ref = None
        if streamed:
            log(f"streaming the host oracle on {threads} threads; checking {chk:,} rows")
            g0 = time.time()
            off_o, cols_o = O.topdown_get_rows(a.rows, a.cols, a.density, a.arity, a.seed, rows_global[:chk], threads)
            gen_s = time.time() - g0
        else:
            log(f"building the host oracle structure on {threads} threads")
            g0 = time.time()
            ref = O.OracleTree.topdown(a.rows, a.cols, a.density, a.arity, a.seed, threads)
            gen_s = time.time() - g0
            log(f"host structure built in {gen_s:.1f} s; checking {chk:,} rows")
            off_o, cols_o = ref.get_rows(rows_global[:chk], threads)
        exact = bool(np.array_equal(off_o, off_h) and np.array_equal(cols_o, cols_h))
        parity = {"rows_checked": chk, "labels_checked": int(len(cols_o)), "bit_exact": exact,
                  "csr_hash_gpu": csr_hash(off_h, cols_h), "csr_hash_oracle": csr_hash(off_o, cols_o),
                  "scope": ("the whole global batch" if chk == G else f"the first {chk:,} rows of the global batch")
                           + f" of the last timed step (batch {last_k}, seed {a.seed + last_k})"
                           + (f", reassembled by the all-gatherv from {world} ranks" if world > 1 else "")}
        if streamed:
            parity["oracle"] = f"streamed top-down oracle ({gen_s:.0f} s on {threads} threads)"
        del off_o, cols_o
        if world == 1 and ref is not None:
            def timed(n_rows, th):
                sample = rows_global[:n_rows]
                c0 = time.perf_counter()
                ref.time_rows(sample, th)
                return len(sample) / (time.perf_counter() - c0)
            plain = timed(a.cpu_sample, threads)
            plain1 = timed(a.cpu_sample_1t, 1)
            c0 = time.time()
            ref.to_rrr(threads)  # the reference's bit_vector_rrr<63> cost profile
            rrr_s = time.time() - c0
            rrr = timed(a.cpu_sample // 10, threads)
            rrr1 = timed(a.cpu_sample_1t // 10, 1)
            cpu = {"value": rrr, "unit": "rows/s", "cores": threads, "kind": "port",
                   "sample": f"first {a.cpu_sample // 10:,} rows of the batch on the same {a.rows:,} x {a.cols:,} "
                             f"structure: the oracle's restatement of BRWT::get_row over sdsl-RRR-like index "
                             f"vectors (63-bit blocks, class + combinatorial number, samples every 32 blocks: "
                             f"bit_vector_rrr<63>'s cost profile; host build {gen_s:.0f} s + RRR encode "
                             f"{rrr_s:.0f} s); {threads} threads = the job's CPU share (OMP_NUM_THREADS "
                             f"{omp or 'unset'}, affinity {share}; the node's nproc {nproc} is shared by 8 GPU jobs)",
                   "single_thread": {"value": rrr1, "unit": "rows/s", "cores": 1,
                                     "sample": f"first {a.cpu_sample_1t // 10:,} rows, RRR-like"},
                   "plain_rank": {"value": plain, "unit": "rows/s", "cores": threads,
                                  "sample": f"first {a.cpu_sample:,} rows, plain bit vectors + rank samples"},
                   "plain_rank_single_thread": {"value": plain1, "unit": "rows/s", "cores": 1,
                                                "sample": f"first {a.cpu_sample_1t:,} rows"},
                   "nproc": nproc}
        del ref

    # the drop-in path end to end (host ids -> host CSR), N = 1, rank 0
    e2e = None
    if rank == 0 and world == 1 and have_global and not a.no_e2e:
        dev_hash = csr_hash(off_h, cols_h)
        e2e = end_to_end(mat, np.ascontiguousarray(rows_global[:chk]), int(off_h[-1]), dev_t, dev_hash)
        e2e["scope"] = (f"the bench's batch {last_k} ({chk:,} rows) through mbrwt_get_rows; csr_hash compared with the "
                        f"device-resident CSR of the same batch (itself checked against the oracle: parity)")
        log(f"end-to-end: pageable {e2e['pageable']['ms']:.2f} ms, pinned {e2e['pinned']['ms']:.2f} ms, "
            f"PCIe bound {e2e['pcie_bound_ms']:.2f} ms")

    # roofline of the dominant kernel: its layout-true algorithmic bytes per
    # launch (the bytes the layout must move: DESIGN.md §6) / its HIP-event
    # time (achieved, frac); the measured HBM traffic beside it (traffic,
    # traffic_frac); SURVEY §8(d)'s probe-equivalent figure labelled as such
    ks = kern_ms / 1e3
    alg_bytes, alg_basis = None, None
    if rstats is not None and not rstats.get("variable"):
        B = rstats["block_bytes"]
        tiles = (nb + 63) // 64
        spf = rstats["spilled_rows"] / a.rows
        # row id + block + spill reload (spilled rows) read; count + u16 label
        # per label + tile count written into the tile regions
        alg_bytes = nb * (8 + B + 2) + nb * spf * B + 2 * labels + 4 * tiles
        alg_basis = (f"k_traverse_rows: per row 8 B id + {B} B block + 2 B count, {B} B per spilled row "
                     f"({spf:.4f} of rows), 2 B per label (u16 temp), 4 B per 64-row tile")
    elif rstats is not None:
        rec = rstats["record_bytes"] / a.rows
        # loc + count + CSR offset read per row, the record's whole 16-byte
        # chunks (~ record + 12 B), 4 B per label written into the CSR
        alg_bytes = nb * (8 + 4 + 8 + rec + 12) + 4 * labels
        alg_basis = (f"k_var_decode: per row 20 B (locate output, CSR offset) + {rec:.1f} B record + ~12 B "
                     f"16-byte-chunk rounding; 4 B per label written into the CSR")
    roof = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "kernel": kname, "kernel_ms": kern_ms,
            "kernel_ms_basis": ("HIP events around the kernel on its own stream, one context, no other batch beside "
                                "it (the isolated pass after the timed region)" if iso is not None else
                                "HIP events around the kernel in the timed region"),
            "kernel_ms_overlapped": kern_ms_overlapped,
            "step_minus_kernel_ms": elapsed / a.steps * 1e3 - kern_ms if world == 1 else None,
            "step_implied_frac": (alg_bytes / (elapsed / a.steps) / 1e9 / HBM_PEAK_GBS
                                  if alg_bytes and world == 1 else None),
            "achieved": alg_bytes / ks / 1e9 if alg_bytes else None,
            "frac": alg_bytes / ks / 1e9 / HBM_PEAK_GBS if alg_bytes else None,
            "alg_bytes_per_launch": alg_bytes, "alg_basis": alg_basis, "traffic": None,
            "probe_equivalent": ({"bytes_per_launch": probe_bytes, "achieved": probe_bytes / ks / 1e9,
                                  "frac": probe_bytes / ks / 1e9 / HBM_PEAK_GBS,
                                  "note": "SURVEY §8(d): 64 B x V + 16 + 4 L per row, V = index-bit probes of the "
                                          "reference recursion; the row-record layouts issue none of these probes"}
                                 if probe_bytes is not None else None),
            "visits_per_row": visits / max(1, nb) if visits is not None else None,
            "labels_per_row": labels / max(1, nb),
            "stream_read_measured": stream_gbs}
    if iso is not None:
        iks = iso["kernel_ms"] / 1e3
        iso.update({"step_minus_kernel_ms": iso["ms_per_step"] - iso["kernel_ms"],
                    "note": "the kernel with one context on one stream (no other batch beside it), 20 "
                            "untimed-for-value steps after the timed region: roofline.kernel_ms / achieved / frac "
                            "are computed from this time; kernel_ms_overlapped is the HIP-event time in the timed "
                            "region, where batch k+1's traversal runs beside batch k's compaction"})
        roof["isolated"] = iso
    seg = 64
    if rstats is not None and not rstats.get("variable"):
        seg = rstats["block_bytes"]
        roof["row_records"] = dict(rstats, spilled_fraction=rstats["spilled_rows"] / a.rows)
        # one block per row, plus one spill entry per spilled row
        roof["block_requests_per_launch"] = nb * (1.0 + rstats["spilled_rows"] / a.rows)
        roof["block_requests_per_s"] = roof["block_requests_per_launch"] / ks
    elif rstats is not None:
        roof["row_records"] = rstats
    if traffic is not None and world == 1:
        tb = traffic["traffic_bytes"]
        if alg_bytes is None:  # (node images: the measured bytes stand in)
            roof.update({"achieved": tb / ks / 1e9, "frac": tb / ks / 1e9 / HBM_PEAK_GBS,
                         "alg_basis": "measured traffic (node-image kernels)"})
        roof.update({"traffic_achieved": tb / ks / 1e9, "traffic_frac": tb / ks / 1e9 / HBM_PEAK_GBS, "traffic": tb,
                     "read_bytes": traffic["read_bytes"], "write_bytes": traffic["write_bytes"],
                     "traffic_source": traffic.get("source", "live rocprofv3 --pmc passes of this run") +
                                       f" (sources {traffic['source_hash']})"})
        req = traffic["read_bytes"] / 64.0  # FETCH_SIZE in 64-byte units (calibrated on random 64-B segments)
        roof["read_requests_per_launch"] = req
        roof["read_requests_per_s"] = req / ks
    # first-class keys: the physical read fraction, and how
    # close the block requests run to the measured random-request ceiling --
    # the binding limit of this layout: one random request per row caps the
    # read fraction at ceiling x segment / peak (about 0.38-0.39 at 64 B)
    if traffic is not None and world == 1:
        roof["read_frac"] = traffic["read_bytes"] / ks / 1e9 / HBM_PEAK_GBS
    if rnd is not None and rnd.get(f"seg{seg}_per_s"):
        ceil = rnd[f"seg{seg}_per_s"]
        roof["read_frac_cap_by_request_ceiling"] = ceil * seg / 1e9 / HBM_PEAK_GBS
        if "block_requests_per_launch" in roof:
            roof["request_ceiling_frac"] = roof["block_requests_per_launch"] / ks / ceil
        elif "read_requests_per_launch" in roof:
            roof["request_ceiling_frac"] = roof["read_requests_per_launch"] / ks / ceil
    if rnd is not None:
        roof["ceiling_random64_per_s"] = rnd.get("seg64_per_s")
        roof["ceiling_random128_per_s"] = rnd.get("seg128_per_s")
        roof["ceiling_sweep_best"] = {k: v for k, v in rnd.items() if k.endswith("_best")}
        ceil = rnd.get(f"seg{seg}_per_s")
        if rstats is not None and not rstats.get("variable") and ceil:
            roof[f"ceiling_random{seg}_frac"] = roof["block_requests_per_s"] / ceil
            if iso is not None:
                iso[f"ceiling_random{seg}_frac"] = roof["block_requests_per_launch"] / (iso["kernel_ms"] / 1e3) / ceil
        elif traffic is not None and world == 1 and ceil:
            roof["ceiling_random64_frac"] = roof["read_requests_per_s"] / ceil
            if iso is not None:
                iso["ceiling_random64_frac"] = roof["read_requests_per_launch"] / (iso["kernel_ms"] / 1e3) / ceil

    value = G * a.steps / elapsed
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "rows/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": a.scaling,
        "vs_baseline": None,
        "dtype": "u32/u64",
        "data": f"synthetic (top-down i.i.d. Bernoulli columns, seed {a.seed}; {K} batches of uniform random rows, "
                f"seeds {a.seed}..{a.seed + K - 1}, rotated over the steps)",
        "config": {
            "workload": f"Multi-BRWT {a.rows:,} x {a.cols:,}, d={a.density}, arity {a.arity} "
                        f"({a.workload}: BASELINE configs[{ {'c2': 1, 'c3': 2, 'c4': 3}[a.workload] }]); "
                        f"global batch {G:,} rows, {nb:,} per GPU ({a.scaling} scaling)",
            "num_rows": a.rows, "num_columns": a.cols, "density": a.density, "arity": a.arity,
            "global_batch": G, "batch_per_gpu": nb, "batches": K, "layout": a.layout,
            "api": "mbrwt_get_rows_device_async" if use_async else "mbrwt_get_rows_device",
            "query_streams": Q,
            "rows_code": {0: "auto", 1: "nibble", 2: "terminal", 3: "byte"}[a.rows_code],
            **({"rows_block": a.rows_block} if a.rows_block else {}),
            "records": ("terminal" if rstats and rstats.get("terminal_records") else
                        "nibble" if rstats and rstats.get("nibble_codes") else "byte"),
            **({"compact_cus_of_32": a.compact_cus} if a.compact_cus else {}),
            "parallelism": f"batch-sharded x{world}, tree replicated" + ("" if world == 1 or a.no_gather
                                                                         else ", all-gatherv over " + ("RCCL" if a.dist_backend == "nccl" else a.dist_backend)
                                                                         + (" (device-sized wire, no host sync)" if wire is not None else " (host-sized)")),
            "structure_bytes": struct_bytes,
            "setup_s": round(setup_s, 2),
        },
        "roofline": roof,
        "phases": phases,
        "end_to_end": e2e,
        "cpu_baseline": cpu,
        "no_gather": no_gather,
        "reassembly": reassembly,
        "parity": parity,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
