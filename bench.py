"""bench.py -- get_rows()/s on a Kingsford-shaped Multi-BRWT (BASELINE.json).

Workload (config.workload): BASELINE.json configs[3] shape on one GPU per rank
-- a 3.7 B x 2,652 Multi-BRWT (i.i.d. d = 0.3 % columns, basic arity-8
partitioner, generated top-down on the device: DESIGN.md "Synthetic
matrices"), replicated on every GPU; each rank queries its own 8 M-row batch
(uniform 64-bit row ids, seed 42 + rank).  One step = one batched get_rows
over the rank's batch, device-resident row ids -> CSR in HBM, plus (N > 1)
the RCCL all-gatherv that reassembles the global CSR on every rank.

Prints ONE JSON line (rank 0).  roofline: algorithmic bytes of the traversal
kernel per launch (64 B x V + 8 + 8 + 4 B x L per row, V and
L counted exactly on the device for the batch) / its HIP-event-timed average
duration.  cpu_baseline: the oracle's restatement of BRWT::get_row on the
same structure (generated on the host from the same spec), timed on a bounded
row sample on all host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "get_rows()/s on Multi-BRWT, 3.7B×2,652 Kingsford-shape @1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip-level table (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", type=int, default=3_700_000_000)
    ap.add_argument("--cols", type=int, default=2652)
    ap.add_argument("--density", type=float, default=0.003)
    ap.add_argument("--arity", type=int, default=8)
    ap.add_argument("--batch", type=int, default=8_000_000, help="query rows per GPU")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the all-gatherv reassembly")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--cpu-sample", type=int, default=400_000, help="rows timed on the CPU")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = all host cores")
    ap.add_argument("--check-rows", type=int, default=0,
                    help="GPU rows checked element-wise against the oracle (0 = the whole batch)")
    ap.add_argument("--kernel", type=int, default=0, help="MBRWT_OPT_KERNEL variant (0 = library default)")
    ap.add_argument("--dist-backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    return ap.parse_args()


def committed_traffic(cfg):
    """Per-launch HBM traffic of the traversal kernel from the committed PMC
    summary of this exact workload (profiles/*/traffic_*.json, written by
    tools/pmc_traffic.py from separate rocprofv3 --pmc passes of this script),
    or None when no summary matches."""
    import glob
    hit = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic_*.json"))):
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        if {k: str(v) for k, v in cfg.items()} == {k: str(v) for k, v in t.get("config", {}).items()}:
            hit = (t["traffic_bytes"], os.path.relpath(path, ROOT))
    return hit


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    local = local % max(1, ndev)  # (rehearsal only: several ranks may share one GPU under gloo)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(a.dist_backend)
    else:
        torch.cuda.set_device(local)
    from genome_graph_annotation_amd import BRWTDevice, _lib as L
    from genome_graph_annotation_amd.dist import AllGatherV, allgatherv_csr

    dev_t = torch.device("cuda", local)
    t0 = time.time()
    mat = BRWTDevice.synthetic(a.rows, a.cols, a.density, a.arity, a.seed, device=local)
    setup_s = time.time() - t0
    log(f"device structure built in {setup_s:.1f} s ({mat.device_bytes() / 1e9:.1f} GB)")
    if a.kernel:
        mat.set_option(L.MBRWT_OPT_KERNEL, a.kernel)

    rows_np = np.random.default_rng(a.seed + 1000 * rank).integers(0, a.rows, a.batch, dtype=np.uint64)
    rows_t = torch.from_numpy(rows_np.view(np.int64)).to(dev_t)
    off_t = torch.empty(a.batch + 1, dtype=torch.int64, device=dev_t)
    stream = torch.cuda.current_stream(dev_t)
    sptr = stream.cuda_stream
    # size the label buffer once (capacity protocol), outside the timed region
    probe = torch.empty(1, dtype=torch.int32, device=dev_t)
    try:
        need = mat.get_rows_device(rows_t, off_t, probe, sptr)
    except L.MBRWTError as e:
        if e.status != L.MBRWT_ERR_CAPACITY:
            raise
        need = e.needed
    cols_t = torch.empty(int(need * 1.02) + 1024, dtype=torch.int32, device=dev_t)

    # N > 1: steps are pipelined -- batch k's all-gatherv (RCCL stream) runs
    # while batch k+1 is traversed, so the outputs are double-buffered; drain()
    # completes the last exchange inside the timed region
    gather = world > 1 and not a.no_gather
    bufs = [(off_t, cols_t)]
    if gather:
        bufs.append((torch.empty_like(off_t), torch.empty_like(cols_t)))
    state = {"i": 0, "pending": None}

    def step():
        o, cb = bufs[state["i"] % len(bufs)]
        state["i"] += 1
        n_lab = mat.get_rows_device(rows_t, o, cb, sptr)
        if gather:
            if state["pending"] is not None:
                state["pending"].finish()
            state["pending"] = AllGatherV(o, cb, n_labels=n_lab, num_columns=a.cols)
        return n_lab

    def drain():
        if state["pending"] is not None:
            state["pending"].finish()
            state["pending"] = None

    for _ in range(a.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    mat.take_timing()
    mat.set_option(L.MBRWT_OPT_TIMING, 1)
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
    log(f"timed {a.steps} steps: {elapsed / a.steps * 1e3:.3f} ms/step")
    mat.set_option(L.MBRWT_OPT_TIMING, 0)
    kern_ms_total, launches = mat.take_timing()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev_t)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # N > 1: the reassembled global CSR must hold this rank's slice verbatim
    # (every rank checks its own slice; the verdicts are all-reduced)
    reassembly = None
    last_off, last_cols = bufs[(state["i"] - 1) % len(bufs)]
    if gather:
        g_off, g_cols = allgatherv_csr(last_off, last_cols, n_labels=n_lab, num_columns=a.cols)
        lo, hi = rank * a.batch, (rank + 1) * a.batch
        b0 = int(g_off[lo].item())
        ok = bool(torch.equal(g_off[lo:hi + 1] - b0, last_off) and
                  torch.equal(g_cols[b0:b0 + n_lab], last_cols[:n_lab]) and
                  g_off.numel() == world * a.batch + 1)
        flag = torch.tensor([0 if ok else 1], dtype=torch.int64, device=dev_t)
        dist.all_reduce(flag, op=dist.ReduceOp.SUM)
        reassembly = (f"all-gatherv CSR ({g_off.numel() - 1:,} rows, {g_cols.numel():,} labels) holds every "
                      f"rank's slice verbatim" if int(flag.item()) == 0 else f"MISMATCH on {int(flag.item())} ranks")
        del g_off, g_cols

    # measured streaming-read rate of this GPU (report beside the spec peak)
    big = torch.ones(1 << 30, dtype=torch.float32, device=dev_t)  # 4 GiB
    big.sum()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        big.sum()
    e1.record()
    torch.cuda.synchronize()
    stream_gbs = 5 * big.numel() * 4 / (e0.elapsed_time(e1) / 1e3) / 1e9
    del big

    # exact work accounting for the roofline (untimed diagnostic pass)
    visits, labels = mat.count_work_device(rows_t, sptr)
    assert labels == n_lab, (labels, n_lab)
    alg_bytes = 64 * visits + 16 * a.batch + 4 * labels
    kern_ms = kern_ms_total / max(1, launches)
    achieved = alg_bytes / (kern_ms / 1e3) / 1e9

    # GPU result of the last timed step for the parity gate
    chk = min(a.check_rows, a.batch) if a.check_rows > 0 else a.batch
    off_h = last_off[: chk + 1].cpu().numpy().view(np.uint64)
    cols_h = last_cols[: int(off_h[-1])].cpu().numpy().view(np.uint32)

    cpu = None
    parity = None
    if rank == 0 and world == 1 and not a.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU baseline leg only

        threads = a.cpu_threads or len(os.sched_getaffinity(0))
        threads = min(threads, 16)
        log(f"building the host oracle structure on {threads} threads")
        g0 = time.time()
        ref = O.OracleTree.topdown(a.rows, a.cols, a.density, a.arity, a.seed, threads)
        gen_s = time.time() - g0
        log(f"host structure built in {gen_s:.1f} s; checking {chk} rows and timing {a.cpu_sample} rows")
        off_o, cols_o = ref.get_rows(rows_np[:chk], threads)
        parity = bool(np.array_equal(off_o, off_h) and np.array_equal(cols_o, cols_h))
        del off_o, cols_o
        sample = rows_np[: a.cpu_sample]
        c0 = time.perf_counter()
        ref.time_rows(sample, threads)
        cpu_s = time.perf_counter() - c0
        cpu = {"value": len(sample) / cpu_s, "unit": "rows/s", "cores": threads, "kind": "port",
               "sample": f"first {len(sample):,} rows of the rank-0 batch on the same {a.rows:,} x {a.cols:,} "
                         f"structure (oracle restatement of BRWT::get_row, plain rank/select; host build {gen_s:.0f} s)"}
        del ref

    kname = mat.traverse_kernel()
    tcfg = {"rows": a.rows, "cols": a.cols, "density": a.density, "arity": a.arity, "batch": a.batch,
            "kernel": a.kernel, "kernel_name": kname}
    traffic = committed_traffic(tcfg)

    value = world * a.batch * a.steps / elapsed
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "rows/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32/u64",
        "data": "synthetic (top-down i.i.d. Bernoulli columns, seed 42; uniform random rows)",
        "config": {
            "workload": f"Multi-BRWT {a.rows:,} x {a.cols:,}, d={a.density}, arity {a.arity} "
                        f"(Kingsford shape, BASELINE configs[3]); batch {a.batch:,} rows per GPU",
            "num_rows": a.rows, "num_columns": a.cols, "density": a.density, "arity": a.arity,
            "batch_per_gpu": a.batch, "global_batch": a.batch * world,
            "parallelism": f"batch-sharded x{world}, tree replicated" + ("" if world == 1 or a.no_gather
                                                                         else ", all-gatherv over " + ("RCCL" if a.dist_backend == "nccl" else a.dist_backend)),
            "structure_bytes": mat.device_bytes(), "setup_s": round(setup_s, 2),
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "stream_read_measured": stream_gbs,
            "traffic": None if traffic is None else traffic[0],
            "traffic_source": None if traffic is None else traffic[1] + " (rocprofv3 PMC, calibrated; per launch)",
            "kernel": kname,
            "kernel_ms": kern_ms,
            "alg_bytes_per_launch": alg_bytes, "visits_per_row": visits / a.batch,
            "labels_per_row": labels / a.batch,
        },
        "cpu_baseline": cpu,
        "reassembly": reassembly,
        "parity": None if parity is None else f"{'bit-exact' if parity else 'MISMATCH'} on {chk:,} rows"
                                                f"{' (the whole timed batch)' if chk == a.batch else ''}"
                                                f" vs the oracle, element-wise CSR",
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
