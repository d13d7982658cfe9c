"""footprint_scale.py -- device bytes against the reference's compressed size
at 100 M rows on correlated data (the reference's claim is
compression: /root/reference/README.md:26-37).

Matrices (100 M x 2,652, d = 0.3 % unless given): the laws of the
reference's own generators (experiments/main.cpp:218-285,
data_generation.cpp:114-200), drawn on the device with torch's generator
instead of mt19937 (the reference's exact streams are pinned at 1 M rows by
tools/footprint.py and the oracle; at 100 M rows its host generator would
take hours):
  iid              the synthetic top-down law (the C4 law)
  uniform_rows     `unique` distinct rows, each repeated n / unique times, shuffled
  weighted_rows    `unique` distinct rows with frequencies n / (H_unique i)
                   (generate_row_counts_index_inverse), shuffled
  uniform_columns  `unique` distinct columns, each repeated m / unique times, shuffled
Each under the basic arity-8 partitioner and greedy + relax 10
(scripts/kingsford/convert.sh:24) where asked.  Per matrix and partitioner:
the tree is built on the device from its columns (mbrwt_create_from_columns,
node layout), exported, and its index vectors' sdsl rrr_vector<63> bytes
counted exactly (rrr_bytes below, the layout oracle_rrr_bytes counts --
tests/test_footprint_tool.py pins it against the oracle); then the row-record
image without and with record classes (MBRWT_BUILD_ROWS_CLASSES) from the
same tree, and get_rows/s of every layout on 8 M-row batches (the traversal
kernel's HIP-event time beside the synchronous call), the record layouts
checked against the node layout on every batch row.  One JSON line per case.

    python tools/footprint_scale.py --cases uniform_rows:basic,uniform_rows:greedy
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(msg):
    print(f"[footprint_scale {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


# ---- sdsl rrr_vector<63> bytes of one bit vector (oracle_rrr_bytes' layout) ----
_C63 = [math.comb(63, k) for k in range(64)]
_SPACE = np.array([0 if c <= 1 else int(c - 1).bit_length() for c in _C63], dtype=np.int64)


def rrr_bytes(size: int, words: np.ndarray) -> int:
    """Bytes of an rrr_vector<63> over `size` bits (LSB-first u64 words):
    size, 6-bit block classes, the blocks' numbers at ceil(log2 C(63, k))
    bits, number-pointer and rank samples every 32 blocks, invert bits."""
    size = int(size)
    nb = (size + 63) // 63
    ns = (nb + 31) // 32
    w = np.zeros((size + 63) // 64 + 1, dtype=np.uint64)
    src = np.asarray(words, dtype=np.uint64)[: (size + 63) // 64]
    w[: len(src)] = src
    cum = np.zeros(len(w) + 1, dtype=np.int64)
    np.cumsum(np.bitwise_count(w), out=cum[1:])
    pos = np.minimum(np.arange(nb + 1, dtype=np.int64) * 63, size)
    i, o = pos >> 6, (pos & 63).astype(np.uint64)
    mask = np.where(o == 0, np.uint64(0), (np.uint64(1) << o) - np.uint64(1))
    rank = cum[i] + np.bitwise_count(w[i] & mask).astype(np.int64)
    k = np.diff(rank)
    btnr = int(_SPACE[k].sum())
    ones = int(rank[-1])
    words_of = lambda bits: (bits + 63) // 64 * 8
    width = lambda v: v.bit_length() if v else 64
    return (8 + (9 + words_of(nb * 6)) + (8 + words_of(max(btnr, 64))) + (9 + words_of(ns * width(btnr))) +
            (9 + words_of((ns + 1) * width(ones))) + (8 + words_of(ns)))


def tree_rrr_bytes(tree) -> tuple[int, int]:
    """(plain index bytes, RRR bytes) of an exported tree (every node's index)."""
    plain = rrr = 0
    for size, words in zip(tree["vec_size"], tree["words"]):
        plain += int(size) // 8
        rrr += rrr_bytes(int(size), words)
    return plain, rrr


# ---- matrices on the device (column words on the host for the builder) --------
def _pack(bits):
    """bool[n] (cuda) -> LSB-first uint64 words (numpy)."""
    import torch
    n = bits.numel()
    W = (n + 63) // 64
    b = torch.zeros(W * 64, dtype=torch.uint8, device=bits.device)
    b[:n] = bits.to(torch.uint8)
    b = b.view(W, 8, 8)
    byte = (b << torch.arange(8, device=b.device, dtype=torch.uint8)).sum(dim=2, dtype=torch.uint8)  # LSB-first bytes
    return byte.contiguous().view(-1).cpu().numpy().view(np.uint64)


def replicated_rows_columns(n, m, d, freqs, seed):
    """generate_random_rows: distinct rows (Bernoulli(d) columns), row i
    repeated freqs[i] times, the rows shuffled -> (column words, rows)."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    u = len(freqs)
    reps = torch.repeat_interleave(torch.arange(u, device="cuda"), torch.as_tensor(freqs, device="cuda"))
    rows = reps.numel()
    assign = reps[torch.randperm(rows, device="cuda", generator=g)]
    del reps
    cols = []
    for j in range(m):
        has = torch.rand(u, device="cuda", generator=g) < d
        cols.append(_pack(has[assign]))
        if j % 500 == 0:
            log(f"  column {j}/{m}")
    return cols, rows


def uniform_columns(n, m, d, unique, seed):
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    gen = [_pack(torch.rand(n, device="cuda", generator=g) < d) for _ in range(unique)]
    freq = m // unique
    src = np.repeat(np.arange(unique), freq)
    src = src[torch.randperm(len(src), generator=torch.Generator().manual_seed(seed)).numpy()]
    return [gen[s] for s in src], n


def weighted_freqs(n, unique):
    """generate_row_counts_index_inverse (data_generation.cpp:168-200)."""
    H = float(np.sum(1.0 / np.arange(1, unique + 1)))
    f = np.floor(n / H / np.arange(1, unique + 1)).astype(np.int64)
    f[f == 0] = 1
    return f


# ---- measurement -----------------------------------------------------------
def timed(dev, n_rows, batch, reps, ref=None):
    import torch
    from genome_graph_annotation_amd import _lib as L
    rng = np.random.default_rng(7)
    rows = [torch.from_numpy(rng.integers(0, n_rows, batch, dtype=np.uint64).view(np.int64)).cuda() for _ in range(2)]
    ot = torch.empty(batch + 1, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    try:
        need = dev.get_rows_device(rows[0], ot, torch.empty(1, dtype=torch.int32, device="cuda"), s)
    except L.MBRWTError as e:
        need = e.needed
    ct = torch.empty(int(need * 1.2) + 4096, dtype=torch.int32, device="cuda")
    for k in range(2):
        dev.get_rows_device(rows[k % 2], ot, ct, s)
    torch.cuda.synchronize()
    dev.take_timing()
    dev.set_option(L.MBRWT_OPT_TIMING, 1)
    t0 = time.perf_counter()
    for k in range(reps):
        dev.get_rows_device(rows[k % 2], ot, ct, s)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    dev.set_option(L.MBRWT_OPT_TIMING, 0)
    km, kl = dev.take_timing()
    out = {"rows_per_s": batch / el, "ms_per_batch": el * 1e3, "kernel_ms": km / max(1, kl)}
    # the last batch against the reference layout's answer for it
    got = dev.get_rows_device(rows[(reps - 1) % 2], ot, ct, s)
    res = (ot.cpu().numpy().copy(), ct[:got].cpu().numpy().copy())
    if ref is not None:
        out["same_as_nodes"] = bool(np.array_equal(res[0], ref[0]) and np.array_equal(res[1], ref[1]))
    return out, res


def measure(name, part, make_cols, n, m, d, batch, reps, do_classes=True):
    import torch
    from genome_graph_annotation_amd import BRWTDevice, _lib as L
    from genome_graph_annotation_amd.brwt import build_option
    t0 = time.time()
    if make_cols is None:  # the synthetic top-down law (iid columns, arity 8)
        nodes = BRWTDevice.synthetic(n, m, d, 8, 42, layout="nodes")
        rows = n
    else:
        cols, rows = make_cols()
        m = len(cols)
        log(f"{name}: columns generated ({time.time() - t0:.0f} s)")
        relax = 10 if part == "greedy" else 0
        nodes = BRWTDevice.from_columns(cols, rows, 8 if part == "basic" else 2, relax_max_arity=relax,
                                        layout="nodes", partitioner=part)
        del cols
    log(f"{name}/{part}: node image built ({time.time() - t0:.0f} s)")
    rec = {"matrix": name, "rows": rows, "columns": m, "partitioner": part if part == "basic" else "greedy + relax 10",
           "nodes": nodes.num_nodes(), "relations": nodes.num_relations()}
    tree = nodes.export()
    plain, rrr = tree_rrr_bytes(tree)
    rec.update(plain_index_bytes=plain, rrr_bytes=rrr)
    log(f"{name}/{part}: exported, RRR {rrr / 1e9:.3f} GB ({time.time() - t0:.0f} s)")
    tm, ref = timed(nodes, rows, batch, reps)
    rec["nodes_layout"] = {"device_bytes": nodes.device_bytes(), "over_rrr": nodes.device_bytes() / rrr, **tm}
    nodes.close()
    torch.cuda.empty_cache()
    for key, cls in (("rows_layout", 0), ("rows_classes", -1 if do_classes else None)):
        if cls is None:
            continue
        with build_option(L.MBRWT_BUILD_ROWS_CLASSES, cls):
            try:
                dev = BRWTDevice.from_tree(tree, layout="rows")
            except L.MBRWTError as e:
                rec[key] = {"error": str(e)[:160]}
                continue
        st = dev.rows_stats()
        tm, _ = timed(dev, rows, batch, reps, ref)
        rec[key] = {"device_bytes": dev.device_bytes(), "over_rrr": dev.device_bytes() / rrr, "kernel": dev.traverse_kernel(),
                    "block_bytes": st["block_bytes"], "rows_per_block": st["rows_per_block"],
                    "classes": st.get("classes", 0), "class_bits": st.get("class_bits", 0),
                    "class_index_bytes": st.get("class_index_bytes", 0),
                    "class_sample_distinct": st.get("class_sample_distinct", 0), **tm}
        dev.close()
        torch.cuda.empty_cache()
        log(f"{name}/{part}: {key} {rec[key]['device_bytes'] / 1e9:.3f} GB, {tm['rows_per_s'] / 1e9:.2f} G rows/s")
    rec["build_and_measure_s"] = round(time.time() - t0, 1)
    print(json.dumps(rec), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--cols", type=int, default=2652)
    ap.add_argument("--density", type=float, default=0.003)
    ap.add_argument("--unique-rows", type=int, default=1_000_000)
    ap.add_argument("--unique-cols", type=int, default=265)
    ap.add_argument("--batch", type=int, default=8_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cases", default="iid:basic,uniform_rows:basic,uniform_rows:greedy,weighted_rows:basic,"
                                       "uniform_columns:basic,uniform_columns:greedy")
    a = ap.parse_args()
    n, m, d = a.rows, a.cols, a.density
    ur = a.unique_rows
    for case in a.cases.split(","):
        name, part = case.split(":")
        if name == "iid":
            make = None
        elif name == "uniform_rows":
            make = lambda: replicated_rows_columns(n, m, d, np.full(ur, n // ur), 42)
        elif name == "weighted_rows":
            make = lambda: replicated_rows_columns(n, m, d, weighted_freqs(n, ur), 42)
        elif name == "uniform_columns":
            make = lambda: uniform_columns(n, m, d, a.unique_cols, 42)
        else:
            raise SystemExit(f"unknown matrix {name}")
        measure(name, part, make, n, m, d, a.batch, a.reps)


if __name__ == "__main__":
    main()
