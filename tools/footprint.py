"""footprint.py -- device bytes against the reference's compressed size
(the reference's whole claim is compression:
/root/reference/README.md:26-37).

For each matrix: the plain index bits of the BRWT, the same indexes as sdsl
rrr_vector<63> streams (the reference's bit_vector_rrr<63>; exact by
oracle_rrr_bytes for materialised trees, the expectation under the top-down
law for the full-size synthetic ones -- checked against the exact count on a
materialised top-down tree first), and libmbrwt's device bytes for the
per-node layout and the row-record layout, with get_rows()/s of each layout
(bit-exact against the oracle where the tree is materialised).

Matrices: the reference's own generators (experiments/main.cpp:218-285,
data_generation.cpp, mt19937 seed 42) at 1 M x 2,652, d = 0.3 %: i.i.d.
columns, uniform_rows (10,000 distinct rows x 100) and uniform_columns (265
distinct columns x 10), each under the basic arity-8 partitioner and greedy +
relax 10 (scripts/kingsford/convert.sh:24); then the synthetic C4 (3.7 B x
2,652) and C3 (1 B x 3,173, d = 3.8 %) at full size.  Prints JSON lines.

    python tools/footprint.py [--skip-full]
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
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def log(msg):
    print(f"[footprint] {msg}", file=sys.stderr, flush=True)


def rrr_expected_bytes(size, p):
    """E[bytes] of an rrr_vector<63> stream over `size` i.i.d. Bernoulli(p)
    bits (the layout oracle_rrr_bytes counts)."""
    from scipy.stats import binom
    nb = size // 63 + 1
    k = np.arange(64)
    C = np.array([math.comb(63, int(x)) for x in k], dtype=object)
    space = np.array([0 if c <= 1 else int(c - 1).bit_length() for c in C])
    e_space = float((binom.pmf(k, 63, p) * space).sum())
    ns = (nb + 31) // 32
    btnr = nb * e_space
    w = lambda v: max(1, int(v).bit_length())
    words = lambda bits: math.ceil(bits / 64) * 8
    return (8 + 9 + words(nb * 6) + 8 + words(max(btnr, 64)) + 9 + words(ns * w(btnr)) +
            9 + words((ns + 1) * w(size * p)) + 8 + words(ns))


def law_nodes(shape, n, m, d):
    """(size, p) of every node's index under the top-down law."""
    nc, fc = np.asarray(shape["num_children"]), np.asarray(shape["first_child"])
    N = len(nc)
    cols = np.zeros(N, dtype=np.int64)
    for u in range(N - 1, -1, -1):
        cols[u] = 1 if nc[u] == 0 else cols[fc[u]:fc[u] + nc[u]].sum()
    q = 1.0 - (1.0 - d) ** cols
    out = []
    parent_q = {0: None}
    for u in range(N):
        pq = parent_q.get(u)
        size = n if pq is None else n * pq
        p = q[u] if pq is None else q[u] / pq
        out.append((size, p))
        for c in range(nc[u]):
            parent_q[int(fc[u]) + c] = q[u]
    return out


def timed_rows(dev, n_rows, batch=1_000_000, reps=10, ref=None):
    import torch
    rows = np.random.default_rng(7).integers(0, n_rows, batch, dtype=np.uint64)
    rt = torch.from_numpy(rows.view(np.int64)).cuda()
    ot = torch.empty(batch + 1, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    from genome_graph_annotation_amd import _lib as L
    try:
        need = dev.get_rows_device(rt, ot, torch.empty(1, dtype=torch.int32, device="cuda"), s)
    except L.MBRWTError as e:
        need = e.needed
    ct = torch.empty(int(need) + 1, dtype=torch.int32, device="cuda")
    for _ in range(2):
        dev.get_rows_device(rt, ot, ct, s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        dev.get_rows_device(rt, ot, ct, s)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    exact = None
    if ref is not None:
        off_o, cols_o = ref.get_rows(rows)
        exact = bool(np.array_equal(ot.cpu().numpy().view(np.uint64), off_o) and
                     np.array_equal(ct[:need].cpu().numpy().view(np.uint32), cols_o))
    return batch / el, exact


def device_legs(make, n_rows, ref=None):
    import torch
    out = {}
    for layout in ("nodes", "rows"):
        try:
            dev = make(layout)
        except Exception as e:  # noqa: BLE001 -- report what did not fit
            out[layout] = {"error": str(e)[:200]}
            continue
        r = {"device_bytes": int(dev.device_bytes()), "layout": dev.layout(), "kernel": dev.traverse_kernel()}
        if layout == "rows":
            r["rows_stats"] = dev.rows_stats()
        r["rows_per_s"], r["bit_exact"] = timed_rows(dev, n_rows, ref=ref)
        out[layout] = r
        del dev
        torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--cols", type=int, default=2652)
    ap.add_argument("--density", type=float, default=0.003)
    ap.add_argument("--skip-full", action="store_true")
    a = ap.parse_args()
    import oracle as O
    from genome_graph_annotation_amd import BRWTDevice

    n, m, d = a.rows, a.cols, a.density
    # the law's expectation against the exact count on a materialised top-down tree
    t = O.OracleTree.topdown(20_000_000, m, d, 8, 42)
    exact = t.rrr_bytes()
    model = sum(rrr_expected_bytes(sz, p) for sz, p in law_nodes(t.export(), 20_000_000, m, d))
    print(json.dumps({"check": "rrr expectation vs exact", "tree": f"top-down 20 M x {m}, d={d}, arity 8",
                      "exact_bytes": int(exact), "expected_bytes": int(model), "ratio": model / exact}), flush=True)
    shape = {k: t.export()[k] for k in ("num_children", "first_child", "leaf_column")}
    del t

    mats = [("iid columns", O.generate_columns(n, m, d, 42), n, m)]
    w, nr = O.generate_uniform_rows(n, m, d, 10_000, 42)
    mats.append(("uniform_rows (10,000 distinct x 100)", w, nr, m))
    w, mc = O.generate_uniform_columns(n, m, d, 265, 42)
    mats.append(("uniform_columns (265 distinct x 10)", w, n, mc))
    for name, words, nn, mm in mats:
        for part, arity, relax in (("basic", 8, 0), ("greedy", 2, 10)):
            t0 = time.time()
            t = O.OracleTree.from_words(words, nn, mm, part, arity, relax)
            exp = t.export()
            rec = {"matrix": f"{name}: {nn:,} x {mm:,}, d={d} (mt19937 seed 42)",
                   "partitioner": f"{part}" + (f" arity {arity}" if part == "basic" else f" + relax {relax}"),
                   "nodes": int(t.num_nodes()), "depth": int(t.depth()), "relations": int(t.num_relations()),
                   "plain_index_bytes": int(t.total_column_size() // 8), "rrr_bytes": int(t.rrr_bytes()),
                   "oracle_build_s": round(time.time() - t0, 1)}
            rec.update(device_legs(lambda lay: BRWTDevice.from_tree(exp, layout=lay), nn, ref=t))
            for lay in ("nodes", "rows"):
                if "device_bytes" in rec.get(lay, {}):
                    rec[lay]["device_over_rrr"] = rec[lay]["device_bytes"] / rec["rrr_bytes"]
            print(json.dumps(rec), flush=True)
            del t, exp
    if a.skip_full:
        return
    for name, (nn, mm, dd) in (("C4 Kingsford shape", (3_700_000_000, 2652, 0.003)),
                               ("C3 RefSeq shape", (1_000_000_000, 3173, 0.038))):
        t = O.OracleTree.topdown(1000, mm, dd, 8, 42)
        law = law_nodes(t.export(), nn, mm, dd)
        del t
        rrr = sum(rrr_expected_bytes(sz, p) for sz, p in law)
        plain = sum(sz for sz, _ in law) / 8
        rec = {"matrix": f"{name}: {nn:,} x {mm:,}, d={dd} (top-down law, arity 8)",
               "plain_index_bytes_expected": int(plain), "rrr_bytes_expected": int(rrr)}
        rec.update(device_legs(lambda lay: BRWTDevice.synthetic(nn, mm, dd, 8, 42, layout=lay), nn))
        for lay in ("nodes", "rows"):
            if "device_bytes" in rec.get(lay, {}):
                rec[lay]["device_over_rrr"] = rec[lay]["device_bytes"] / rrr
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
