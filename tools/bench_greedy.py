"""bench_greedy.py -- get_rows()/s on the reference's production tree shape:
the Kingsford build path (scripts/kingsford/convert.sh:24: transform_anno
--anno-type brwt --greedy, then relax_brwt with --relax-arity 10, the default
of config.hpp:32), i.e. binary_grouping_greedy (partitionings.cpp:148-201),
BRWTBottomUpBuilder::build (BRWT_builders.cpp:119-163) and
BRWTOptimizer::relax (:166-211), over the C2 columns (1 M x 2,652, d = 0.3 %,
the reference's own mt19937 column generator).  The tree is built by the CPU
oracle (the greedy partitioner has no device version) and uploaded through
mbrwt_create; the basic arity-8 tree of the same columns is measured beside
it.  Every timed batch is checked against the oracle.  Prints ONE JSON line.
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
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def log(msg):
    print(f"[bench_greedy] {msg}", file=sys.stderr, flush=True)


def measure(dev, rows_np, ref, variants, reps):
    """ref = (offsets, cols) of the oracle for rows_np."""
    from genome_graph_annotation_amd import _lib as L
    n = len(rows_np)
    rows_t = torch.from_numpy(rows_np.view(np.int64)).cuda()
    off_t = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    off_o, cols_o = ref
    cols_t = torch.empty(len(cols_o) + 1024, dtype=torch.int32, device="cuda")
    try:
        visits, labels = dev.count_work_device(rows_t, s)
    except L.MBRWTError:  # terminal records: no V accounting
        visits, labels = 0, len(ref[1])
    out = {}
    for v in variants:
        if isinstance(v, str):  # "wN": row records with MBRWT_OPT_ROWS_WALK = N
            dev.set_option(L.MBRWT_OPT_KERNEL, 0)
            dev.set_option(L.MBRWT_OPT_ROWS_WALK, int(v[1:]))
        else:
            dev.set_option(L.MBRWT_OPT_KERNEL, v)
        name = dev.traverse_kernel()
        nl = dev.get_rows_device(rows_t, off_t, cols_t, s)
        torch.cuda.synchronize()
        exact = (nl == len(cols_o) and np.array_equal(off_t.cpu().numpy().view(np.uint64), off_o)
                 and np.array_equal(cols_t[:nl].cpu().numpy().view(np.uint32), cols_o))
        # warm-up of >= 0.2 s: the oracle ran on the host for seconds before,
        # and an idle GPU's first milliseconds of work run at idle clocks
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.2:
            dev.get_rows_device(rows_t, off_t, cols_t, s)
        torch.cuda.synchronize()
        dev.take_timing()
        dev.set_option(L.MBRWT_OPT_TIMING, 1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            dev.get_rows_device(rows_t, off_t, cols_t, s)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps
        dev.set_option(L.MBRWT_OPT_TIMING, 0)
        ms, k = dev.take_timing()
        out[str(v)] = {"kernel": name, "kernel_ms": ms / k, "step_ms": wall * 1e3, "rows_per_s": n / wall,
                       "bit_exact": bool(exact)}
        log(f"variant {v} ({name}): kernel {ms / k:.3f} ms, step {wall * 1e3:.3f} ms, "
            f"{n / wall / 1e9:.2f} G rows/s, bit-exact {exact}")
    dev.set_option(L.MBRWT_OPT_KERNEL, 0)
    if dev.layout() != "nodes":
        dev.set_option(L.MBRWT_OPT_ROWS_WALK, 0)
    return {"visits_per_row": visits / n, "labels_per_row": labels / n, "variants": out}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--cols", type=int, default=2652)
    ap.add_argument("--density", type=float, default=0.003)
    ap.add_argument("--relax", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="0,5")
    ap.add_argument("--scaled-rows", type=int, default=0,
                    help="also measure the greedy + relax SHAPE of the C2 build with the synthetic law at this "
                         "many rows (mbrwt_create_synthetic_shaped; parity by the streamed shaped oracle)")
    ap.add_argument("--scaled-batch", type=int, default=8_000_000)
    ap.add_argument("--skip-small", action="store_true", help="only the scaled shape")
    ap.add_argument("--shapes", default="greedy+relax,basic arity 8", help="comma-separated subset of the shapes")
    ap.add_argument("--shape-npz", default="",
                    help="the greedy + relax tree shape of the C2 build (num_children / first_child / "
                         "leaf_column, BFS) from a file written by --save-shape: skips the oracle's greedy build "
                         "(~2.5 min) and measures only the scaled shape")
    ap.add_argument("--save-shape", default="", help="write the greedy + relax shape of the C2 build to this .npz")
    ap.add_argument("--compact", action="store_true",
                    help="row records built with MBRWT_BUILD_ROWS_FOOTPRINT = MBRWT_ROWS_COMPACT (the smallest image "
                         "within 30 %% of the fewest modelled requests per row)")
    ap.add_argument("--blocks", default="",
                    help="scaled shape: comma-separated row-record block shapes 'B:S' to build and measure one after "
                         "the other (MBRWT_BUILD_ROWS_BLOCK; '' = the automatic choice only, 'auto' names it)")
    ap.add_argument("--rows-codes", default="0",
                    help="comma-separated MBRWT_BUILD_ROWS_CODE values for the scaled shape: 0 mask bytes, "
                         "2 terminal records (DESIGN §4h)")
    ap.add_argument("--layout", default="nodes", choices=["nodes", "rows", "both"],
                    help="device layout (include/mbrwt.h MBRWT_BUILD_LAYOUT)")
    a = ap.parse_args()
    import oracle as O
    from genome_graph_annotation_amd import BRWTDevice

    variants = [x if x.startswith("w") else int(x) for x in a.variants.split(",")]
    rows_np = np.random.default_rng(42).integers(0, a.rows, a.batch, dtype=np.uint64)
    res = {}
    shapes = {}
    want = set(a.shapes.split(","))
    if a.shape_npz:
        z = np.load(a.shape_npz)
        shapes["greedy+relax"] = ({"num_children": z["num_children"], "first_child": z["first_child"],
                                   "leaf_column": z["leaf_column"]}, 0.0)
        want = set()
    for shape, part, arity, relax in [("greedy+relax", "greedy", 2, a.relax), ("basic arity 8", "basic", 8, 0)]:
        if shape not in want:
            continue
        if a.skip_small:
            t0 = time.time()
            t = O.OracleTree.norepl(a.rows, a.cols, a.density, 42, part, arity, relax)
            shapes[shape] = (t.export(), time.time() - t0)
            if a.save_shape and shape == "greedy+relax":
                ex = shapes[shape][0]
                np.savez(a.save_shape, num_children=ex["num_children"], first_child=ex["first_child"],
                         leaf_column=ex["leaf_column"])
            del t
            continue
        t0 = time.time()
        t = O.OracleTree.norepl(a.rows, a.cols, a.density, 42, part, arity, relax)
        build_s = time.time() - t0
        exp = t.export()
        nc = np.asarray(exp["num_children"])
        dev = BRWTDevice.from_tree(exp, layout=a.layout)
        log(f"{shape}: oracle build {build_s:.0f} s, {t.num_nodes()} nodes, depth {t.depth()}, "
            f"avg arity {t.avg_arity():.2f}, max arity {int(nc.max())}; device {dev.device_bytes() / 1e6:.1f} MB, "
            f"kernel {dev.traverse_kernel()}")
        r = measure(dev, rows_np, t.get_rows(rows_np), variants, a.reps)
        r.update({"layout": dev.layout(), "rows_stats": dev.rows_stats(), "nodes": int(t.num_nodes()), "depth": int(t.depth()), "avg_arity": t.avg_arity(),
                  "max_arity": int(nc.max()), "device_bytes": int(dev.device_bytes()), "oracle_build_s": build_s})
        res[shape] = r
        shapes[shape] = (exp, build_s)
        del dev, t
    if a.scaled_rows:
        srows = np.random.default_rng(42).integers(0, a.scaled_rows, a.scaled_batch, dtype=np.uint64)
        for shape, (exp, build_s) in shapes.items():
            keep = {k: exp[k] for k in ("num_children", "first_child", "leaf_column")}
            nc = np.asarray(keep["num_children"])
            from genome_graph_annotation_amd import _lib as LB
            from genome_graph_annotation_amd.brwt import build_option
            ref = None
            for blk, code in [(b, int(c)) for b in (a.blocks.split(",") if a.blocks else ["auto"])
                              for c in a.rows_codes.split(",")]:
                t0 = time.time()
                bs = 0 if blk == "auto" else (int(blk.split(":")[0]) << 8) | int(blk.split(":")[1])
                with build_option(LB.MBRWT_BUILD_ROWS_FOOTPRINT,
                                  LB.MBRWT_ROWS_COMPACT if a.compact else LB.MBRWT_ROWS_FAST), \
                        build_option(LB.MBRWT_BUILD_ROWS_BLOCK, bs), build_option(LB.MBRWT_BUILD_ROWS_CODE, code):
                    dev = BRWTDevice.synthetic_shaped(a.scaled_rows, keep, a.density, 42, layout=a.layout)
                torch.cuda.synchronize()
                gen_s = time.time() - t0
                t0 = time.time()
                if ref is None:
                    ref = O.topdown_get_rows_shaped(a.scaled_rows, keep, a.density, 42, srows)
                log(f"scaled {shape} (blocks {blk}, code {code}): {a.scaled_rows:,} rows, {len(nc)} nodes, max arity "
                    f"{int(nc.max())}, device {dev.device_bytes() / 1e9:.2f} GB (generated in {gen_s:.1f} s), "
                    f"kernel {dev.traverse_kernel()}, rows_stats {dev.rows_stats()}")
                r = measure(dev, srows, ref, variants, a.reps)
                r.update({"layout": dev.layout(), "rows_stats": dev.rows_stats(), "nodes": len(nc),
                          "max_arity": int(nc.max()), "device_bytes": int(dev.device_bytes()),
                          "generate_s": gen_s, "rows": a.scaled_rows, "batch": a.scaled_batch,
                          "num_relations": int(dev.num_relations()), "blocks": blk, "rows_code": code})
                res[f"scaled {shape}" + ("" if blk == "auto" else f" blocks {blk}") + (f" code {code}" if code else "")] = r
                del dev
                torch.cuda.empty_cache()
    print(json.dumps({"workload": f"C2 columns {a.rows:,} x {a.cols:,} d={a.density} (mt19937 seed 42), batch "
                                  f"{a.batch:,} uniform rows (seed 42)", "shapes": res}), flush=True)


if __name__ == "__main__":
    main()
