"""Layout A/B on one synthetic structure (calibration tool, not the bench):
builds the same tree as per-node images and as row records (several block
shapes), times get_rows on the same batch and checks that every
configuration returns the identical CSR.

    python tools/rows_ab.py --rows 3700000000 --batch 8000000 --configs nodes,rows,rows:64,2,rows:128,4
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
from genome_graph_annotation_amd import BRWTDevice, _lib as L  # noqa: E402
from genome_graph_annotation_amd.brwt import build_option  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=3_700_000_000)
ap.add_argument("--cols", type=int, default=2652)
ap.add_argument("--density", type=float, default=0.003)
ap.add_argument("--arity", type=int, default=8)
ap.add_argument("--batch", type=int, default=8_000_000)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--seed", type=int, default=42)
ap.add_argument("--shape", default="", help="npz with num_children/first_child/leaf_column: synthetic_shaped")
ap.add_argument("--configs", default="nodes,rows")
ap.add_argument("--oracle", action="store_true",
                help="check the first configuration's CSR against the streamed top-down oracle (whole batch)")
a = ap.parse_args()

rows_np = np.random.default_rng(a.seed).integers(0, a.rows, a.batch, dtype=np.uint64)
rows = torch.from_numpy(rows_np.view(np.int64)).cuda()
off = torch.empty(a.batch + 1, dtype=torch.int64, device="cuda")
s = torch.cuda.current_stream().cuda_stream
shape = dict(np.load(a.shape)) if a.shape else None
ref = None
cols = None
ASYNC = [False]
status = torch.zeros(3, dtype=torch.int64, device="cuda")


def set_variant(kv, m=None):
    """'' default; 'w6' the general walk on a uniform tree (MBRWT_OPT_ROWS_WALK);
    'async' the timed steps through mbrwt_get_rows_device_async"""
    ASYNC[0] = False
    walk = 0
    for part in kv.split("."):  # e.g. "w6.async"
        if part in ("w6", "w7"):  # the general walk / the odometer without the path table
            walk = int(part[1])
        elif part == "async":
            ASYNC[0] = True
    if m is not None and m.layout() != "nodes":
        m.set_option(L.MBRWT_OPT_ROWS_WALK, walk)


# config = layout[:B,S][@variant+variant...]: one build, every variant timed on it
for cfg in a.configs.split(";") if ";" in a.configs else a.configs.split(","):
    cfg_k, _, kvs = cfg.partition("@")
    layout, _, bs = cfg_k.partition(":")
    block = 0
    if bs:  # row-record blocks "B,S" (build option MBRWT_BUILD_ROWS_BLOCK)
        b_, s_ = (int(x) for x in bs.split(","))
        block = b_ << 8 | s_
    set_variant("")
    t0 = time.time()
    with build_option(L.MBRWT_BUILD_ROWS_BLOCK, block):
        if shape is not None:
            m = BRWTDevice.synthetic_shaped(a.rows, shape, a.density, a.seed, layout=layout)
        else:
            m = BRWTDevice.synthetic(a.rows, a.cols, a.density, a.arity, a.seed, layout=layout)
    build_s = time.time() - t0
    if cols is None:
        try:
            need = m.get_rows_device(rows, off, torch.empty(1, dtype=torch.int32, device="cuda"), s)
        except L.MBRWTError as e:
            need = e.needed
        cols = torch.empty(int(need) + 1024, dtype=torch.int32, device="cuda")
    for kv in (kvs.split("+") if kvs else [""]):
        set_variant(kv, m)
        for _ in range(3):
            nl = m.get_rows_device(rows, off, cols, s)
        torch.cuda.synchronize()
        h = hashlib.blake2b(digest_size=8)
        h.update(off.cpu().numpy().tobytes())
        h.update(cols[:nl].cpu().numpy().tobytes())
        hx = h.hexdigest()
        if ref is None:
            ref = hx
            if a.oracle:
                sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
                import oracle as O  # checker only
                t2 = time.time()
                if shape is not None:
                    off_o, cols_o = O.topdown_get_rows_shaped(a.rows, shape, a.density, a.seed, rows_np)
                else:
                    off_o, cols_o = O.topdown_get_rows(a.rows, a.cols, a.density, a.arity, a.seed, rows_np)
                exact = (np.array_equal(off.cpu().numpy().view(np.uint64), off_o)
                         and np.array_equal(cols[:nl].cpu().numpy().view(np.uint32), cols_o))
                print(json.dumps({"oracle": "streamed top-down", "rows_checked": a.batch,
                                  "labels_checked": int(len(cols_o)), "bit_exact": bool(exact),
                                  "oracle_s": round(time.time() - t2, 1)}), flush=True)
                if not exact:
                    print("MISMATCH vs oracle", flush=True)
                    sys.exit(1)
        m.take_timing()
        m.set_option(L.MBRWT_OPT_TIMING, 1)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        status.zero_()
        for _ in range(a.steps):
            if ASYNC[0]:
                m.get_rows_device_async(rows, off, cols, status, s)
            else:
                m.get_rows_device(rows, off, cols, s)
        torch.cuda.synchronize()
        if ASYNC[0]:
            assert status.cpu().tolist()[1:] == [0, 1], status
        el = (time.perf_counter() - t1) / a.steps
        m.set_option(L.MBRWT_OPT_TIMING, 0)
        kms, k = m.take_timing()
        out = {"config": cfg_k + ("@" + kv if kv else ""), "kernel": m.traverse_kernel(), "layout": m.layout(),
               "build_s": round(build_s, 1), "device_gb": m.device_bytes() / 1e9, "kernel_ms": kms / max(1, k),
               "step_ms": el * 1e3, "rows_per_s": a.batch / el, "labels": int(nl), "csr_hash": hx,
               "same_as_first": hx == ref, "rows_stats": m.rows_stats()}
        print(json.dumps(out), flush=True)
        if hx != ref:
            print("MISMATCH", flush=True)
            sys.exit(1)
    set_variant("")
    del m
    torch.cuda.empty_cache()
