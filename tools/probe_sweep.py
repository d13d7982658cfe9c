"""Sweep of the random-request ceiling: random segment reads
over a buffer far larger than the Infinity Cache, by segment size, segments in
flight per lane group and resident waves per CU (tools/probe.hip
`probe_random_seg`).  Prints one line per configuration and the maximum per
segment size; bench.py reports the 64-byte maximum as `ceiling_random64`.

    python tools/probe_sweep.py [--gib 64]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=64.0)
    ap.add_argument("--out", default="")
    ap.add_argument("--segs", default="64,0,32,128,256", help="segment bytes (0: one 64-B segment per lane)")
    a = ap.parse_args()
    import torch

    lib = C.CDLL(os.path.join(ROOT, "tools", "_build", "libprobe.so"))
    lib.probe_random_seg.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                     C.POINTER(C.c_double)]
    dev = torch.device("cuda:0")
    nbytes = int(a.gib * (1 << 30))
    buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    buf.fill_(1)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream().cuda_stream
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    res = []
    best = {}
    for seg in [int(x) for x in a.segs.split(",")]:
        for u in (1, 2, 4, 8, 16):
            if seg == 0 and u > 4:
                continue
            for wpc in (8, 16, 32):  # resident waves per CU (256-lane workgroups)
                grid = cus * wpc // 4
                v = C.c_double(0)
                rc = lib.probe_random_seg(buf.data_ptr(), nbytes, seg, u, grid, 256, s, C.byref(v))
                if rc:
                    print(f"seg={seg} u={u} wpc={wpc}: error {rc}", flush=True)
                    continue
                segb = seg or 64
                r = {"seg_bytes": segb, "lanewise": seg == 0, "inflight": u, "waves_per_cu": wpc,
                     "G_per_s": v.value / 1e9, "TB_per_s": v.value * segb / 1e12}
                res.append(r)
                key = ("lane64" if seg == 0 else str(segb))
                if key not in best or r["G_per_s"] > best[key]["G_per_s"]:
                    best[key] = r
                print(json.dumps(r), flush=True)
    print("BEST " + json.dumps(best), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"gib": a.gib, "cus": cus, "results": res, "best": best}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
