"""pmc_traffic.py -- turn rocprofv3 --pmc CSVs into the per-launch HBM traffic
figure bench.py reports as roofline.traffic.

Usage:
  python tools/pmc_traffic.py --kernel REGEX --fetch FETCH.csv [--write WRITE.csv]
      [--rdreq RDREQ.csv] [--calib CALIB_FETCH.csv --calib-segments N]
      --config KEY=VALUE ... -o OUT.json

FETCH.csv / WRITE.csv / RDREQ.csv are counter_collection.csv files of separate
rocprofv3 passes (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950,
MI355X_MICROARCH.md "rocprofv3").  FETCH_SIZE/WRITE_SIZE are in KiB.

Correction (MI355X_MICROARCH.md § HBM): FETCH_SIZE = TCC_EA0_RDREQ x 64 B and
under-reports wide streaming reads by 2x; other widths are uncalibrated.  The
traversal's reads are random 64-B segments, so the factor is calibrated on a
known count of exactly that pattern (tools/gather_probe <GiB> calib): factor =
64 B x segments / FETCH_SIZE bytes of the calibration dispatch.
"""
from __future__ import annotations

import argparse
import csv
import json
import re
import statistics


def per_dispatch(path, kernel_re, counter):
    vals = {}
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter or not re.search(kernel_re, r["Kernel_Name"]):
                continue
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write")
    ap.add_argument("--rdreq")
    ap.add_argument("--calib")
    ap.add_argument("--calib-kernel", default="k_probe_group")
    ap.add_argument("--calib-segments", type=int, default=0)
    ap.add_argument("--config", nargs="*", default=[])
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()

    fetch = per_dispatch(a.fetch, a.kernel, "FETCH_SIZE")
    if not fetch:
        raise SystemExit(f"no FETCH_SIZE rows for {a.kernel!r} in {a.fetch}")
    out = {"kernel_regex": a.kernel, "dispatches": len(fetch),
           "fetch_size_bytes": statistics.median(fetch) * 1024}
    factor = 1.0
    if a.calib:
        cal = per_dispatch(a.calib, a.calib_kernel, "FETCH_SIZE")
        cal_bytes = statistics.median(cal) * 1024
        factor = 64.0 * a.calib_segments / cal_bytes
        out["calibration"] = {"kernel": a.calib_kernel, "segments_64B": a.calib_segments,
                              "fetch_size_bytes": cal_bytes, "factor": factor}
    out["read_bytes"] = out["fetch_size_bytes"] * factor
    if a.write:
        w = per_dispatch(a.write, a.kernel, "WRITE_SIZE")
        out["write_bytes"] = statistics.median(w) * 1024 if w else None
    if a.rdreq:
        rq = per_dispatch(a.rdreq, a.kernel, "TCC_EA0_RDREQ_sum")
        out["tcc_ea0_rdreq"] = statistics.median(rq) if rq else None
    out["traffic_bytes"] = out["read_bytes"] + (out.get("write_bytes") or 0.0)
    out["config"] = dict(kv.split("=", 1) for kv in a.config)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
