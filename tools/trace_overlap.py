"""Per-dispatch overlap of the two-stream C4 step: from a
rocprofv3 --kernel-trace CSV of bench.py, how much of each k_compact_tiles
(and the tile scan) runs beside a k_traverse_rows, and how long each
traversal lasts alone vs beside the other stream's compaction.

    python tools/trace_overlap.py run_kernel_trace.csv [--skip 12] > summary.json
"""
import argparse
import csv
import json
import re

import numpy as np


def load(path):
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         r.get("Queue_Id", r.get("Stream_Id", "?"))))
    rows.sort(key=lambda x: x[1])
    return rows


def covered(a0, a1, ivs):
    """ns of [a0, a1) covered by the union of intervals ivs (sorted by start)."""
    tot, cur0, cur1 = 0, None, None
    for b0, b1 in ivs:
        b0, b1 = max(a0, b0), min(a1, b1)
        if b1 <= b0:
            continue
        if cur1 is None or b0 > cur1:
            if cur1 is not None:
                tot += cur1 - cur0
            cur0, cur1 = b0, b1
        else:
            cur1 = max(cur1, b1)
    if cur1 is not None:
        tot += cur1 - cur0
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--skip", type=int, default=12, help="traversal dispatches to skip (sizing + warm-up)")
    ap.add_argument("--take", type=int, default=50, help="traversal dispatches to keep after the skip")
    a = ap.parse_args()
    rows = load(a.csv)
    trav = [(s, e, q) for k, s, e, q in rows if re.search(r"k_traverse_rows", k)]
    comp = [(s, e, q) for k, s, e, q in rows if re.search(r"k_compact_tiles", k)]
    scan = [(s, e, q) for k, s, e, q in rows if re.search(r"DeviceScan|scan|Scan", k) and "k_traverse" not in k]
    trav = trav[a.skip:a.skip + a.take]
    t0, t1 = trav[0][0], trav[-1][1]
    comp = [c for c in comp if c[0] >= t0 and c[1] <= t1 + 10**6]
    scan = [c for c in scan if c[0] >= t0 and c[1] <= t1 + 10**6]
    civ = sorted((s, e) for s, e, _ in comp + scan)
    tiv = sorted((s, e) for s, e, _ in trav)
    td = np.array([(e - s) / 1e3 for s, e, _ in trav])
    tov = np.array([covered(s, e, civ) / max(1, e - s) for s, e, _ in trav])
    cd = np.array([(e - s) / 1e3 for s, e, _ in comp])
    cov = np.array([covered(s, e, tiv) / max(1, e - s) for s, e, _ in comp])
    starts = np.array([s for s, _, _ in trav])
    out = {
        "source": a.csv, "traversals": len(trav), "compactions": len(comp), "scans": len(scan),
        "step_us_from_traversal_starts": float(np.diff(starts).mean() / 1e3) if len(starts) > 1 else None,
        "span_us": (t1 - t0) / 1e3,
        "traversal_us": {"mean": float(td.mean()), "p10": float(np.percentile(td, 10)),
                         "p90": float(np.percentile(td, 90))},
        "traversal_fraction_beside_compaction_or_scan": float(tov.mean()),
        "traversal_us_mostly_alone": float(td[tov < 0.2].mean()) if (tov < 0.2).any() else None,
        "traversal_us_mostly_beside": float(td[tov >= 0.5].mean()) if (tov >= 0.5).any() else None,
        "compaction_us": {"mean": float(cd.mean()) if len(cd) else None},
        "compaction_fraction_beside_traversal": float(cov.mean()) if len(cov) else None,
        "traversals_in_flight_at_once": float(sum((e - s) for s, e, _ in trav) / max(1, t1 - t0)),
        "queues": sorted({q for _, _, q in trav}),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
