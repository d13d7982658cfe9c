"""PCIe / host-copy rates of this box (measurement tool, not the bench): the
bounds of the end-to-end get_rows path (host row ids -> host CSR).

Prints one JSON line: H2D / D2H GB/s from pinned and from pageable host
memory (hipMemcpyAsync via torch), concurrent H2D + D2H, and host memcpy
GB/s (one thread and the job's threads).

    python tools/pcie_probe.py [--mib 256]
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--mib", type=int, default=256)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
nb = a.mib << 20
dev = torch.empty(nb, dtype=torch.uint8, device="cuda")
dev2 = torch.empty(nb, dtype=torch.uint8, device="cuda")
pin = torch.empty(nb, dtype=torch.uint8).pin_memory()
pin2 = torch.empty(nb, dtype=torch.uint8).pin_memory()
page = torch.from_numpy(np.ones(nb, dtype=np.uint8))
page2 = torch.from_numpy(np.ones(nb, dtype=np.uint8))
dev.fill_(1)
torch.cuda.synchronize()


def rate(fn):
    fn()
    torch.cuda.synchronize()
    best = 0.0
    for _ in range(a.reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = max(best, nb / (time.perf_counter() - t0) / 1e9)
    return best


out = {"bytes": nb}
out["h2d_pinned_GBs"] = rate(lambda: dev.copy_(pin, non_blocking=True))
out["d2h_pinned_GBs"] = rate(lambda: pin.copy_(dev, non_blocking=True))
out["h2d_pageable_GBs"] = rate(lambda: dev.copy_(page))
out["d2h_pageable_GBs"] = rate(lambda: page.copy_(dev))
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def both():
    with torch.cuda.stream(s1):
        dev2.copy_(pin2, non_blocking=True)
    with torch.cuda.stream(s2):
        pin.copy_(dev, non_blocking=True)


out["h2d_plus_d2h_pinned_GBs_each"] = rate(both)
src = np.ones(nb, dtype=np.uint8)
dst = np.empty(nb, dtype=np.uint8)
np.copyto(dst, src)
t0 = time.perf_counter()
for _ in range(a.reps):
    np.copyto(dst, src)
out["host_memcpy_1t_GBs"] = nb * a.reps / (time.perf_counter() - t0) / 1e9
ts = torch.from_numpy(src)
td = torch.from_numpy(dst)
td.copy_(ts)
t0 = time.perf_counter()
for _ in range(a.reps):
    td.copy_(ts)
out["host_memcpy_torch_GBs"] = nb * a.reps / (time.perf_counter() - t0) / 1e9
# page-locking the caller's own (pageable) buffer for direct DMA: the cost
# of hipHostRegister + hipHostUnregister per call
import ctypes as C
hip = C.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipHostUnregister.argtypes = [C.c_void_p]
buf = np.ones(nb, dtype=np.uint8)
t0 = time.perf_counter()
rc1 = hip.hipHostRegister(buf.ctypes.data, nb, 0)
t1 = time.perf_counter()
rc2 = hip.hipHostUnregister(buf.ctypes.data)
t2 = time.perf_counter()
out["host_register_ms"] = (t1 - t0) * 1e3
out["host_unregister_ms"] = (t2 - t1) * 1e3
out["host_register_rc"] = [rc1, rc2]
out["torch_threads"] = torch.get_num_threads()
out["affinity_cpus"] = len(os.sched_getaffinity(0))
print(json.dumps(out), flush=True)
