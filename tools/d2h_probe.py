#!/usr/bin/env python3
"""Device -> host copy ceilings on this box (the C5 mesh copy, bench c5.extract_ms): 1 GiB from HBM into
(a) torch pinned memory, (b) a fresh pageable torch tensor (.cpu()), (c) mqr_memcpy into a fresh numpy
array (first-touch page faults inside the copy) and (d) into the same array again (pages present), and
(e) the cost of first-touching a fresh array alone (np.empty + fill, one thread), and (f) mqr_memcpy into a
fresh mqr._lib.host_empty array (2 MiB-aligned MADV_HUGEPAGE mapping, what the library's callers use).
MQR_D2H_THREADS sets the host threads of libmqr's staged copy (default 8).  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))


def main():
    import numpy as np
    import torch
    from mqr import _lib
    nbytes = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
    n = nbytes // 4
    dev = torch.empty(n, dtype=torch.float32, device="cuda").fill_(1.0)
    torch.cuda.synchronize()
    gbs = lambda t: nbytes / t / 1e9  # noqa: E731
    out = {"bytes": nbytes, "threads": int(os.environ.get("MQR_D2H_THREADS", 8))}
    pin = torch.empty(n, dtype=torch.float32, pin_memory=True)
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        pin.copy_(dev)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    out["torch_pinned_gbs"] = gbs(best)
    del pin
    t0 = time.perf_counter()
    x = dev.cpu()
    out["torch_pageable_fresh_gbs"] = gbs(time.perf_counter() - t0)
    del x
    a = np.empty(n, np.float32)
    t0 = time.perf_counter()
    _lib.call("mqr_memcpy", _lib.ptr(a), _lib.MQR_HOST, ctypes.c_void_p(dev.data_ptr()), _lib.MQR_DEVICE, nbytes, 0)
    out["mqr_fresh_gbs"] = gbs(time.perf_counter() - t0)
    ok = bool(a[0] == 1.0 and a[-1] == 1.0)
    t0 = time.perf_counter()
    _lib.call("mqr_memcpy", _lib.ptr(a), _lib.MQR_HOST, ctypes.c_void_p(dev.data_ptr()), _lib.MQR_DEVICE, nbytes, 0)
    out["mqr_touched_gbs"] = gbs(time.perf_counter() - t0)
    out["values_ok"] = ok and bool(np.all(a[:: 1 << 16] == 1.0))
    del a
    h = _lib.host_empty(n, np.float32)
    t0 = time.perf_counter()
    _lib.call("mqr_memcpy", _lib.ptr(h), _lib.MQR_HOST, ctypes.c_void_p(dev.data_ptr()), _lib.MQR_DEVICE, nbytes, 0)
    out["mqr_fresh_host_empty_gbs"] = gbs(time.perf_counter() - t0)
    out["values_ok"] = out["values_ok"] and bool(np.all(h[:: 1 << 16] == 1.0) and h[-1] == 1.0)
    del h
    t0 = time.perf_counter()
    b = np.empty(n, np.float32)
    b.fill(0.0)
    out["first_touch_1thread_gbs"] = gbs(time.perf_counter() - t0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
