#!/usr/bin/env python3
"""Device -> host copy ceilings on this box (the C5 mesh copy, bench c5.extract_ms): 1 GiB from HBM into
(a) torch pinned memory, (b) a fresh pageable torch tensor (.cpu()), (c) mqr_memcpy into a fresh numpy
array (first-touch page faults inside the copy) and (d) into the same array again (pages present), and
(e) the cost of first-touching a fresh array alone (np.empty + fill, one thread), (f) mqr_memcpy into a
fresh 2 MiB-aligned private MADV_HUGEPAGE mapping and (g) into a second fresh np.empty array.  (c) is the
process's first large copy and also pays the staging set-up (pinned buffers, streams, threads): compare
(g), not (c), with (f).
MQR_D2H_THREADS sets the host threads of libmqr's staged copy (default 8).  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))


def huge_empty(nbytes):
    """float32 array over a 2 MiB-aligned private anonymous mapping advised MADV_HUGEPAGE (MAP_PRIVATE:
    Python's default anonymous mmap is shared memory, whose huge pages follow shmem_enabled)."""
    import mmap
    import numpy as np
    mm = mmap.mmap(-1, nbytes + (2 << 20), flags=mmap.MAP_PRIVATE)
    view = ctypes.c_char.from_buffer(mm)
    off = (-ctypes.addressof(view)) % (2 << 20)
    del view
    mm.madvise(mmap.MADV_HUGEPAGE, off, nbytes)
    return np.frombuffer(mm, np.float32, nbytes // 4, off)


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
    small = np.empty((48 << 20) // 4, np.float32)  # above the parallel threshold (32 MiB)
    for name in ("first_48mb_copy_ms", "second_48mb_copy_ms"):
        t0 = time.perf_counter()
        _lib.call("mqr_memcpy", _lib.ptr(small), _lib.MQR_HOST, ctypes.c_void_p(dev.data_ptr()), _lib.MQR_DEVICE,
                  small.nbytes, 0)
        out[name] = (time.perf_counter() - t0) * 1e3
    del small
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
    for name in ("mqr_fresh_hugepage_gbs", "mqr_second_fresh_gbs"):
        h = huge_empty(nbytes) if name == "mqr_fresh_hugepage_gbs" else np.empty(n, np.float32)
        t0 = time.perf_counter()
        _lib.call("mqr_memcpy", _lib.ptr(h), _lib.MQR_HOST, ctypes.c_void_p(dev.data_ptr()), _lib.MQR_DEVICE, nbytes, 0)
        out[name] = gbs(time.perf_counter() - t0)
        out["values_ok"] = out["values_ok"] and bool(np.all(h[:: 1 << 16] == 1.0) and h[-1] == 1.0)
        del h
    src = np.ones(n, np.float32)  # uploads from a present pageable array: torch, then the ring (mqr_memcpy)
    best_t, best_m = 1e9, 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        dev.copy_(torch.from_numpy(src))
        torch.cuda.synchronize()
        best_t = min(best_t, time.perf_counter() - t0)
        t0 = time.perf_counter()
        _lib.call("mqr_memcpy", ctypes.c_void_p(dev.data_ptr()), _lib.MQR_DEVICE, _lib.ptr(src), _lib.MQR_HOST, nbytes, 0)
        best_m = min(best_m, time.perf_counter() - t0)
    out["torch_h2d_pageable_gbs"] = gbs(best_t)
    out["mqr_h2d_pageable_gbs"] = gbs(best_m)
    out["values_ok"] = out["values_ok"] and bool(dev[:: 1 << 16].eq(1.0).all().item())
    del src
    t0 = time.perf_counter()
    b = np.empty(n, np.float32)
    b.fill(0.0)
    out["first_touch_1thread_gbs"] = gbs(time.perf_counter() - t0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
