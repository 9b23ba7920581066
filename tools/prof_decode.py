#!/usr/bin/env python3
"""The bench's ingest leg alone (mqr_decode_depth over 500 x 640x480 device-resident frames), for
`rocprofv3 --kernel-trace --stats -- python3 tools/prof_decode.py`: kernel time vs the call's wall
time, for the four (float64 denominator, confidence mask) combinations."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from mqr import _lib
    _lib.load()
    B, H, W = 500, 480, 640
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    raw = torch.rand((B, H, W), generator=g, device=dev)
    conf = torch.rand((B, H, W), generator=g, device=dev, dtype=torch.float64)
    vc = torch.randint(0, 8, (B, H, W), generator=g, device=dev, dtype=torch.int32)
    out = torch.empty_like(raw)
    nears, fars = np.full(B, 0.1), np.full(B, np.inf)
    ok = np.zeros(B, np.uint8)
    for strong in (0, 3):
        for mask in (0, 1):
            st = np.full(B, strong, np.uint8)
            has = np.full(B, mask, np.uint8)
            times = []
            for _ in range(5):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                _lib.call("mqr_decode_depth", 0, ctypes.c_void_p(raw.data_ptr()), 1, B, H, W,
                          _lib.ptr(nears, _lib._f64p), _lib.ptr(fars, _lib._f64p), _lib.ptr(st, _lib._u8p),
                          ctypes.c_void_p(conf.data_ptr()), ctypes.c_void_p(vc.data_ptr()), _lib.ptr(has, _lib._u8p),
                          1, 0.3, 2, ctypes.c_void_p(out.data_ptr()), 1, _lib.ptr(ok, _lib._u8p))
                times.append(time.perf_counter() - t0)
            t = float(np.median(times[1:]))
            nbytes = (20 if mask else 8) * H * W * B
            print(json.dumps({"strong": strong, "mask": mask, "ms": t * 1e3, "alg_gbs": nbytes / t / 1e9}),
                  flush=True)


if __name__ == "__main__":
    main()
