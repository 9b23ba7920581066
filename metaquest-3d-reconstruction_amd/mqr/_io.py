"""Host file I/O threads shared by the drop-in loops (``o3d_utils.integrate`` reads raw depth +
confidence npz per frame, ``confidence.estimate_depth_confidences`` decodes frames and writes one
npz per reference frame).  File reads, ``np.load`` / ``np.savez`` spend their time in system calls
and memory copies that release the GIL, so a few threads multiply the host-side rate; order is
kept by the callers (``map`` / futures in submission order)."""
from __future__ import annotations

import os
import threading
from concurrent.futures import ThreadPoolExecutor

_pool = None
_lock = threading.Lock()


def io_threads() -> int:
    """MQR_IO_THREADS, else min(16, usable CPUs).  (16 against 8 on an MI355X box's 16-CPU share: the
    drop-in integrate's 500-frame call 37.7 -> 29.7 ms, its reads 12.6 -> 4.4 ms,
    profiles/r05_ab_io_threads.json.)"""
    env = os.environ.get("MQR_IO_THREADS")
    if env:
        return max(1, int(env))
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def io_pool() -> ThreadPoolExecutor:
    global _pool
    with _lock:
        if _pool is None:
            _pool = ThreadPoolExecutor(max_workers=io_threads(), thread_name_prefix="mqr-io")
        return _pool
