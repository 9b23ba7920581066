"""Large host <-> device copies.  Downloads into pageable memory from 32 MiB on go through
csrc/extract.hip ring_copy (copy kernels into a ring of pinned slots, host threads copying them out),
used by mqr_memcpy, mqr_geom_copy and the host-array outputs of colouring, ray casting, confidence and
decoding; uploads use HIP's pageable path.  Byte-exact against torch's own copy for: more chunks than
ring slots, lengths that are not a multiple of the chunk or of 16 bytes, sources / destinations that are
not 16-byte aligned (byte-copy path), offsets inside larger arrays, page-locked host buffers (direct DMA),
and copies ordered behind a torch side stream's write (mqr_set_stream)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MIB = 1 << 20


def _copy(torch, src_t, nbytes, src_off=0, dst=None, dst_off=0):
    from mqr import _lib
    out = np.full(nbytes + dst_off + 7, 0xEE, np.uint8) if dst is None else dst
    _lib.call("mqr_memcpy", ctypes.c_void_p(out.ctypes.data + dst_off), _lib.MQR_HOST,
              ctypes.c_void_p(src_t.data_ptr() + src_off), _lib.MQR_DEVICE, nbytes, 0)
    return out


@pytest.mark.parametrize("nbytes,src_off", [
    (32 * MIB, 0),                 # the threshold, 4 chunks
    (200 * MIB + 12, 0),           # 26 chunks (> 8 ring slots), tail not a multiple of 16
    (97 * MIB + 5, 3),             # unaligned source: byte-copy kernel
    (64 * MIB, 16),                # aligned but offset source
])
def test_large_d2h_copy_exact(nbytes, src_off):
    import torch
    g = torch.Generator(device="cuda").manual_seed(nbytes)
    src = torch.randint(0, 256, (nbytes + src_off + 64,), dtype=torch.uint8, device="cuda", generator=g)
    ref = src.cpu().numpy()
    out = _copy(torch, src, nbytes, src_off=src_off, dst_off=5)
    assert np.array_equal(out[5:5 + nbytes], ref[src_off:src_off + nbytes])
    assert (out[:5] == 0xEE).all() and (out[5 + nbytes:] == 0xEE).all()  # nothing written outside


def test_large_d2h_copy_repeated_reuses_ring():
    import torch
    for i in range(3):
        src = torch.full((40 * MIB,), i + 1, dtype=torch.uint8, device="cuda")
        out = _copy(torch, src, src.numel())
        assert (out[:src.numel()] == i + 1).all()


def test_large_d2h_copy_ordered_after_caller_stream():
    """The source is written on a torch side stream behind a spin kernel; the copy is called inside
    torch.cuda.stream(s) with no synchronize, so only the stream ordering makes it see the write."""
    import torch
    from mqr import _lib
    n = 48 * MIB
    src = torch.zeros(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        torch.cuda._sleep(100_000_000)
        src.fill_(7)
        out = np.zeros(n, np.uint8)
        _lib.call("mqr_memcpy", ctypes.c_void_p(out.ctypes.data), _lib.MQR_HOST, ctypes.c_void_p(src.data_ptr()),
                  _lib.MQR_DEVICE, n, 0)
    assert (out == 7).all()


@pytest.mark.parametrize("nbytes,dst_off", [(32 * MIB, 0), (200 * MIB + 12, 0), (97 * MIB + 5, 3), (64 * MIB, 16)])
def test_large_h2d_copy_exact(nbytes, dst_off):
    import torch
    from mqr import _lib
    rng = np.random.default_rng(nbytes)
    host = rng.integers(0, 256, nbytes + 11, dtype=np.uint8)
    dev = torch.full((nbytes + dst_off + 64,), 0xEE, dtype=torch.uint8, device="cuda")
    _lib.call("mqr_memcpy", ctypes.c_void_p(dev.data_ptr() + dst_off), _lib.MQR_DEVICE,
              ctypes.c_void_p(host.ctypes.data + 11), _lib.MQR_HOST, nbytes, 0)
    back = dev.cpu().numpy()
    assert np.array_equal(back[dst_off:dst_off + nbytes], host[11:])
    assert (back[:dst_off] == 0xEE).all() and (back[dst_off + nbytes:] == 0xEE).all()


def test_large_copies_pinned_host_buffers():
    import torch
    from mqr import _lib
    n = 72 * MIB + 4
    src = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    pin = torch.empty(n, dtype=torch.uint8).pin_memory()
    _lib.call("mqr_memcpy", ctypes.c_void_p(pin.data_ptr()), _lib.MQR_HOST, ctypes.c_void_p(src.data_ptr()),
              _lib.MQR_DEVICE, n, 0)
    assert torch.equal(pin, src.cpu())
    dst = torch.zeros(n, dtype=torch.uint8, device="cuda")
    _lib.call("mqr_memcpy", ctypes.c_void_p(dst.data_ptr()), _lib.MQR_DEVICE, ctypes.c_void_p(pin.data_ptr()),
              _lib.MQR_HOST, n, 0)
    assert torch.equal(dst, src)
