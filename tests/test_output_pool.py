"""decode_bits' recycled output buffers (ldpc_amd.api._OutputPool): a returned array is reused only after the
caller has dropped it and every view of it, always comes back with its tail rows zero, and the pool holds at
most `keep` free buffers within `max_bytes` (CPU only: the pool is host-side)."""
import gc

import numpy as np

from ldpc_amd.api import _OutputPool


def test_reuse_only_after_release_and_tail_zeroed():
    pool = _OutputPool(keep=2, max_bytes=1 << 26)
    a = pool.array((10, 8), 7)
    assert a.shape == (10, 8) and a.dtype == np.float64 and not a[7:].any()
    a[:] = 5.0
    pa = a.ctypes.data
    b = pool.array((10, 8), 7)
    assert b.ctypes.data != pa                     # a is alive: a different buffer
    v = a[:3].T[1:]                                # a view (of a view) keeps a's buffer out of the pool
    del a
    gc.collect()
    c = pool.array((10, 8), 4)
    assert c.ctypes.data not in (pa, b.ctypes.data)
    del v
    gc.collect()
    d = pool.array((10, 8), 4)                     # now a's buffer is free: reused, tail zeroed
    assert d.ctypes.data == pa and not d[4:].any() and (d[:4] == 5.0).all()
    e = pool.array((3, 8), 3)                      # another size: its own buffer
    assert e.shape == (3, 8) and e.ctypes.data != pa


def test_pool_bounds():
    pool = _OutputPool(keep=1, max_bytes=10 * 8 * 8 * 2)
    arrs = [pool.array((10, 8), 10) for _ in range(3)]
    del arrs
    gc.collect()
    assert pool.free_count() == 1
    big = pool.array((100, 100), 0)                # larger than max_bytes: a plain np.zeros, not pooled
    assert not big.any() and big.shape == (100, 100)


def test_release_from_gc_inside_the_lock_does_not_deadlock():
    """an array in a reference cycle is freed by the cyclic GC, which can run on the thread that
    already holds the pool's lock (inside array()).  The finalizer must not take that lock."""
    import threading
    pool = _OutputPool(keep=2, max_bytes=1 << 26)
    done = threading.Event()

    def body():
        a = pool.array((6, 4), 6)
        cyc = [a]
        cyc.append(cyc)                 # a reference cycle: only the cyclic GC frees `a`
        del a, cyc
        with pool._lock:                # as inside array(): the GC pass runs with the lock held
            gc.collect()
        done.set()

    gc.disable()
    try:
        t = threading.Thread(target=body, daemon=True)
        t.start()
        t.join(10)
    finally:
        gc.enable()
    assert done.is_set(), "finalizer deadlocked on the pool lock"
    assert pool.free_count() == 1        # the buffer came back through the lock-free path
    b = pool.array((6, 4), 2)
    assert not b[2:].any()
