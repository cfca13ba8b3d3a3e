"""Bisects the round-2 failure of per-call stream-ordered pool scratch in
rf_dedup_digests_device (DESIGN.md §5 "Device-form scratch"): the library's
own dedup kernels with the scratch taken per call from the default memory
pool (RF_DEDUP_SCRATCH=pool*, capi.cpp dedup_pool_diag), called back to back
on one stream, then on a second context's stream.  Every call must give
exactly n - n/100 classes (digests are random, 1% are copies).

    python tools/pool_diag.py <mode> [n]     mode: scratch | pool | pool_sync | pool_fill | pool_nothresh
"""
import faulthandler
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mode = sys.argv[1]
if mode != "scratch":
    os.environ["RF_DEDUP_SCRATCH"] = mode
from reflow_amd import capi  # noqa: E402

faulthandler.dump_traceback_later(120, exit=True)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
ctx = capi.Context(0, host_threads=0)
rng = np.random.default_rng(1)
dig = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
dig[n // 2:n // 2 + n // 100] = dig[:n // 100]
want = n - n // 100
d = ctx.upload(dig)
canon, nu = ctx.alloc(4 * n), ctx.alloc(64)
bad = 0


def one(tag, stream=None, c=ctx):
    global bad
    t = time.perf_counter()
    ctx.dedup_digests_device(d.ptr, n, canon.ptr, nu.ptr, stream=stream)
    c.sync()
    dt = (time.perf_counter() - t) * 1e3
    got = int(nu.to_numpy()[:4].view(np.uint32)[0])
    cn = canon.to_numpy().view(np.uint32)
    ok = got == want and bool((cn[n // 2:n // 2 + n // 100] == np.arange(n // 100)).all())
    bad += not ok
    print("%-14s %-9s %8.2f ms  unique %#010x (want %#010x)  %s" % (mode, tag, dt, got, want, "ok" if ok else "WRONG"),
          flush=True)


for k in range(6):
    one("call%d" % k)
c2 = capi.Context(0, host_threads=0)
for k in range(3):
    one("stream2_%d" % k, stream=c2.stream, c=c2)
    one("back_%d" % k)
c2.close()
print("%s: %d wrong of 12" % (mode, bad), flush=True)
sys.exit(1 if bad else 0)
