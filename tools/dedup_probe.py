"""Isolates rf_dedup_digests_device timing (diagnostic for a stall seen in
bench_canon): n random digests with 1% duplicates, timed calls."""
import faulthandler
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reflow_amd import capi  # noqa: E402

faulthandler.dump_traceback_later(60, exit=True)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
ctx = capi.Context(0, host_threads=0)
rng = np.random.default_rng(1)
dig = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
dig[n // 2:n // 2 + n // 100] = dig[:n // 100]
d = ctx.upload(dig)
canon, nu = ctx.alloc(4 * n), ctx.alloc(64)
for k in range(4):
    t = time.perf_counter()
    ctx.dedup_digests_device(d.ptr, n, canon.ptr, nu.ptr)
    print("call %d enqueued in %.3f s" % (k, time.perf_counter() - t), flush=True)
    ctx.sync()
    print("call %d done in %.3f s, unique %x" % (k, time.perf_counter() - t, int(nu.to_numpy()[:4].view(np.uint32)[0])),
          flush=True)
for k in range(3):
    ctx.timer_start()
    ctx.dedup_digests_device(d.ptr, n, canon.ptr, nu.ptr)
    print("timed %d: %.3f ms" % (k, ctx.timer_stop()), flush=True)
