"""Diagnostic: the K1 host leg's rate on this box.  16 x 1 GiB messages in
HBM, every one on the host leg (RF_SHA_ALL_HOST), at several thread counts;
with RF_HOST_LEG_TIMING=1 the library prints per-run wait/hash sums."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from reflow_amd import capi  # noqa: E402
from reflow_amd.workloads import GiB, arena_layout  # noqa: E402

ctx = capi.Context(0)
print("host_info", ctx.host_info(), flush=True)
n = int(os.environ.get("PROBE_FILES", "32"))
size = int(float(os.environ.get("PROBE_GIB", "1")) * GiB)
lens = np.full(n, size, dtype=np.uint64)
offs, tot = arena_layout(lens)
arena = ctx.alloc(tot)
d_o, d_l = ctx.upload(offs), ctx.upload(lens)
out = ctx.alloc(32 * n)
ctx.gen_fill(arena.ptr, d_o.ptr, d_l.ptr, n, 5, tot)
ctx.sync()
for th in [int(x) for x in os.environ.get("PROBE_THREADS", "8,12,14,16,20,24,32").split(",")]:
    ctx.set_host_threads(th)
    plan = ctx.sha_plan(offs, lens, capi.RF_SHA_ALL_HOST)
    plan.run(arena.ptr, out.ptr)  # warm (stages)
    ctx.sync()
    t0 = time.perf_counter()
    plan.run(arena.ptr, out.ptr)
    ctx.sync()
    dt = time.perf_counter() - t0
    print("threads %2d: %.2f GB/s (%.1f ms)" % (th, n * size / dt / 1e9, dt * 1e3), flush=True)
    plan.close()

if os.environ.get("PROBE_C2"):
    from reflow_amd.workloads import c2_sizes
    arena.free()
    lens = c2_sizes(total_bytes=64 * GiB, seed=0x5EED0002)
    offs, tot = arena_layout(lens)
    arena = ctx.alloc(tot)
    d_o, d_l = ctx.upload(offs), ctx.upload(lens)
    out = ctx.alloc(32 * len(lens))
    ctx.gen_fill(arena.ptr, d_o.ptr, d_l.ptr, len(lens), 0x5EED0002, tot)
    ctx.sync()
    ctx.set_host_threads(None)
    for name, flags in [("c2 all-host", capi.RF_SHA_ALL_HOST), ("c2 hybrid", 0), ("c2 all-host", capi.RF_SHA_ALL_HOST),
                        ("c2 hybrid", 0), ("c2 hybrid", 0)]:
        plan = ctx.sha_plan(offs, lens, flags)
        t0 = time.perf_counter()
        plan.run(arena.ptr, out.ptr)
        st = plan.stats()
        dt = time.perf_counter() - t0
        print("%s: %.2f GB/s (%.1f ms) host %d files %.1f GiB in %.1f ms, duo %d %.1f ms, lanes %.1f ms"
              % (name, lens.sum() / dt / 1e9, dt * 1e3, st.n_host, st.host_bytes / GiB, st.last_ms_host,
                 st.n_solo, st.last_ms_solo, st.last_ms_lanes), flush=True)
        plan.close()
