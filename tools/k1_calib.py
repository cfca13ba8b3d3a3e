"""K1 calibration on the GPU: throughput of the lanes kernel at several
message counts and the per-message chain rate of lanes vs solo mode.
Prints one line per case; used to set the planner constants."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reflow_amd import capi  # noqa: E402


def run_case(ctx, name, lens, flags, reps=3):
    lens = np.array(lens, dtype=np.uint64)
    offs = np.zeros(len(lens), dtype=np.uint64)
    pos = 0
    for i, n in enumerate(lens):
        offs[i] = pos
        pos += (int(n) + 255) // 256 * 256
    arena = ctx.alloc(max(pos, 16))
    d_offs = ctx.upload(offs)
    d_lens = ctx.upload(lens)
    out = ctx.alloc(len(lens) * 32)
    ctx.gen_fill(arena.ptr, d_offs.ptr, d_lens.ptr, len(lens), 1, arena.nbytes)
    ctx.sync()
    plan = ctx.sha_plan(offs, lens, flags)
    best = None
    for _ in range(reps):
        plan.run(arena.ptr, out.ptr)
        st = plan.stats()
        best = st.last_ms_total if best is None else min(best, st.last_ms_total)
    st = plan.stats()
    gbs = float(lens.sum()) / (best * 1e-3) / 1e9
    blocks = st.total_blocks
    ops = blocks * 1464
    print("%-28s n=%7d bytes=%.3e solo=%d  %.3f ms  %.1f GB/s  %.2f Tops/s(1464/blk)  maxblk=%d"
          % (name, len(lens), float(lens.sum()), st.n_solo, best, gbs, ops / (best * 1e-3) / 1e12,
             st.max_blocks), flush=True)
    plan.close()
    arena.free()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    ctx = capi.Context(0)
    KB, MB = 1024, 1024 * 1024
    run_case(ctx, "c1 4096x256KiB lanes", [256 * KB] * 4096, capi.RF_SHA_NO_SOLO)
    run_case(ctx, "c1 4096x256KiB plan", [256 * KB] * 4096, 0)
    run_case(ctx, "many 65536x64KiB", [64 * KB] * 65536, capi.RF_SHA_NO_SOLO)
    run_case(ctx, "many 262144x16KiB", [16 * KB] * 262144, capi.RF_SHA_NO_SOLO)
    run_case(ctx, "many 1048576x4KiB", [4 * KB] * 1048576, capi.RF_SHA_NO_SOLO)
    if not a.quick:
        run_case(ctx, "many 131072x64KiB", [64 * KB] * 131072, capi.RF_SHA_NO_SOLO)
    # single-message chain rates
    run_case(ctx, "1x16MiB lane", [16 * MB], capi.RF_SHA_NO_SOLO, reps=2)
    run_case(ctx, "1x16MiB solo(1-lane)", [16 * MB], capi.RF_SHA_ALL_SOLO | capi.RF_SHA_ONE_LANE_CHAIN, reps=2)
    run_case(ctx, "1x16MiB duo", [16 * MB], capi.RF_SHA_ALL_SOLO, reps=2)
    run_case(ctx, "256x4MiB solo", [4 * MB] * 256, capi.RF_SHA_ALL_SOLO, reps=2)
    run_case(ctx, "1024x4MiB solo", [4 * MB] * 1024, capi.RF_SHA_ALL_SOLO, reps=2)
    run_case(ctx, "1024x4MiB lanes", [4 * MB] * 1024, capi.RF_SHA_NO_SOLO, reps=2)


if __name__ == "__main__":
    main()
