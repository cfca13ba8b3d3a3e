"""Diagnostic: the wave-per-message (duo) SHA path on single messages of
chosen lengths against hashlib; prints one line per length."""
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reflow_amd import capi  # noqa: E402


def main():
    ctx = capi.Context(0)
    lens = [0, 1, 55, 56, 64, 119, 120, 127, 128, 64 * 63 - 9, 64 * 64 - 9, 64 * 64, 64 * 65, 64 * 128,
            64 * 129 + 3, 69804, 300000]
    rng = np.random.default_rng(5)
    for flags in (capi.RF_SHA_ALL_SOLO, capi.RF_SHA_ALL_SOLO | capi.RF_SHA_ONE_LANE_CHAIN):
        for n in lens:
            m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            offs = np.array([0], dtype=np.uint64)
            ln = np.array([n], dtype=np.uint64)
            arena = ctx.upload(np.frombuffer(m + b"\0" * 256, dtype=np.uint8))
            out = ctx.alloc(32)
            plan = ctx.sha_plan(offs, ln, flags)
            plan.run(arena.ptr, out.ptr)
            ctx.sync()
            got = out.to_numpy().tobytes()
            print("flags=%d len=%7d blocks=%5d %s" % (flags, n, (n + 72) // 64,
                  "ok" if got == hashlib.sha256(m).digest() else "MISMATCH"), flush=True)
            plan.close()


if __name__ == "__main__":
    main()
