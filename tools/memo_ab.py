"""A/B of K2's memoized chaining values on one box: the same DAG loaded twice
(RF_K2_MEMO=1 / 0, read per load), steps timed alternately, the slot tables
compared, and the blocks memo jobs skipped per step (rf_graph_memo_stats).
  python tools/memo_ab.py --layout mt|ps|c2 [--steps 20] [--reps 3]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

from reflow_amd import capi  # noqa: E402
from reflow_amd.workloads import Dag1000, PartitionedDag1000  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="mt")
    ap.add_argument("--ranks", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    ctx = capi.Context(0, host_threads=0)
    if a.layout == "mt":
        pc = PartitionedDag1000(27594, 32, a.ranks, 0, nparts=8)
        desc, dag = pc.desc, pc.dag
        n_global = 2 * 32 * 27594 * 8
    elif a.layout == "ps":
        dag = Dag1000(27594 * 8 // a.ranks, 32)
        desc, n_global = dag.arrays(), 2 * 32 * 27594 * 8
    else:
        dag = Dag1000(22075, 32)
        desc, n_global = dag.arrays(), None
    slots, old, new = dag.change_set(0.01, n_global=n_global)
    gs = {}
    for m in ("1", "0"):
        os.environ["RF_K2_MEMO"] = m
        g = capi.Graph.from_arrays(ctx, desc)
        g.set_slots(dag.file_slots, dag.leaf_ids)
        g.recompute(True)
        gs[m] = g
    os.environ.pop("RF_K2_MEMO")
    d_slots, d_old, d_new = ctx.upload(slots), ctx.upload(old), ctx.upload(new)
    every = np.arange(desc["n_slots"], dtype=np.uint32)
    res = {"layout": a.layout, "ranks": a.ranks, "changed": int(len(slots)),
           "memo_jobs": gs["1"].memo_stats()[0], "memo_entries": gs["1"].memo_stats()[1], "ms": {"1": [], "0": []}}
    state = {m: 0 for m in gs}

    def step(m):
        g = gs[m]
        ver = d_new if state[m] == 0 else d_old
        state[m] ^= 1
        g.set_slots_device(d_slots.ptr, ver.ptr, len(slots), ctx.stream)
        g.recompute_async(False, ctx.stream)

    for rep in range(a.reps):
        for m in ("1", "0"):
            for _ in range(4):
                step(m)
            ctx.sync()
            s0 = gs[m].memo_stats()[2]
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step(m)
            ctx.sync()
            ms = (time.perf_counter() - t0) / a.steps * 1e3
            res["ms"][m].append(round(ms, 4))
            if m == "1":
                res.setdefault("skipped_blocks_per_step", []).append((gs[m].memo_stats()[2] - s0) / a.steps)
            print("rep %d memo=%s %.4f ms/step" % (rep, m, ms), file=sys.stderr, flush=True)
    for m in gs:
        if state[m]:
            step(m)
    ctx.sync()
    res["slots_equal"] = bool((gs["1"].get_slots(every) == gs["0"].get_slots(every)).all())
    print(json.dumps(res), flush=True)
    for g in gs.values():
        g.close()
    ctx.close()


if __name__ == "__main__":
    main()
