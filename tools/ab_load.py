"""Same-process A/B of a load-time option: the bench DAG loaded twice (B with
an environment variable set during its load, read per load by
rf_graph_load), then timed blocks of incremental steps alternating A, B, A,
B ... on the same change set (box drift hits both alike), the library's
default forms; every slot of A and B compared at the end.

  python tools/ab_load.py --env RF_K2_SPLIT=1 [--c2] [--c4-ranks 1] [--reps 6] [--steps 10] [--wg]

Calibration (an A/A run, --env RF_AB_NOTHING=1): at 100M nodes the second
graph (B) steps ~0.017 ms faster with nothing changed; configs[2] and the
8-rank piece are within 0.6 us.
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from reflow_amd import capi  # noqa: E402
from reflow_amd.workloads import Dag1000, PartitionedDag1000  # noqa: E402


def ab(ctx, name, desc, file_slots, leaf_ids, change, env, reps, steps, wg=False):
    k, v = env.split("=", 1)
    graphs = []
    for setenv in (False, True):
        if setenv:
            os.environ[k] = v
        if wg:
            os.environ["RF_K2_WGSTAMPS"] = "1"
        g = capi.Graph.from_arrays(ctx, desc)
        os.environ.pop(k, None)
        os.environ.pop("RF_K2_WGSTAMPS", None)
        g.set_slots(file_slots, leaf_ids)
        g.recompute(True)
        graphs.append(g)
    slots, old, new = change
    d_slots, d_old, d_new = ctx.upload(slots), ctx.upload(old), ctx.upload(new)
    times = {"A": [], "B": []}
    ver = {"A": 0, "B": 0}

    def step(tag, g):
        g.set_slots_device(d_slots.ptr, (d_new if ver[tag] == 0 else d_old).ptr, len(slots), ctx.stream)
        ver[tag] ^= 1
        g.recompute_async(False, ctx.stream)

    for rep in range(reps):
        for tag, g in (("A", graphs[0]), ("B", graphs[1])):
            for _ in range(2):
                step(tag, g)
            ctx.sync()
            t0 = time.perf_counter()
            for _ in range(steps):
                step(tag, g)
            ctx.sync()
            times[tag].append(round((time.perf_counter() - t0) / steps * 1e3, 4))
    every = np.arange(graphs[0].stats().n_slots, dtype=np.uint32)
    for tag, g in (("A", graphs[0]), ("B", graphs[1])):
        if ver[tag] == 0:  # both at the changed version
            step(tag, g)
    ctx.sync()
    if wg:  # one synchronous step each, back and forth (the library prints its per-level records)
        for tag, g in (("A", graphs[0]), ("B", graphs[1])):
            for rep in range(2):
                print("[ab] %s step %d" % (tag, rep), file=sys.stderr, flush=True)
                g.set_slots(slots, old if rep == 0 else new)
                g.recompute(False)
    equal = bool((graphs[0].get_slots(every) == graphs[1].get_slots(every)).all())
    res = {"graph": name, "env_B": env, "A_ms": times["A"], "B_ms": times["B"],
           "A_median": statistics.median(times["A"]), "B_median": statistics.median(times["B"]),
           "slots_equal": equal}
    print(json.dumps(res), file=sys.stderr, flush=True)
    for b in (d_slots, d_old, d_new):
        b.free()
    for g in graphs:
        g.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", required=True)
    ap.add_argument("--c2", action="store_true")
    ap.add_argument("--c4-ranks", default="")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--wg", action="store_true", help="per-level workgroup records (RF_K2_WGSTAMPS) after the timing")
    a = ap.parse_args()
    import faulthandler
    faulthandler.dump_traceback_later(500, exit=True)
    ctx = capi.Context(0, host_threads=0)
    out = []
    if a.c2:
        dag = Dag1000(22075, 32)
        out.append(ab(ctx, "configs[2]", dag.arrays(), dag.file_slots, dag.leaf_ids, dag.change_set(0.01), a.env,
                      a.reps, a.steps, a.wg))
        del dag
    for r in [int(x) for x in a.c4_ranks.split(",") if x]:
        pc = PartitionedDag1000(27594, 32, r, 0, nparts=8)
        out.append(ab(ctx, "configs[3] rank 0 of %d" % r, pc.desc, pc.dag.file_slots, pc.dag.leaf_ids,
                      pc.dag.change_set(0.01, n_global=2 * 32 * 27594 * 8), a.env, a.reps, a.steps, a.wg))
        del pc
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
