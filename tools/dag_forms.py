"""A/B of the incremental level-kernel forms on the bench's DAGs, one process,
one graph load each: every level in k2_level_pl (two-lane latency form), every
level in k2_level_lf (lane-per-job throughput form), and the library's
per-level choice -- set between steps by rf_graph_set_forms.  For each
graph: ms/step of each form over the same toggled 1 % change set, and every
slot of each form compared after an odd step.

  python tools/dag_forms.py [--c2] [--c4-ranks 1,2,4,8] [--steps 20]

--c4-ranks r: rank 0's piece of the strong-scaling 100M-node layout at r
ranks (the local step only, no exchange): what one GPU of an r-GPU run hashes.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from reflow_amd import capi  # noqa: E402
from reflow_amd.workloads import Dag1000, PartitionedDag1000  # noqa: E402

# pl: every level in the latency form; lf: every level in the throughput
# form; auto: the library's per-level choice (the default thresholds)
FORMS = {"pl": capi.Graph.NEVER, "lf": 0, "auto": None}
# --extra: also "lfs" (levels of short jobs lane-per-job, levels of long jobs
# in the latency form) and "plw" (the reverse)
EXTRA = {"lfs": (capi.Graph.THRU_DEFAULT, capi.Graph.NEVER, capi.Graph.THRU_MARK_DEFAULT),
         "plw": (capi.Graph.NEVER, 0, capi.Graph.THRU_MARK_DEFAULT)}


def run(ctx, name, g, slots, old, new, steps):
    d_slots = ctx.upload(slots)
    d_old, d_new = ctx.upload(old), ctx.upload(new)
    every = np.arange(g.stats().n_slots, dtype=np.uint32)
    res = {"graph": name, "changed_slots": int(len(slots))}
    snaps = {}
    for rep in range(2):
        for form, thr in FORMS.items():
            if thr is None:
                g.set_forms(g.THRU_DEFAULT, g.THRU_WIDE_DEFAULT, g.THRU_MARK_DEFAULT)
            elif isinstance(thr, tuple):
                g.set_forms(*thr)
            else:
                g.set_forms(thr)
            state = {"v": 0}

            def step():
                ver = d_new if state["v"] == 0 else d_old
                state["v"] ^= 1
                g.set_slots_device(d_slots.ptr, ver.ptr, len(slots), ctx.stream)
                g.recompute_async(False, ctx.stream)

            for _ in range(2):
                step()
            ctx.sync()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            ctx.sync()
            ms = (time.perf_counter() - t0) / steps * 1e3
            res.setdefault(form, []).append(round(ms, 4))
            if rep == 0:  # an odd step: the changed version everywhere
                step()
                ctx.sync()
                snaps[form] = g.get_slots(every)
                step()
                ctx.sync()
            st = g.stats()
            print(name, form, "%.4f ms/step" % ms, "(sinks on level %d, lf levels %d, octo levels %d, half levels %d, "
                  "split %d)" % (st.last_sink_attach if st.last_sink_attach != 0xFFFFFFFF else -1,
                                 st.last_levels_lf, st.last_levels_oct, st.last_levels_half, st.split_block0),
                  file=sys.stderr, flush=True)
    res["slots_equal"] = bool(all((snaps["pl"] == snaps[f]).all() for f in snaps))
    g.set_forms(g.THRU_DEFAULT, g.THRU_WIDE_DEFAULT, g.THRU_MARK_DEFAULT)
    for b in (d_slots, d_old, d_new):
        b.free()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c2", action="store_true")
    ap.add_argument("--c4-ranks", default="")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--lib", default="", help="another build of the library (A/B of builds)")
    ap.add_argument("--persample", default="", help="per-sample-root layout (SURVEY C3/C4): ranks, e.g. 8,1")
    ap.add_argument("--extra", action="store_true", help="also the mixed forms (EXTRA)")
    a = ap.parse_args()
    if a.extra:
        FORMS.update(EXTRA)
    if a.lib:
        capi.LIB_PATH = os.path.abspath(a.lib)
        print("library: %s" % capi.LIB_PATH, file=sys.stderr)
    import faulthandler
    faulthandler.dump_traceback_later(500, exit=True)
    ctx = capi.Context(0, host_threads=0)
    out = []
    if a.c2:
        dag = Dag1000(22075, 32)
        g = capi.Graph.from_arrays(ctx, dag.arrays())
        g.set_slots(dag.file_slots, dag.leaf_ids)
        g.recompute(True)
        slots, old, new = dag.change_set(0.01)
        out.append(run(ctx, "configs[2]", g, slots, old, new, a.steps))
        g.close()
        del dag
    for r in [int(x) for x in a.c4_ranks.split(",") if x]:
        t0 = time.perf_counter()
        pc = PartitionedDag1000(27594, 32, r, 0, nparts=8)
        g = capi.Graph.from_arrays(ctx, pc.desc)
        g.set_slots(pc.dag.file_slots, pc.dag.leaf_ids)
        g.recompute(True)
        slots, old, new = pc.dag.change_set(0.01, n_global=2 * 32 * 27594 * 8)
        print("c4 r=%d loaded in %.1f s" % (r, time.perf_counter() - t0), file=sys.stderr, flush=True)
        res = run(ctx, "configs[3] rank 0 of %d (%d nodes)" % (r, pc.n_nodes), g, slots, old, new, a.steps)
        out.append(res)
        g.close()
        del pc, g
    for r in [int(x) for x in a.persample.split(",") if x]:
        # SURVEY §8(d) C3/C4 as written: per-sample roots, no Merge tree; rank
        # 0's piece at r ranks is its first 8/r parts' samples (no exchange)
        t0 = time.perf_counter()
        dag = Dag1000(27594 * 8 // r, 32)
        g = capi.Graph.from_arrays(ctx, dag.arrays())
        g.set_slots(dag.file_slots, dag.leaf_ids)
        g.recompute(True)
        slots, old, new = dag.change_set(0.01, n_global=2 * 32 * 27594 * 8)
        print("per-sample r=%d loaded in %.1f s" % (r, time.perf_counter() - t0), file=sys.stderr, flush=True)
        out.append(run(ctx, "per-sample roots, rank 0 of %d (%d samples)" % (r, 27594 * 8 // r), g, slots, old,
                       new, a.steps))
        g.close()
        del dag, g
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
