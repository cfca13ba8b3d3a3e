"""K2/K3 HBM traffic against the algorithmic bytes: run this
under `rocprofv3 --pmc FETCH_SIZE` and again under `--pmc WRITE_SIZE`, then
tools/pmc_dag_summary.py.

    python tools/pmc_dag.py --c2            configs[2] (10M nodes), 1 % toggled
    python tools/pmc_dag.py --c4-ranks R    rank 0's piece of the 100M layout at R ranks (1 = the whole DAG)

The graph is loaded and fully recomputed, then STEPS incremental steps
(default forms) toggle the same 1 % change set.  stdout: one JSON line with
the per-step algorithmic bytes -- for every job the step re-hashed (its
output slot changed; early cut-off does not occur on these change sets):
8 (record) + 4 deg (hole slot ids) + 32 deg (child digests) + template bytes
+ 32 (the digest written), deg = its holes -- and the dirty blocks, so the
summary can divide each step's FETCH + WRITE bytes by them."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from reflow_amd import capi  # noqa: E402
from reflow_amd.workloads import Dag1000, PartitionedDag1000  # noqa: E402


def algorithmic(a, before, after):
    """Jobs whose output slot changed between two slot tables: their
    algorithmic bytes and blocks."""
    out = np.asarray(a["out_slot"], dtype=np.int64)
    ch = (before[out] != after[out]).any(axis=1)
    deg = np.diff(np.asarray(a["hole_ptr"], dtype=np.int64))
    ln = np.asarray(a["tmpl_len"], dtype=np.int64)
    blk = (ln + 9 + 63) // 64
    b = 8 + 4 * deg + 32 * deg + ln + 32
    return int(ch.sum()), int(b[ch].sum()), int(blk[ch].sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c2", action="store_true")
    ap.add_argument("--c4-ranks", type=int, default=0)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--lib", default="", help="another build of the library (A/B of builds)")
    args = ap.parse_args()
    if args.lib:
        capi.LIB_PATH = os.path.abspath(args.lib)
    ctx = capi.Context(0, host_threads=0)
    if args.c2:
        dag = Dag1000(22075, 32)
        a = dag.arrays()
        slots, old, new = dag.change_set(0.01)
        name = "configs[2]"
    else:
        pc = PartitionedDag1000(27594, 32, args.c4_ranks, 0, nparts=8)
        dag, a = pc.dag, pc.desc
        slots, old, new = dag.change_set(0.01, n_global=2 * 32 * 27594 * 8)
        name = "configs[3] rank 0 of %d" % args.c4_ranks
    g = capi.Graph.from_arrays(ctx, a)
    g.set_slots(dag.file_slots, dag.leaf_ids)
    g.recompute(True)
    every = np.arange(a["n_slots"], dtype=np.uint32)
    t_old = g.get_slots(every)
    d_slots, d_old, d_new = ctx.upload(slots), ctx.upload(old), ctx.upload(new)
    g.set_slots_device(d_slots.ptr, d_new.ptr, len(slots), ctx.stream)
    g.recompute_async(False, ctx.stream)
    ctx.sync()
    t_new = g.get_slots(every)
    jobs, byts, blocks = algorithmic(a, t_old, t_new)
    print("[pmc_dag] %s: %d jobs, %d algorithmic bytes, %d blocks per step" % (name, jobs, byts, blocks),
          file=sys.stderr, flush=True)
    # the profiled steps: back to old, then alternate (every step re-hashes
    # the same closure)
    for k in range(args.steps):
        ver = d_old if k % 2 == 0 else d_new
        g.set_slots_device(d_slots.ptr, ver.ptr, len(slots), ctx.stream)
        g.recompute_async(False, ctx.stream)
        ctx.sync()
    print(json.dumps({"graph": name, "steps": args.steps + 1, "jobs_per_step": jobs,
                      "algorithmic_bytes_per_step": byts, "dirty_blocks_per_step": blocks,
                      "changed_slots": int(len(slots)), "levels": int(g.stats().n_levels)}), flush=True)
    g.close()
    ctx.close()


if __name__ == "__main__":
    main()
