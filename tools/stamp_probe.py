"""One incremental step with RF_K2_STAMPS=1: prints workgroup 0's per-phase
times for every launched level (chain wave, producer wave) and the jobs
hashed per level.

  python tools/stamp_probe.py [S]        configs[2] (S samples, default 22075)
  python tools/stamp_probe.py c4 R       rank 0's piece of the 100M layout at R ranks
  python tools/stamp_probe.py ps R       rank 0's piece of the per-sample-root layout at R ranks
RF_K2_WGSTAMPS=1 (with RF_K2_STAMPS=0): per-workgroup start / end / CU of every level launch.
"""
import os
import sys

os.environ.setdefault("RF_K2_STAMPS", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reflow_amd import capi  # noqa: E402

# the stamps exist only in a diagnostic build (make -C reflow_amd/csrc
# EXTRA=-DRF_DIAG BUILD=build_diag OUT=../../tools/_ab/libreflow_diag.so ...):
# STAMP_LIB=path picks it
if os.environ.get("STAMP_LIB"):
    capi.LIB_PATH = os.path.abspath(os.environ["STAMP_LIB"])
from reflow_amd.workloads import Dag1000, PartitionedDag1000  # noqa: E402

ctx = capi.Context(0, host_threads=0)
if len(sys.argv) > 2 and sys.argv[1] == "ps":  # the per-sample-root layout's rank 0 of R (1: the whole 100M DAG)
    dag = Dag1000(27594 * 8 // int(sys.argv[2]), 32)
    desc, n_global = dag.arrays(), 2 * 32 * 27594 * 8
elif len(sys.argv) > 2 and sys.argv[1] == "c4":
    pc = PartitionedDag1000(27594, 32, int(sys.argv[2]), 0, nparts=8)
    dag, desc, n_global = pc.dag, pc.desc, 2 * 32 * 27594 * 8
else:
    dag = Dag1000(int(sys.argv[1]) if len(sys.argv) > 1 else 22075, 32)
    desc, n_global = dag.arrays(), None
print("built: %d jobs" % len(desc["out_slot"]), flush=True)
g = capi.Graph.from_arrays(ctx, desc)
print("loaded", flush=True)
g.set_slots(dag.file_slots, dag.leaf_ids)
g.recompute(full=True)
print("full recompute done", flush=True)
slots, old, new = dag.change_set(0.01, n_global=n_global) if n_global else dag.change_set(0.01)
for v in (new, old, new):
    g.set_slots(slots, v)
    print("recomputed", g.recompute(full=False), flush=True)
g.close()
ctx.close()
