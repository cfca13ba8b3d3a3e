"""One configs[2] incremental step with RF_K2_STAMPS=1: prints workgroup 0's
per-phase times for every launched level (chain wave, producer wave)."""
import os
import sys

os.environ.setdefault("RF_K2_STAMPS", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reflow_amd import capi  # noqa: E402
from reflow_amd.workloads import Dag1000  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 22075
ctx = capi.Context(0, host_threads=0)
dag = Dag1000(S, 32)
g = capi.Graph.from_arrays(ctx, dag.arrays())
g.set_slots(dag.file_slots, dag.leaf_ids)
g.recompute(full=True)
slots, old, new = dag.change_set(0.01)
for v in (new, old, new):
    g.set_slots(slots, v)
    print("recomputed", g.recompute(full=False), flush=True)
g.close()
ctx.close()
