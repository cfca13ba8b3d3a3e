"""Smoke check of a diagnostic build (-DRF_DIAG): a small 1000align DAG
loaded, fully recomputed and stepped once with the library at argv[1],
progress printed after each call, every slot compared with the oracle."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import numpy as np  # noqa: E402

from reflow_amd import capi  # noqa: E402

capi.LIB_PATH = os.path.abspath(sys.argv[1])
from reflow_amd.workloads import Dag1000  # noqa: E402
import reflow_oracle as O  # noqa: E402

ctx = capi.Context(0, host_threads=0)
print("ctx", flush=True)
dag = Dag1000(20, 4)
a = dag.arrays()
g = capi.Graph.from_arrays(ctx, a)
print("loaded", flush=True)
g.set_slots(dag.file_slots, dag.leaf_ids)
print("set", flush=True)
g.recompute(full=True)
print("full", flush=True)
sl, _, nv = dag.change_set(0.1)
g.set_slots(sl, nv)
n = g.recompute(full=False)
print("incremental", n, flush=True)
og = O.OGraph(a)
og.set_inputs(dag.file_slots, dag.leaf_ids)
og.full()
og.update(sl, nv)
every = np.arange(a["n_slots"], dtype=np.uint32)
print("equal", bool((g.get_slots(every) == og.slots[:a["n_slots"]]).all()), flush=True)
g.close()
ctx.close()
