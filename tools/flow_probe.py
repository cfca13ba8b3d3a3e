"""Diagnostic: synchronous flow steps on configs[3]'s 100M-node DAG (or a
piece) with a library built -DRF_FLOW_PROFILE (the flow kernel's per-wave
tallies printed by rf_graph_recompute on stderr).

  make -C reflow_amd/csrc EXTRA=-DRF_FLOW_PROFILE BUILD=build_prof OUT=../../tools/_prof/libreflow_hip.so \
      ../../tools/_prof/libreflow_hip.so
  python tools/flow_probe.py [--ranks 1] [--steps 3]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from reflow_amd import capi  # noqa: E402
from reflow_amd.workloads import PartitionedDag1000  # noqa: E402

_PROF = os.environ.get("FLOW_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_prof",
                                                   "libreflow_hip.so")
if os.path.exists(_PROF):  # the diagnostic build, if made
    capi.LIB_PATH = _PROF


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=1)
    ap.add_argument("--samples", type=int, default=27594)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--flow", type=int, default=1)
    a = ap.parse_args()
    ctx = capi.Context(0, host_threads=0)
    pc = PartitionedDag1000(a.samples, 32, a.ranks, 0, nparts=8)
    g = capi.Graph.from_arrays(ctx, pc.desc)
    g.set_slots(pc.dag.file_slots, pc.dag.leaf_ids)
    g.recompute(True)
    g.set_flow(a.flow)
    slots, old, new = pc.dag.change_set(0.01, n_global=2 * 32 * a.samples * 8)
    for i in range(a.steps):
        g.set_slots(slots, new if i % 2 == 0 else old)
        t0 = time.perf_counter()
        n = g.recompute(False)
        st = g.stats()
        print("step %d: %d jobs, %.3f ms (device %.3f ms), flow %d" % (i, n, (time.perf_counter() - t0) * 1e3,
                                                                    st.last_ms, st.last_flow), file=sys.stderr, flush=True)
    g.close()
    ctx.close()


if __name__ == "__main__":
    main()
