"""The throughput forms the library picks BY ITSELF (no RF_K2_THRU override,
no rf_graph_set_forms), against the oracle.

A change set of >= 98,304 input slots marks in k3_mark_slots_lf, and a level
that can receive >= 24,576 chains (min(level jobs, marked slots)) runs in
k2_level_lf -- the forms configs[3]'s 100M-node step takes on one GPU.  Here
a 1000align DAG of 1,600 samples x 32 pairs (102,400 leaf files, ~0.73M
nodes, the oracle's size) changes 97 % and then 100 % of its File IDs: the
step's choice is read back (rf_graph_stats: last_mark_lf, last_levels_lf),
and every job of the GPU's table is re-derived by the oracle from the
table's own holes (orc_graph_check, flow.go:675-750 per node), with the input
slots at their assigned values -- parity of the whole table with the full
evaluation.  The serial oracle (orc_graph_update) then replays the same
change and every slot is compared, and stepping back must give the full
recompute's table."""
import numpy as np
import pytest

import reflow_oracle as O
from reflow_amd.workloads import Dag1000
from test_gpu_dag import load

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from reflow_amd import capi
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


@pytest.mark.parametrize("frac", [0.97, 1.0])
def test_default_throughput_forms_match_oracle(ctx, frac):
    from reflow_amd import capi
    dag = Dag1000(1600, 32)
    a = dag.arrays()
    every = np.arange(a["n_slots"], dtype=np.uint32)
    g = load(ctx, dag)
    g.recompute(full=True)
    full = g.get_slots(every)
    slots, old, new = dag.change_set(frac)
    assert len(slots) >= capi.Graph.THRU_MARK_DEFAULT
    og = O.OGraph(a)
    og.set_inputs(dag.file_slots, dag.leaf_ids)
    og.full()
    assert (og.slots[:a["n_slots"]] == full).all()
    for version in (new, old, new):
        g.set_slots(slots, version)
        assert g.stats().last_mark_lf == 1  # k3_mark_slots_lf, by the default threshold
        n = g.recompute(full=False)
        assert g.stats().last_levels_lf >= 1  # k2_level_lf on at least the Exec level
        assert 0 < n <= len(a["out_slot"])
        table = g.get_slots(every)
        ids = dag.leaf_ids.copy()
        ids[slots] = version
        assert (table[dag.file_slots] == ids).all()
        bad, first = O.check_slots(a, table, 8)
        assert bad == 0, ("jobs mismatching the oracle", bad, first)
        hashed = og.update(slots, version)
        assert (og.slots[:a["n_slots"]] == table).all()
        assert hashed == n  # the same dirty closure, early cut-off included
    # back to the original IDs: the full recompute's table
    g.set_slots(slots, old)
    g.recompute(full=False)
    assert (g.get_slots(every) == full).all()
    og.close()
    g.close()


def test_default_forms_latency_below_thresholds(ctx):
    """1 % of the same DAG (1,024 slots): the latency forms, same table as the
    oracle's -- the other side of the default choice."""
    dag = Dag1000(1600, 32)
    a = dag.arrays()
    every = np.arange(a["n_slots"], dtype=np.uint32)
    g = load(ctx, dag)
    g.recompute(full=True)
    slots, old, new = dag.change_set(0.01)
    g.set_slots(slots, new)
    assert g.stats().last_mark_lf == 0
    g.recompute(full=False)
    assert g.stats().last_levels_lf == 0
    table = g.get_slots(every)
    bad, first = O.check_slots(a, table, 8)
    assert bad == 0, (bad, first)
    g.close()
