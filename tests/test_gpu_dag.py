"""GPU parity of the incremental digest DAG on the 1000align-shaped workload.

Small S: every slot against the oracle (logical digests and physical keys),
before and after 1% File-ID changes.  Large S: size-independent property --
the incremental recompute equals a full recompute of the same inputs, slot
for slot, and it hashes exactly the dirty closure."""
import numpy as np
import pytest

from reflow_amd.workloads import Dag1000

pytestmark = pytest.mark.gpu

PHYS = {"pR1": "R1", "pE1": "E1", "pE2": "E2", "pE3": "E3", "pES": "ES", "pXS": "XS"}


@pytest.fixture(scope="module")
def ctx():
    from reflow_amd import capi
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


def load(ctx, dag):
    from reflow_amd import capi
    a = dag.arrays()
    g = capi.Graph(ctx, a["n_slots"], a["out_slot"], a["tmpl_off"], a["tmpl_len"], a["hole_ptr"],
                   a["hole_pos"], a["hole_slot"], a["blob"])
    g.set_slots(dag.file_slots, dag.leaf_ids)
    return g


def check_against_oracle(g, dag, ids):
    T = dag.oflow(file_ids=lambda i: ids[i].tobytes())
    for name, nodes in T.items():
        got = g.get_slots(dag.kinds[name].out_slot)
        for i, f in enumerate(nodes):
            assert got[i].tobytes() == f.digest(), (name, i)
    for pname, name in PHYS.items():
        got = g.get_slots(dag.kinds[pname].out_slot)
        for i, f in enumerate(T[name]):
            assert got[i].tobytes() == f.physical_digest(), (pname, i)


@pytest.mark.parametrize("S,P", [(2, 3), (4, 8)])
def test_dag1000_gpu_vs_oracle(ctx, S, P):
    dag = Dag1000(S, P)
    g = load(ctx, dag)
    assert g.recompute(full=True) == dag.n_jobs
    ids = dag.leaf_ids.copy()
    check_against_oracle(g, dag, ids)
    slots, old, new = dag.change_set(0.1)
    for version in (new, old, new):
        g.set_slots(slots, version)
        n = g.recompute(full=False)
        ids[slots] = version
        check_against_oracle(g, dag, ids)
        assert 0 < n < dag.n_jobs


def test_dag1000_incremental_equals_full_large(ctx):
    """~0.9M nodes: incremental after 1% changes == full recompute."""
    dag = Dag1000(2000, 32)
    g = load(ctx, dag)
    g.recompute(full=True)
    slots, old, new = dag.change_set(0.01)
    all_slots = np.arange(dag.n_slots, dtype=np.uint32)
    g.set_slots(slots, new)
    n_inc = g.recompute(full=False)
    inc = g.get_slots(all_slots)
    g.recompute(full=True)
    full = g.get_slots(all_slots)
    assert (inc == full).all()
    # dirty closure per changed leaf file: V, C, E1, C3, K1, C4, E2, C5, K2, C6, E3,
    # C7 + pE1 of its pair; KS, CS1, ES, CS2, XS of its sample (shared when
    # several changed leaves fall in one pair or sample)
    pair_of = slots // 2
    samples = np.unique(pair_of // dag.P)
    pairs = np.unique(pair_of)
    expect = len(slots) * 2 + len(pairs) * (10 + 1) + len(samples) * 5
    assert n_inc == expect
    # back to the old IDs: digests return to the initial state
    g.set_slots(slots, old)
    g.recompute(full=False)
    g2 = load(ctx, dag)
    g2.recompute(full=True)
    assert (g.get_slots(all_slots) == g2.get_slots(all_slots)).all()
