"""GPU parity of the latency form's overflow lanes (k2_level_pl ovf): when a
latency-form level can receive more chains than one 64-job workgroup per CU
holds (estimated from the step's marked slots), one workgroup per CU takes
64 chains and the rest run one chain per lane (lf_job, the fused chain
followed in the lane) in workgroups after them, before any attached sinks.
A small DAG exercises it on a pretended 4-CU chip (RF_K2_OVF_CU=4, read at
load): the Exec level's ~hundreds of chains overflow 4 x 64.  Every step is
checked against the same graph loaded with the overflow lanes off
(RF_K2_OVF=0) slot for slot, against orc_graph_check over the whole table
(flow.go:675-792 per job), and the lanes at the chains' priority
(RF_K2_OVF=2) give the same table."""
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


@pytest.mark.parametrize("ovf", ["1", "2"])
def test_overflow_lanes_match_oracle(ctx, monkeypatch, ovf):
    dag = Dag1000(400, 32)
    a = dag.arrays()
    every = np.arange(a["n_slots"], dtype=np.uint32)
    monkeypatch.setenv("RF_K2_OVF_CU", "4")
    monkeypatch.setenv("RF_K2_OVF", ovf)
    g = load(ctx, dag)          # overflow lanes above 256 chains
    monkeypatch.setenv("RF_K2_OVF", "0")
    gp = load(ctx, dag)         # latency form only (a second workgroup round)
    monkeypatch.delenv("RF_K2_OVF")
    monkeypatch.delenv("RF_K2_OVF_CU")
    for gg in (g, gp):
        gg.recompute(full=True)
    ids = dag.leaf_ids.copy()
    for frac, seed in ((0.02, 1), (0.05, 2), (0.2, 3), (0.02, 1)):
        slots, old, new = dag.change_set(frac, seed=seed)
        version = np.where((ids[slots] == new).all(axis=1)[:, None], old, new).astype(ids.dtype)
        for gg in (g, gp):
            gg.set_slots(slots, version)
            gg.recompute(full=False)
        ids[slots] = version
        table = g.get_slots(every)
        assert (table[dag.file_slots] == ids).all()
        assert (table == gp.get_slots(every)).all(), frac
        bad, first = O.check_slots(a, table, 8)
        assert bad == 0, (frac, bad, first)
    g.close()
    gp.close()


@pytest.mark.parametrize("split_half", ["0", "1"])
def test_half_workgroups_match_oracle(ctx, monkeypatch, split_half):
    """Half workgroups (k2_level_pl<2, false, 32>: one chain wave and the
    producer, 32 jobs) run a latency-form level estimated at more than 64
    chains per CU and at most 96: on a pretended 6-CU chip, 512 marked slots
    (2 % of the leaf files) put the Exec level there.  Its pass structure,
    split block 0 and sink lanes are those of the 64-job form; the table must
    equal the 64-job form's (the device's CUs: one 64-job round) and the
    oracle's, step after step; with and without block 0 split in them
    (RF_K2_SPLIT_HALF, read at load)."""
    dag = Dag1000(400, 32)
    a = dag.arrays()
    every = np.arange(a["n_slots"], dtype=np.uint32)
    monkeypatch.setenv("RF_K2_OVF_CU", "6")
    monkeypatch.setenv("RF_K2_SPLIT_HALF", split_half)
    g = load(ctx, dag)
    monkeypatch.delenv("RF_K2_OVF_CU")
    monkeypatch.delenv("RF_K2_SPLIT_HALF")
    gp = load(ctx, dag)
    for gg in (g, gp):
        gg.recompute(full=True)
    ids = dag.leaf_ids.copy()
    for frac, seed in ((0.02, 1), (0.02, 5), (0.018, 6), (0.02, 1)):
        slots, old, new = dag.change_set(frac, seed=seed)
        assert 6 * 64 < len(slots) <= 6 * 96  # (the half-workgroup range for the Exec level)
        version = np.where((ids[slots] == new).all(axis=1)[:, None], old, new).astype(ids.dtype)
        for gg in (g, gp):
            gg.set_slots(slots, version)
            gg.recompute(full=False)
        ids[slots] = version
        table = g.get_slots(every)
        assert (table[dag.file_slots] == ids).all()
        assert (table == gp.get_slots(every)).all(), (frac, seed)
        bad, first = O.check_slots(a, table, 8)
        assert bad == 0, (frac, seed, bad, first)
    g.close()
    gp.close()
