"""GPU parity of the latency form's width variants on a level a little wider
than the chip: half workgroups (32 jobs) on a pretended small chip
(RF_K2_OVF_CU: the CU count the form choice sizes for, read at load), checked
against the 64-job form slot for slot and against orc_graph_check over the
whole table (flow.go:675-792 per job).  (The overflow lanes, measured slower,
are a diagnostic-build form since round 5.)"""
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
