"""GPU parity of split block 0 (k2_level_pl cb0 = 2, GraphDev::split_b0): in
a fused link's chain pass the producer expands the upper half of the fusion
target's block-0 schedule (from the W words the chain stages) while the chain
runs the lower half, and the target's template-only block 1 was built by the
producer during the job before it, into the row buffer that job's last block
left free (the buffers' parity flips per pass).  Targets of 2 and 3 blocks
(Dag1000's pair chain) both occur.  The reference hashes the same bytes
(flow.go:675-750 per node); only the order of work on the GPU changes, so
the slot table must equal the oracle's and the table of the same graph
loaded with the split off (RF_K2_SPLIT=0), slot for slot, step after step --
and a checkpoint restore keeps the split (rf_graph_stats.split_block0) and
the same table."""
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


@pytest.mark.parametrize("mode", [1, 2])
def test_split_block0_matches_unsplit_and_oracle(ctx, monkeypatch, tmp_path, mode):
    """mode 1: the producer expands K+W[32..63] of block 0; 2 (default):
    K+W[16..63], the chain writes K+W[0..15] only."""
    from reflow_amd import capi
    dag = Dag1000(400, 32)
    a = dag.arrays()
    every = np.arange(a["n_slots"], dtype=np.uint32)
    monkeypatch.setenv("RF_K2_SPLIT", str(mode))
    g = load(ctx, dag)
    monkeypatch.setenv("RF_K2_SPLIT", "0")
    gp = load(ctx, dag)
    monkeypatch.setenv("RF_K2_SPLIT", str(mode))  # (the restore below reads it too)
    assert g.stats().split_block0 == mode  # Dag1000: every fusion target's hole at byte 2
    assert gp.stats().split_block0 == 0
    for gg in (g, gp):
        gg.recompute(full=True)
    full = g.get_slots(every)
    assert (full == gp.get_slots(every)).all()
    ids = dag.leaf_ids.copy()
    for frac, seed in ((0.001, 1), (0.01, 2), (0.05, 3), (0.01, 2)):
        slots, old, new = dag.change_set(frac, seed=seed)
        version = new if not (ids[slots] == new).all() else old
        for gg in (g, gp):
            gg.set_slots(slots, version)
            gg.recompute(full=False)
        ids[slots] = version
        table = g.get_slots(every)
        assert (table[dag.file_slots] == ids).all()
        assert (table == gp.get_slots(every)).all(), frac
        bad, first = O.check_slots(a, table, 8)
        assert bad == 0, (frac, bad, first)
    # a restored graph rebuilds the rows and steps to the same table
    path = str(tmp_path / "split.ckpt")
    g.save(path)
    r = capi.Graph.restore(ctx, path)
    assert r.stats().split_block0 == mode
    slots, old, new = dag.change_set(0.01, seed=7)
    version = np.where((ids[slots] == new).all(axis=1)[:, None], old, new).astype(ids.dtype)
    for gg in (g, r):
        gg.set_slots(slots, version)
        gg.recompute(full=False)
    table = r.get_slots(every)
    assert (table == g.get_slots(every)).all()
    bad, first = O.check_slots(a, table, 8)
    assert bad == 0, (bad, first)
    for gg in (g, gp, r):
        gg.close()
