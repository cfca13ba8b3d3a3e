"""The flow step (k2_flow): one readiness-driven launch over a step's levels
instead of one kernel per level, a job starting as soon as the jobs it reads
have finished (GraphDev "flow", rf_graph_set_flow; the reference evaluator's
ready loop, /root/reference/eval.go:376-411, todo :902-955).

Checked against the oracle (random fused-chain graphs through the CPU
evaluation of tests/test_gpu_dag_fusion.py, the 1000align DAG through
Dag1000.oflow, a merge-tree layout through orc_graph_check over the whole
table) and against level-by-level steps of the same graph, slot for slot;
early cut-off (a slot set and set back in one step: its consumers are queued
and hash to their old digests, so nothing further runs) keeps the count the
level-by-level step reports; a checkpoint restores the flow structures."""
import os
import random
import sys

import numpy as np
import pytest

from reflow_amd.workloads import Dag1000, PartitionedDag1000
from test_gpu_dag import check_against_oracle
from test_gpu_dag import load as load_dag
from test_gpu_dag_fusion import evaluate, random_jobs
from test_gpu_dag_fusion import load as load_jobs

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import reflow_oracle as O  # noqa: E402  (the checker)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from reflow_amd import capi
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


def _set(g, slots, vals):
    g.set_slots(np.asarray(slots, np.uint32), np.frombuffer(b"".join(vals), np.uint8).reshape(-1, 32))


@pytest.mark.parametrize("seed", [31, 32, 33])
def test_flow_random_jobs_vs_cpu(ctx, seed):
    """Every launchable level in the flow launch (mode 2) on random graphs of
    fused chains, wide jobs and parked jobs (a job's producers at several
    levels), against the CPU evaluation; the same steps level by level on a
    second load report the same hashed-job counts."""
    n_in = 64
    jobs = random_jobs(seed, n_in=n_in, n_jobs=2500)
    rng = random.Random(seed)
    inputs = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(n_in)]
    gf, gl = load_jobs(ctx, n_in, jobs), load_jobs(ctx, n_in, jobs)
    gl.set_flow(0)
    for g in (gf, gl):
        _set(g, range(n_in), inputs)
        g.recompute(full=True)
    gf.set_flow(2)
    outs = np.array([o for o, _, _ in jobs], np.uint32)
    flowed = 0
    for step, k in enumerate([1, 3, 8, 20, 64, 2, 64]):
        pick = rng.sample(range(n_in), k)
        new = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in pick]
        for i, v in zip(pick, new):
            inputs[i] = v
        counts = []
        for g in (gf, gl):
            _set(g, pick, new)
            counts.append(g.recompute(full=False))
        flowed += gf.stats().last_flow
        assert gl.stats().last_flow == 0
        assert counts[0] == counts[1], (seed, step, counts)
        want = evaluate(n_in, jobs, inputs)
        got = gf.get_slots(outs)
        for i, o in enumerate(outs.tolist()):
            assert got[i].tobytes() == want[o], (seed, step, o)
    assert flowed >= 6  # (a step whose change reaches one launchable level runs level by level)
    # early cut-off: slots set to new values and back within one step -- their
    # consumers are queued, hash to their old digests, and stop there
    pick = rng.sample(range(n_in), 16)
    tmp = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in pick]
    before = gf.get_slots(outs)
    counts = []
    for g in (gf, gl):
        _set(g, pick, tmp)
        _set(g, pick, [inputs[i] for i in pick])
        counts.append(g.recompute(full=False))
    assert counts[0] == counts[1]
    assert (gf.get_slots(outs) == before).all()
    gf.close()
    gl.close()


def test_flow_dag1000_vs_oracle(ctx):
    dag = Dag1000(4, 8)
    g = load_dag(ctx, dag)
    g.recompute(full=True)
    g.set_flow(2)
    ids = dag.leaf_ids.copy()
    slots, old, new = dag.change_set(0.1)
    for version in (new, old, new):
        g.set_slots(slots, version)
        assert 0 < g.recompute(full=False) < dag.n_jobs
        assert g.stats().last_flow == 1
        ids[slots] = version
        check_against_oracle(g, dag, ids)
    g.close()


def _steps(g, slots, versions):
    out = []
    for v in versions:
        g.set_slots(slots, v)
        out.append(g.recompute(full=False))
    return out


@pytest.mark.parametrize("frac", [0.01, 0.3])
def test_flow_auto_equals_levels(ctx, frac):
    """The automatic choice (mode 1) on a 0.45M-node 1000align DAG whose levels
    all run in the throughput form (set_forms(0)): the Exec, OpK and sink
    levels in one flow launch; slot for slot and count for count against the
    same graph stepped level by level."""
    dag = Dag1000(1000, 32)
    sl, old, new = dag.change_set(frac)
    every = np.arange(dag.n_slots, dtype=np.uint32)
    gf, gl = load_dag(ctx, dag), load_dag(ctx, dag)
    gf.set_flow(1)
    gl.set_flow(0)
    for g in (gf, gl):
        g.recompute(full=True)
        g.set_forms(0)
    cf = _steps(gf, sl, [new, old, new])
    assert gf.stats().last_flow == 1
    cl = _steps(gl, sl, [new, old, new])
    assert cf == cl
    assert (gf.get_slots(every) == gl.get_slots(every)).all()
    gf.close()
    gl.close()


def test_flow_merge_tree_vs_oracle(ctx):
    """A strong-layout piece (PartitionedDag1000: per part a fan-in-32 Merge
    tree above the fill level): the flow launch over the Exec / OpK / sink
    levels, the merge levels after it level by level -- every job of the
    table re-derived by the oracle from its hole digests (orc_graph_check),
    the inputs at their assigned values."""
    pc = PartitionedDag1000(300, 8, 1, 0, nparts=2)
    from reflow_amd import capi
    g = capi.Graph.from_arrays(ctx, pc.desc)
    g.set_slots(pc.dag.file_slots, pc.dag.leaf_ids)
    g.recompute(True)
    g.set_forms(0)
    g.set_flow(1)
    every = np.arange(pc.desc["n_slots"], dtype=np.uint32)
    ids = pc.dag.leaf_ids.copy()
    slots, old, new = pc.dag.change_set(0.05)
    for version in (new, old):
        g.set_slots(slots, version)
        g.recompute(False)
        assert g.stats().last_flow == 1
        ids[slots] = version
        table = g.get_slots(every)
        assert (table[pc.dag.file_slots] == ids).all()
        bad, first = O.check_slots(pc.desc, table, 4)
        assert bad == 0, first
    g.close()


def test_flow_after_checkpoint(ctx, tmp_path):
    """A restored graph carries the flow structures (checkpoint version 2):
    its flow steps equal the original's."""
    n_in = 64
    jobs = random_jobs(41, n_in=n_in, n_jobs=1500)
    rng = random.Random(41)
    inputs = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(n_in)]
    g = load_jobs(ctx, n_in, jobs)
    _set(g, range(n_in), inputs)
    g.recompute(full=True)
    path = str(tmp_path / "flow.ckpt")
    g.save(path)
    from reflow_amd import capi
    r = capi.Graph.restore(ctx, path)
    outs = np.array([o for o, _, _ in jobs], np.uint32)
    for gg in (g, r):
        gg.set_flow(2)
    for k in (4, 30):
        pick = rng.sample(range(n_in), k)
        new = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in pick]
        for i, v in zip(pick, new):
            inputs[i] = v
        for gg in (g, r):
            _set(gg, pick, new)
            gg.recompute(full=False)
            assert gg.stats().last_flow == 1
        assert (g.get_slots(outs) == r.get_slots(outs)).all()
    want = evaluate(n_in, jobs, inputs)
    got = r.get_slots(outs)
    assert all(got[i].tobytes() == want[o] for i, o in enumerate(outs.tolist()))
    g.close()
    r.close()
