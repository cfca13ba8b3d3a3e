"""GPU parity of the octo level form (k2_level_oct, GraphDev kLvlOct): levels
of few long jobs -- a merge tree above the fill level -- with each job's
whole material staged in LDS and K1's octo chain (8 lanes a job).

Random wide levels put 8-40 holes anywhere in 2-32-block templates (holes
straddling block boundaries, a long constant prefix before the first hole so
the job starts from a load-time midstate, jobs of different lengths in one
workgroup); the strong layout's merge tree (fan-in 32, 18-block jobs) is the
product shape.  Every step is checked against the oracle (a CPU evaluation /
orc_graph_check over the whole slot table) and against the same graph loaded
with the octo form off (RF_K2_OCT=0: k2_level_pl), slot for slot; the form is
read back from rf_graph_stats (last_levels_oct)."""
import random

import numpy as np
import pytest

import reflow_oracle as O
from reflow_amd.workloads import PartitionedDag1000
from test_gpu_dag_fusion import evaluate
from test_gpu_dag_fusion import load as load_jobs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from reflow_amd import capi
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


def wide_jobs(seed, n_in=600):
    """Three wide levels over n_in inputs: A (300 jobs, 8-40 holes on inputs),
    B (21 jobs, 32 holes on A's outputs), C (1 job, 21 holes on B's).  No job
    has a single hole (so none is a fusion target)."""
    rng = random.Random(seed)
    jobs, nxt = [], n_in

    def job(srcs, prefix):
        pos, holes = prefix, []
        for s in srcs:
            holes.append((pos, s))
            pos += 32 + rng.choice([2, 2, 2, 0, 1, 3, 9, 30])
        tlen = min(pos + rng.choice([0, 7, 23, 55, 56, 100]), 32 * 64 - 9)  # <= 32 blocks
        return bytes(rng.getrandbits(8) for _ in range(tlen)), holes

    level_a = []
    for k in range(300):
        nh = rng.randint(8, 40)
        prefix = rng.choice([0, 1, 2, 2, 2, 31, 64, 65, 190, 300])  # >= 64: constant leading blocks
        tmpl, holes = job([rng.randrange(n_in) for _ in range(nh)], prefix)
        if holes[-1][0] + 32 > len(tmpl):
            continue
        jobs.append((nxt, tmpl, holes))
        level_a.append(nxt)
        nxt += 1
    level_b = []
    for k in range(21):
        tmpl, holes = job([rng.choice(level_a) for _ in range(32)], 2)
        jobs.append((nxt, tmpl, holes))
        level_b.append(nxt)
        nxt += 1
    tmpl, holes = job(level_b, 2)
    jobs.append((nxt, tmpl, holes))
    return jobs


def test_oct_random_wide_levels(ctx, monkeypatch):
    rng = np.random.default_rng(11)
    n_in = 600
    jobs = wide_jobs(3, n_in)
    inputs = [rng.integers(0, 256, size=32, dtype=np.uint8).tobytes() for _ in range(n_in)]
    every = np.arange(n_in + len(jobs), dtype=np.uint32)
    g = load_jobs(ctx, n_in, jobs)
    monkeypatch.setenv("RF_K2_OCT", "0")
    gp = load_jobs(ctx, n_in, jobs)  # (read once at load: this graph runs k2_level_pl)
    monkeypatch.delenv("RF_K2_OCT")
    for gg in (g, gp):
        gg.set_slots(np.arange(n_in, dtype=np.uint32), np.frombuffer(b"".join(inputs), np.uint8).reshape(-1, 32))
        gg.recompute(full=True)
    outs = np.array([o for o, _, _ in jobs], np.uint32)
    for step, k in enumerate([1, 7, 60, 600, 3]):
        pick = rng.choice(n_in, size=k, replace=False)
        for i in pick:
            inputs[i] = rng.integers(0, 256, size=32, dtype=np.uint8).tobytes()
        d = np.frombuffer(b"".join(inputs[i] for i in pick), np.uint8).reshape(-1, 32)
        for gg in (g, gp):
            gg.set_slots(pick.astype(np.uint32), d)
            gg.recompute(full=False)
        assert g.stats().last_levels_oct >= 1, step
        assert gp.stats().last_levels_oct == 0
        want = evaluate(n_in, jobs, inputs)
        got = g.get_slots(outs)
        for i, o in enumerate(outs.tolist()):
            assert got[i].tobytes() == want[o], (step, o)
        assert (g.get_slots(every) == gp.get_slots(every)).all(), step
    g.close()
    gp.close()


@pytest.mark.parametrize("nparts", [1, 2])
def test_oct_merge_tree(ctx, monkeypatch, nparts):
    """The strong layout's merge tree (fan-in 32: 18-block, 32-hole merges)
    over 130 samples a part, 1 % and then 30 % of the leaf files changed."""
    pc = PartitionedDag1000(130, 2, 1, 0, nparts=nparts)
    a = pc.desc
    every = np.arange(a["n_slots"], dtype=np.uint32)

    def load():
        from reflow_amd import capi
        gg = capi.Graph.from_arrays(ctx, a)
        gg.set_slots(pc.dag.file_slots, pc.dag.leaf_ids)
        gg.recompute(full=True)
        return gg

    g = load()
    monkeypatch.setenv("RF_K2_OCT", "0")
    gp = load()
    monkeypatch.delenv("RF_K2_OCT")
    ids = pc.dag.leaf_ids.copy()
    for frac, seed in ((0.01, 1), (0.3, 2), (0.3, 2)):
        slots, old, new = pc.dag.change_set(frac, seed=seed)
        version = new if not (ids[slots] == new).all() else old
        for gg in (g, gp):
            gg.set_slots(slots, version)
            gg.recompute(full=False)
        ids[slots] = version
        assert g.stats().last_levels_oct >= 1
        table = g.get_slots(every)
        assert (table[pc.dag.file_slots] == ids).all()
        bad, first = O.check_slots(a, table, 8)
        assert bad == 0, (frac, bad, first)
        assert (table == gp.get_slots(every)).all()
    g.close()
    gp.close()


@pytest.mark.parametrize("sink_at", ["0", "2", "3"])
def test_sink_list_placements(ctx, monkeypatch, sink_at):
    """Where the sink list (physical cache keys whose inputs are final by
    the fill level) runs: 0 the fill level's launch (round 3), 2 the default
    (a latency-form level with CUs to spare, its sinks in low-priority lane
    workgroups), 3 the merge level with the most jobs (its octo launch takes
    the sinks in lane workgroups after its own).  Every placement gives the
    oracle's table and the table of the fill-level placement, slot for slot;
    the level is read back from rf_graph_stats.last_sink_attach."""
    from reflow_amd import capi
    pc = PartitionedDag1000(130, 2, 1, 0, nparts=2)
    a = pc.desc
    every = np.arange(a["n_slots"], dtype=np.uint32)

    def load(mode):
        monkeypatch.setenv("RF_K2_SINK_AT", mode)
        gg = capi.Graph.from_arrays(ctx, a)
        monkeypatch.delenv("RF_K2_SINK_AT")
        gg.set_slots(pc.dag.file_slots, pc.dag.leaf_ids)
        gg.recompute(full=True)
        return gg

    g, g0 = load(sink_at), load("0")
    ids = pc.dag.leaf_ids.copy()
    attach = set()
    for frac, seed in ((0.01, 1), (0.3, 2), (0.05, 3)):
        slots, old, new = pc.dag.change_set(frac, seed=seed)
        version = np.where((ids[slots] == new).all(axis=1)[:, None], old, new).astype(ids.dtype)
        for gg in (g, g0):
            gg.set_slots(slots, version)
            gg.recompute(full=False)
        ids[slots] = version
        attach.add(g.stats().last_sink_attach)
        table = g.get_slots(every)
        assert (table[pc.dag.file_slots] == ids).all()
        assert (table == g0.get_slots(every)).all(), frac
        bad, first = O.check_slots(a, table, 8)
        assert bad == 0, (frac, bad, first)
    assert 0xFFFFFFFF not in attach  # a sink list ran attached every step
    if sink_at == "3":
        assert g.stats().last_levels_oct >= 1
        assert attach != {g0.stats().last_sink_attach}  # above the fill level
    g.close()
    g0.close()
