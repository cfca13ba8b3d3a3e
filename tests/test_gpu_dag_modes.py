"""The forced K2 level variants stay correct: every queueable level run as a
three-wave "wide" workgroup (RF_K2_WIDE=1: k2_level_pl<3>), and every
incremental step in the lane-per-job throughput form (RF_K2_THRU=0:
k2_level_lf).  Both are read once, when a graph is loaded, so one process
covers them.  (The streamed hand-over, measured slower, is a diagnostic-build
form since round 5.)  Checked against the
oracle on the random fused-chain graphs and the 1000align DAG, and on a
larger 1000align DAG against the default mode's incremental recompute."""
import numpy as np
import pytest

from reflow_amd.workloads import Dag1000
from test_gpu_dag import check_against_oracle
from test_gpu_dag import load as load_dag
from test_gpu_dag_fusion import evaluate, random_jobs
from test_gpu_dag_fusion import load as load_jobs

pytestmark = pytest.mark.gpu

# RF_K2_THRU=0: every incremental step in the lane-per-job throughput form
# (k2_level_lf), which the library picks by itself for levels that can
# receive >= 24k chains (tests/test_gpu_dag_default_forms.py)
MODES = [("RF_K2_WIDE", "1"), ("RF_K2_THRU", "0")]


@pytest.fixture(scope="module")
def ctx():
    from reflow_amd import capi
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


@pytest.mark.parametrize("var,val", MODES)
def test_forced_mode_random_jobs(ctx, monkeypatch, var, val):
    monkeypatch.setenv(var, val)
    rng = np.random.default_rng(5)
    n_in = 64
    jobs = random_jobs(31, n_in=n_in)
    inputs = [rng.integers(0, 256, size=32, dtype=np.uint8).tobytes() for _ in range(n_in)]
    g = load_jobs(ctx, n_in, jobs)
    g.set_slots(np.arange(n_in, dtype=np.uint32), np.frombuffer(b"".join(inputs), np.uint8).reshape(-1, 32))
    g.recompute(full=True)
    for step in range(3):
        k = [1, 5, 20][step]
        pick = rng.choice(n_in, size=k, replace=False)
        for i in pick:
            inputs[i] = rng.integers(0, 256, size=32, dtype=np.uint8).tobytes()
        g.set_slots(pick.astype(np.uint32), np.frombuffer(b"".join(inputs[i] for i in pick), np.uint8).reshape(-1, 32))
        g.recompute(full=False)
        want = evaluate(n_in, jobs, inputs)
        outs = np.array([o for o, _, _ in jobs], np.uint32)
        got = g.get_slots(outs)
        for i, o in enumerate(outs.tolist()):
            assert got[i].tobytes() == want[o], (var, step, o)
    g.close()


@pytest.mark.parametrize("var,val", MODES)
def test_forced_mode_dag1000(ctx, monkeypatch, var, val):
    monkeypatch.setenv(var, val)
    dag = Dag1000(4, 8)
    g = load_dag(ctx, dag)
    g.recompute(full=True)
    ids = dag.leaf_ids.copy()
    slots, old, new = dag.change_set(0.1)
    for version in (new, old):
        g.set_slots(slots, version)
        g.recompute(full=False)
        ids[slots] = version
        check_against_oracle(g, dag, ids)
    g.close()
    # 0.45M nodes: the forced mode's incremental slots == the default mode's
    big = Dag1000(1000, 32)
    sl, _, nw = big.change_set(0.01)
    every = np.arange(big.n_slots, dtype=np.uint32)

    def run(gg):
        gg.recompute(full=True)
        gg.set_slots(sl, nw)
        gg.recompute(full=False)

    gf = load_dag(ctx, big)
    run(gf)  # loaded with the mode set
    monkeypatch.delenv(var)
    gd = load_dag(ctx, big)
    run(gd)
    assert (gf.get_slots(every) == gd.get_slots(every)).all()
    gf.close()
    gd.close()


def test_sink_list_attached_below_fill_level(ctx, monkeypatch):
    """The sink level's list (physical keys) rides on the last throughput-form
    launch at or below the fill level: short-job levels forced into the
    throughput form (RF_K2_THRU=1) and the wide OpK level kept in the latency
    form (RF_K2_THRU_WIDE huge) attach it to the Exec level's launch, below the
    fill level -- the strong layout's 4-rank piece.  Checked against the oracle
    and against the default forms' slots."""
    dag = Dag1000(8, 32)  # OpK: 32 holes, 18 blocks (a wide level)
    every = np.arange(dag.n_slots, dtype=np.uint32)
    gd = load_dag(ctx, dag)
    gd.recompute(full=True)
    monkeypatch.setenv("RF_K2_THRU", "1")
    monkeypatch.setenv("RF_K2_THRU_WIDE", str(1 << 62))
    g = load_dag(ctx, dag)
    g.recompute(full=True)
    ids = dag.leaf_ids.copy()
    slots, old, new = dag.change_set(0.1)
    for version in (new, old, new):
        g.set_slots(slots, version)
        g.recompute(full=False)
        ids[slots] = version
        check_against_oracle(g, dag, ids)
    monkeypatch.delenv("RF_K2_THRU")
    monkeypatch.delenv("RF_K2_THRU_WIDE")
    gd.set_slots(slots, new)
    gd.recompute(full=False)
    assert (g.get_slots(every) == gd.get_slots(every)).all()
    g.close()
    gd.close()


def _leading(jobs, kind, seed):
    """random_jobs with every job's first hole in block 0 ("none": no constant
    leading blocks, so every level's listed jobs start from the IV --
    GraphDev::lvl_lead0) or past it ("all": each job with a midstate)."""
    rng = np.random.default_rng(seed)
    out = []
    for o, tmpl, holes in jobs:
        first = holes[0][0]
        if kind == "none" and first >= 64:
            tmpl, holes = tmpl[64:], [(p - 64, s) for p, s in holes]
        elif kind == "all" and first < 64:
            pad = rng.integers(0, 256, size=64 + 64 * int(rng.integers(0, 2)), dtype=np.uint8).tobytes()
            tmpl, holes = pad + tmpl, [(p + len(pad), s) for p, s in holes]
        out.append((o, tmpl, holes))
    return out


@pytest.mark.parametrize("kind", ["none", "all"])
def test_thru_form_leading_blocks(ctx, monkeypatch, tmp_path, kind):
    """The throughput form's per-level IV start (LevelArgs::lead0) against the
    oracle: graphs whose jobs have no constant leading blocks at all, or all
    have them -- and after a checkpoint restore, which leaves the per-level
    flags empty (every listed job then loads its midstate)."""
    from reflow_amd import capi
    monkeypatch.setenv("RF_K2_THRU", "0")
    rng = np.random.default_rng(11)
    n_in = 64
    jobs = _leading(random_jobs(41, n_in=n_in), kind, 3)
    assert all((h[0][0] < 64) == (kind == "none") for _, _, h in jobs)
    inputs = [rng.integers(0, 256, size=32, dtype=np.uint8).tobytes() for _ in range(n_in)]
    g = load_jobs(ctx, n_in, jobs)
    g.set_slots(np.arange(n_in, dtype=np.uint32), np.frombuffer(b"".join(inputs), np.uint8).reshape(-1, 32))
    g.recompute(full=True)
    outs = np.array([o for o, _, _ in jobs], np.uint32)
    for step in range(4):
        if step == 2:
            path = str(tmp_path / "g.ckpt")
            g.save(path)
            g.close()
            g = capi.Graph.restore(ctx, path)
        pick = rng.choice(n_in, size=[1, 6, 6, 24][step], replace=False)
        for i in pick:
            inputs[i] = rng.integers(0, 256, size=32, dtype=np.uint8).tobytes()
        g.set_slots(pick.astype(np.uint32), np.frombuffer(b"".join(inputs[i] for i in pick), np.uint8).reshape(-1, 32))
        g.recompute(full=False)
        want = evaluate(n_in, jobs, inputs)
        got = g.get_slots(outs)
        for i, o in enumerate(outs.tolist()):
            assert got[i].tobytes() == want[o], (kind, step, o)
    g.close()
