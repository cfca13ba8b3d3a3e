"""Constant leading blocks hashed once at load (rf_graph_load -> per-job
midstates, k2_midstates): jobs whose first hole starts past block 0 -- at byte
64, deep in a long template, in the last block, one hole per block after a
prefix, and a fused chain of such jobs -- give the oracle's digests in full and
incremental recomputes, and the same digests as a load with midstates off
(RF_K2_NO_MIDSTATE).  configs[2]'s pE1 physical keys (4 of 8 blocks constant)
are covered in full size by test_gpu_scale.py."""
import numpy as np
import pytest

import reflow_oracle as O
from reflow_amd import capi
from reflow_amd.workloads import append_jobs

pytestmark = pytest.mark.gpu

WD0 = b"\x00\x05" + bytes(32)


def _graph(rng, n_in=40, n_jobs=400):
    a = dict(n_slots=n_in, out_slot=np.zeros(0, np.uint32), tmpl_off=np.zeros(0, np.uint64),
             tmpl_len=np.zeros(0, np.uint32), hole_ptr=np.zeros(1, np.uint64), hole_pos=np.zeros(0, np.uint32),
             hole_slot=np.zeros(0, np.uint32), blob=np.zeros(0, np.uint8))
    jobs = []
    slots = list(range(n_in))
    for j in range(n_jobs):
        kind = j % 5
        if kind == 0:   # first hole exactly at byte 64
            pre, nh = 62, 1
        elif kind == 1:  # long constant prefix, several holes
            pre, nh = int(rng.integers(130, 600)), int(rng.integers(1, 4))
        elif kind == 2:  # hole in the last block
            pre, nh = int(rng.integers(200, 300)), 1
        elif kind == 3:  # no constant prefix
            pre, nh = 0, int(rng.integers(1, 3))
        else:            # a single hole after a prefix: a fusion target of the previous job
            pre, nh = int(rng.integers(70, 200)), 1
        prefix = bytes(rng.integers(0, 256, size=pre, dtype=np.uint8))
        tmpl = prefix + WD0 * nh + bytes(rng.integers(0, 256, size=int(rng.integers(0, 40)), dtype=np.uint8))
        deps = [slots[-1]] if kind == 4 and j else [int(rng.integers(0, len(slots))) for _ in range(nh)]
        deps = deps[:nh] + [int(rng.integers(0, len(slots))) for _ in range(nh - len(deps))]
        holes = [(pre + 34 * h + 2, deps[h]) for h in range(nh)]
        jobs.append((tmpl, holes))
        slots.append(n_in + j)
    a, _ = append_jobs(a, jobs)
    return a


def _run(ctx, a, ids, changes):
    g = capi.Graph.from_arrays(ctx, a)
    n_in = int(a["out_slot"][0])
    inputs = np.arange(n_in, dtype=np.uint32)
    g.set_slots(inputs, ids)
    g.recompute(full=True)
    every = np.arange(a["n_slots"], dtype=np.uint32)
    out = [g.get_slots(every)]
    for sl, new in changes:
        g.set_slots(sl, new)
        g.recompute(full=False)
        out.append(g.get_slots(every))
    g.close()
    return out


def test_midstate_jobs_match_oracle(ctx_env, monkeypatch):
    rng = np.random.default_rng(17)
    a = _graph(rng)
    n_in = int(a["out_slot"][0])
    ids = rng.integers(0, 256, size=(n_in, 32), dtype=np.uint8)
    changes = []
    for k in (1, 7, n_in):
        sl = np.sort(rng.choice(n_in, size=k, replace=False)).astype(np.uint32)
        changes.append((sl, rng.integers(0, 256, size=(k, 32), dtype=np.uint8)))
    got = _run(ctx_env, a, ids, changes)
    og = O.OGraph(a)
    og.set_inputs(np.arange(n_in, dtype=np.uint32), ids)
    og.full()
    want = [og.slots[:a["n_slots"]].copy()]
    for sl, new in changes:
        og.update(sl, new)
        want.append(og.slots[:a["n_slots"]].copy())
    og.close()
    for step, (gg, ww) in enumerate(zip(got, want)):
        assert (gg == ww).all(), step
    # the same graph loaded without midstates: identical digests
    monkeypatch.setenv("RF_K2_NO_MIDSTATE", "1")
    plain = _run(ctx_env, a, ids, changes)
    for gg, pp in zip(got, plain):
        assert (gg == pp).all()
    st = capi.Graph.from_arrays(ctx_env, a)
    monkeypatch.delenv("RF_K2_NO_MIDSTATE")
    st2 = capi.Graph.from_arrays(ctx_env, a)
    assert st2.stats().total_blocks < st.stats().total_blocks  # constant blocks no longer hashed
    st.close()
    st2.close()


@pytest.fixture(scope="module")
def ctx_env():
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()
