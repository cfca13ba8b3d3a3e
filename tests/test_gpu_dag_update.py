"""rf_graph_update_recompute_async: the changed inputs' mark kernel and the
incremental level sequence as ONE hipGraph launch (the mark node's parameters
rewritten per call).  Against the two-launch form (set_slots_device +
recompute_async) and the oracle over a sequence of change sets: the first call
on a fresh graph (full recompute), an empty batch, batches smaller and larger
than the one the graph was captured with (grid size changes), every input, and
calls interleaved with the two-launch form on the same graph."""
import numpy as np
import pytest

import reflow_oracle as O
from reflow_amd import capi
from reflow_amd.workloads import Dag1000

pytestmark = pytest.mark.gpu


def _changes(dag, rng):
    nf = len(dag.file_slots)
    out = []
    for k in (3, 0, 1, 40, nf, 17, nf // 2):
        pick = np.sort(rng.choice(nf, size=k, replace=False)) if k else np.zeros(0, np.int64)
        out.append((dag.file_slots[pick].astype(np.uint32),
                    rng.integers(0, 256, size=(k, 32), dtype=np.uint8)))
    return out


def _run(ctx, dag, changes, mode):
    """mode: 'one' (update_recompute_async), 'two' (set_slots_device +
    recompute_async) or 'mix' (alternating)."""
    a = dag.arrays()
    g = capi.Graph.from_arrays(ctx, a)
    every = np.arange(a["n_slots"], dtype=np.uint32)
    bufs = []
    out = []
    first = True
    for i, (sl, new) in enumerate([(dag.file_slots.astype(np.uint32), dag.leaf_ids)] + changes):
        d_sl = ctx.upload(sl if len(sl) else np.zeros(1, np.uint32))
        d_new = ctx.upload(new if len(new) else np.zeros((1, 32), np.uint8))
        bufs += [d_sl, d_new]
        use_one = mode == "one" or (mode == "mix" and i % 2 == 0)
        if use_one:
            g.update_recompute_async(d_sl.ptr, d_new.ptr, len(sl), ctx.stream)
        else:
            g.set_slots_device(d_sl.ptr, d_new.ptr, len(sl), ctx.stream)
            g.recompute_async(first, ctx.stream)
        first = False
        ctx.sync()
        out.append(g.get_slots(every))
    g.close()
    for b in bufs:
        b.free()
    return out


def test_update_recompute_matches_two_launch_and_oracle(ctx_env):
    rng = np.random.default_rng(5)
    dag = Dag1000(22, 32)
    changes = _changes(dag, rng)
    one = _run(ctx_env, dag, changes, "one")
    two = _run(ctx_env, dag, changes, "two")
    mix = _run(ctx_env, dag, changes, "mix")
    a = dag.arrays()
    og = O.OGraph(a)
    og.set_inputs(dag.file_slots.astype(np.uint32), dag.leaf_ids)
    og.full()
    want = [og.slots[:a["n_slots"]].copy()]
    for sl, new in changes:
        if len(sl):
            og.update(sl, new)
        want.append(og.slots[:a["n_slots"]].copy())
    og.close()
    for step in range(len(want)):
        assert (one[step] == want[step]).all(), ("one", step)
        assert (two[step] == want[step]).all(), ("two", step)
        assert (mix[step] == want[step]).all(), ("mix", step)


@pytest.fixture(scope="module")
def ctx_env():
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()
