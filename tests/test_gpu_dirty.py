"""Eval.dirty (eval.go:874-887) for every node at once (rf_flow_dirty, K3
reachability on the GPU) against the oracle's restatement
(reflow_oracle.eval_dirty): the graph of the reference's TestNoCacheExtern
(test/evaltest/eval_test.go:314-351), random flows over every op, and a
large layered DAG checked against a topological-order recomputation."""
import random

import numpy as np
import pytest

import reflow_oracle as O
from reflow_amd import capi

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


def _csr(nodes):
    idx = {id(f): i for i, f in enumerate(nodes)}
    ptr, deps = [0], []
    for f in nodes:
        deps.extend(idx[id(d)] for d in f.deps)
        ptr.append(len(deps))
    ext = [f.op == O.OP["OpExtern"] for f in nodes]
    return np.array(ptr, np.uint64), np.array(deps, np.uint32), np.array(ext, np.uint8)


def _all_nodes(root):
    seen, out, stack = set(), [], [root]
    while stack:
        f = stack.pop()
        if id(f) in seen:
            continue
        seen.add(id(f))
        out.append(f)
        stack.extend(f.deps)
        if f.mapflow is not None:
            stack.append(f.mapflow)
        if f.parent is not None:
            stack.append(f.parent)
    return out


def test_dirty_no_cache_extern_graph(ctx):
    """TestNoCacheExtern's flow: extern(pullup(map(groupby(intern)))), the map
    function an exec; only the extern is dirty (the map's exec is not a Dep);
    and an exec over an extern is dirty through its Dep."""
    intern = O.OFlow("OpIntern", url="internurl")
    groupby = O.OFlow("OpGroupby", [intern], re="(.*)")
    mf = O.OFlow("OpExec", [O.OFlow("OpVal", value=O.OFileset(map={}))], image="image", cmd="command")
    mp = O.OFlow("OpMap", [groupby], mapflow=mf)
    pullup = O.OFlow("OpPullup", [mp])
    extern = O.OFlow("OpExtern", [pullup], url="externurl")
    consumer = O.OFlow("OpExec", [extern, intern], image="img", cmd="c")
    nodes = _all_nodes(O.OFlow("OpMerge", [consumer, extern]))
    ptr, deps, ext = _csr(nodes)
    for nce in (True, False):
        got = ctx.flow_dirty(ptr, deps, ext, nce)
        memo = {}
        assert list(got) == [O.eval_dirty(f, nce, memo) for f in nodes]
    got = dict(zip(map(id, nodes), ctx.flow_dirty(ptr, deps, ext, True)))
    assert got[id(extern)] and got[id(consumer)] and not got[id(pullup)] and not got[id(intern)]
    assert not got[id(mf)]


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_dirty_random_flows(ctx, seed):
    from flowgen import random_dag
    root, _ = random_dag(seed, n=200)
    nodes = _all_nodes(root)
    ptr, deps, ext = _csr(nodes)
    memo = {}
    want = [O.eval_dirty(f, True, memo) for f in nodes]
    assert list(ctx.flow_dirty(ptr, deps, ext, True)) == want
    assert not ctx.flow_dirty(ptr, deps, ext, False).any()


def test_dirty_large_layered(ctx):
    """600k nodes in 60 layers, 1-4 deps each from earlier layers, 0.05%
    externs: the closure equals a topological-order recomputation."""
    rng = np.random.default_rng(9)
    layers, width = 60, 10_000
    n = layers * width
    deg = rng.integers(1, 5, size=n)
    deg[:width] = 0
    ptr = np.zeros(n + 1, np.uint64)
    ptr[1:] = np.cumsum(deg)
    layer = np.arange(n) // width
    deps = np.empty(int(ptr[-1]), np.uint32)
    for i in range(width, n):
        deps[ptr[i]:ptr[i + 1]] = rng.integers(0, layer[i] * width, size=deg[i])
    ext = (rng.random(n) < 0.0005).astype(np.uint8)
    want = ext.astype(bool).copy()
    for i in range(width, n):  # deps precede i
        if not want[i]:
            want[i] = want[deps[ptr[i]:ptr[i + 1]]].any()
    got = ctx.flow_dirty(ptr, deps, ext, True)
    assert (got == want).all() and 0 < want.sum() < n
