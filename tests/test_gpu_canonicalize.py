"""K5: Canonicalize's flowMap on the GPU.

Flow.Canonicalize (flow.go:814-843) collapses semantically equal flows -- equal
Flow.Digest -- into the first one flowMap.Put registers (:881-907).  The GPU
form inserts every node digest, numbered in canonicalize's post-order, into
an HBM hash table and keeps the smallest index per digest.  Checked against:
  * first-occurrence on random digest arrays (duplicates, probe collisions,
    one hot class), bit-exact;
  * the oracle's node-for-node restatement of canonicalize (Get before
    recursion, Put after, HashV1 Config merge) on random DAGs with cloned
    subtrees, digests computed by K2 on the device;
  * the reference's TestCanonicalize (flow_test.go:46-58) shape.
"""
import copy
import random

import numpy as np
import pytest

import reflow_oracle as O
from flowgen import random_dag
from lowering import Lowerer
from reflow_oracle import OFlow


def _first_occurrence(d: np.ndarray) -> np.ndarray:
    first = {}
    return np.array([first.setdefault(d[i].tobytes(), i) for i in range(len(d))], dtype=np.uint32)


def _postorder(root):
    """canonicalize's visiting order: deps, then the map flow, then the node."""
    seen, out = set(), []

    def rec(f):
        if id(f) in seen:
            return
        seen.add(id(f))
        for d in f.deps:
            rec(d)
        if f.mapflow is not None:
            rec(f.mapflow)
        out.append(f)
    rec(root)
    return out


def _dup_dag(seed, n):
    root, nodes = random_dag(seed, n=n)
    rng = random.Random(seed)
    clones = [copy.deepcopy(rng.choice(nodes)) for _ in range(6)]
    i1, i2 = OFlow("OpIntern", url="url"), OFlow("OpIntern", url="url")
    return OFlow("OpMerge", [root] + clones + [OFlow("OpMerge", [i1, i2])])


def test_oracle_canonicalize_reference_shape():
    """flow_test.go:46-58: Merge(Intern("url"), Intern("url")) -> both deps
    canonicalize to the same flow, the digest is unchanged."""
    i1, i2 = OFlow("OpIntern", url="url"), OFlow("OpIntern", url="url")
    merged = OFlow("OpMerge", [i1, i2])
    canon = O.canonicalize(merged)
    assert canon[id(i1)] is i1 and canon[id(i2)] is i1 and canon[id(merged)] is merged


# --------------------------------------------------------------- GPU side --
@pytest.fixture(scope="module")
def ctx():
    from reflow_amd import capi
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,classes", [(0, 1), (1, 1), (1000, 300), (300000, 50000), (200000, 200000)])
def test_dedup_random(ctx, n, classes):
    rng = np.random.default_rng(n + classes)
    pool = rng.integers(0, 256, size=(classes, 32), dtype=np.uint8)
    d = pool[rng.integers(0, classes, size=n)] if n else np.zeros((0, 32), np.uint8)
    canon, nu = ctx.dedup_digests(d)
    want = _first_occurrence(d)
    assert canon.tolist() == want.tolist()
    assert nu == len(np.unique(want))


@pytest.mark.gpu
def test_dedup_probe_collisions_and_hot_class(ctx):
    rng = np.random.default_rng(7)
    # 4000 distinct digests sharing their first 8 bytes: one probe chain
    d = rng.integers(0, 256, size=(4000, 32), dtype=np.uint8)
    d[:, :8] = 0xAB
    d = np.concatenate([d, d[::-1], d[::3]])  # each class several times
    canon, nu = ctx.dedup_digests(d)
    assert canon.tolist() == _first_occurrence(d).tolist() and nu == 4000
    # one class, 50k members
    h = np.tile(rng.integers(0, 256, size=(1, 32), dtype=np.uint8), (50000, 1))
    canon, nu = ctx.dedup_digests(h)
    assert (canon == 0).all() and nu == 1


@pytest.mark.gpu
@pytest.mark.parametrize("word", [1, 3, 4, 6])
def test_dedup_keys_differing_in_one_word(ctx, word):
    """100k distinct digests equal everywhere but one 4-byte word (bytes 4-7,
    12-15, 16-19, 24-27: the words the round-2 slot hash left out), each
    twice: every class is found (no probe-bound overflow) and canon is the
    first occurrence."""
    rng = np.random.default_rng(word)
    n = 100_000
    d = np.tile(rng.integers(0, 256, size=(1, 32), dtype=np.uint8), (n, 1))
    d[:, 4 * word:4 * word + 4] = np.arange(n, dtype=np.uint32).view(np.uint8).reshape(n, 4)
    d = np.concatenate([d, d[rng.permutation(n)]])
    canon, nu = ctx.dedup_digests(d)
    assert nu == n
    assert canon.tolist() == _first_occurrence(d).tolist()


@pytest.mark.gpu
def test_dedup_device_repeated_calls(ctx):
    """The device form, called back to back on the context's stream and then
    on another stream (the context's scratch is handed between streams in
    stream order): every call gives first-occurrence classes."""
    from reflow_amd import capi
    rng = np.random.default_rng(11)
    n = 2_000_000
    d = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    d[n // 2:n // 2 + 20000] = d[:20000]
    d[-5000:] = d[100:5100]
    want = _first_occurrence(d)
    dd = ctx.upload(d)
    canon, nu = ctx.alloc(4 * n), ctx.alloc(64)
    for k in range(4):
        ctx.dedup_digests_device(dd.ptr, n, canon.ptr, nu.ptr)
        ctx.sync()
        got_nu = int(nu.to_numpy()[:4].view(np.uint32)[0])
        assert got_nu == len(np.unique(want)), (k, hex(got_nu))
        assert (canon.to_numpy().view(np.uint32) == want).all(), k
    c2 = capi.Context(0, host_threads=0)
    ctx.dedup_digests_device(dd.ptr, n, canon.ptr, nu.ptr, stream=c2.stream)
    c2.sync()
    assert (canon.to_numpy().view(np.uint32) == want).all()
    c2.close()
    for x in (dd, canon, nu):
        x.free()


def _gpu_canonical(ctx, top, v1):
    from reflow_amd import capi
    post = _postorder(top)
    low = Lowerer()
    slots = [low.lower(f, v1=v1) for f in post]
    a = low.L.arrays()
    g = capi.Graph(ctx, a["n_slots"], a["out_slot"], a["tmpl_off"], a["tmpl_len"], a["hole_ptr"],
                   a["hole_pos"], a["hole_slot"], a["blob"])
    g.recompute(full=True)
    digs = np.stack([g.get_slots(slots)]).reshape(-1, 32)
    g.close()
    canon, _ = ctx.dedup_digests(digs)
    return post, canon


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_canonicalize_flows_v2(ctx, seed):
    top = _dup_dag(seed, 40)
    post, canon = _gpu_canonical(ctx, top, v1=False)
    want = O.canonicalize(top)
    checked = 0
    for i, f in enumerate(post):
        if id(f) in want:  # nodes the reference's recursion visits
            assert post[canon[i]] is want[id(f)]
            checked += 1
    assert checked > 0
    assert sum(1 for i in range(len(post)) if canon[i] != i) >= 2  # clones collapsed


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12])
def test_canonicalize_flows_hashv1_merge(ctx, seed):
    top = _dup_dag(seed, 14)
    post, canon = _gpu_canonical(ctx, top, v1=True)
    want = O.canonicalize(top, hashv1=True)
    for i, f in enumerate(post):
        if id(f) in want:
            assert post[canon[i]] is want[id(f)]
