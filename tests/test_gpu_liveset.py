"""Liveset build side + Repository.Collect on the GPU:
the bloom wire formats written by the engine, and the batched Collect that
removes every object the liveset does not contain.  Checked bit-exactly
against the oracle (oracle/oracle.c bloom Test/Add restated from
vendor/github.com/willf/bloom/bloom.go:94-190)."""
import base64
import struct

import numpy as np
import pytest

import reflow_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from reflow_amd import capi
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


def _oracle_filter(keys32: bytes, n, p=0.01):
    m, k = O.estimate_parameters(n, p)
    words = np.zeros((m + 63) // 64, dtype=np.uint64)
    length = np.array([m], dtype=np.uint64)
    O.lib().orc_bloomlive_add_batch(words.ctypes.data, length.ctypes.data, m, k, keys32, n)
    return m, k, words, int(length[0])


def _oracle_probe(words, length, m, k, keys32, n):
    out = np.zeros(max(n, 1), dtype=np.uint8)
    if n:
        O.lib().orc_bloomlive_contains_batch(words.ctypes.data, length, m, k, keys32, n, out.ctypes.data, 4)
    return out[:n]


@pytest.mark.parametrize("n_live,n_obj", [(0, 0), (1, 1), (700, 2000), (5000, 4096 * 3 + 17),
                                          (20000, 150000)])
def test_collect_parity(ctx, n_live, n_obj):
    """Repository.Collect (repository/file/repository.go:304-327): the objects
    whose digest the liveset lacks, in walk (index) order, and their bytes."""
    from reflow_amd import capi
    rng = np.random.default_rng(n_obj + 11)
    objs = rng.integers(0, 256, size=32 * n_obj, dtype=np.uint8).tobytes()
    sizes = rng.integers(-(1 << 40), 1 << 40, size=n_obj, dtype=np.int64)
    # the liveset holds a random subset of the objects plus unrelated keys
    live_idx = rng.permutation(n_obj)[:min(n_live, n_obj)]
    live = b"".join(objs[32 * i:32 * i + 32] for i in live_idx)
    live += rng.integers(0, 256, size=32 * 50, dtype=np.uint8).tobytes()
    nl = len(live) // 32
    m, k, words, length = _oracle_filter(live, nl, 0.01)
    b = capi.Bloom.load(ctx, m, k, words, length)
    dead, nbytes = b.collect(np.frombuffer(objs, np.uint8), sizes)
    want = np.flatnonzero(_oracle_probe(words, length, m, k, objs, n_obj) == 0)
    assert dead.tolist() == want.tolist()
    assert nbytes == int(sizes[want].sum())
    assert not set(live_idx.tolist()) & set(dead.tolist())  # no live object collected
    dead2, nb2 = b.collect(np.frombuffer(objs, np.uint8))  # sizes optional
    assert dead2.tolist() == dead.tolist() and nb2 == 0
    b.close()


def test_collect_all_live_and_all_dead(ctx):
    from reflow_amd import capi
    rng = np.random.default_rng(5)
    n = 10000
    objs = rng.integers(0, 256, size=32 * n, dtype=np.uint8)
    b = capi.Bloom.new(ctx, 1 << 20, 7)
    dead, nb = b.collect(objs, np.ones(n, dtype=np.int64))
    assert dead.tolist() == list(range(n)) and nb == n  # empty liveset: everything goes
    b.add(objs)
    dead, nb = b.collect(objs, np.ones(n, dtype=np.int64))
    assert len(dead) == 0 and nb == 0
    b.close()


def test_marshal_roundtrip(ctx):
    """Wire formats out (bloom.go:270-301, bitset.go:628-702): Go's byte
    layout, and what the engine writes reloads to the same filter."""
    from reflow_amd import capi
    rng = np.random.default_rng(12)
    n = 900
    keys = rng.integers(0, 256, size=32 * n, dtype=np.uint8)
    m, k = O.estimate_parameters(n, 0.01)
    b = capi.Bloom.new(ctx, m, k)
    b.add(keys)
    _, _, words, length = _oracle_filter(keys.tobytes(), n, 0.01)
    bits = struct.pack(">Q", length) + b"".join(struct.pack(">Q", int(w)) for w in words)
    assert b.marshal_binary() == struct.pack(">QQ", m, k) + bits
    assert b.marshal_json() == b'{"m":%d,"k":%d,"b":"%s"}' % (m, k, base64.urlsafe_b64encode(bits))
    for b2 in (capi.Bloom.from_json(ctx, b.marshal_json()), capi.Bloom.from_binary(ctx, b.marshal_binary())):
        assert b2.marshal_binary() == b.marshal_binary()
        b2.close()
    for nw in (1, 2, 3):  # 8 + 8*nw bitset bytes: every base64 padding case
        e = capi.Bloom.load(ctx, 64 * nw, 1, np.arange(nw, dtype=np.uint64), 64 * nw)
        raw = struct.pack(">Q", 64 * nw) + b"".join(struct.pack(">Q", i) for i in range(nw))
        assert e.marshal_json() == b'{"m":%d,"k":1,"b":"%s"}' % (64 * nw, base64.urlsafe_b64encode(raw))
        e.close()
    b.close()


def test_marshal_golden_fixture(ctx):
    """The committed bloom fixture's wire bytes are reproduced by the engine's
    writers after loading them (tests/golden/bloom.json)."""
    import hashlib
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import golden_io as G
    from reflow_amd import capi
    for c in G.load("bloom.json")["cases"]:
        if c["json"] is None:
            continue
        b = capi.Bloom.from_json(ctx, c["json"].encode())
        assert b.marshal_json().decode() == c["json"]
        assert hashlib.sha256(b.marshal_binary()).hexdigest() == c["binary_sha256"]
        b.close()


def test_load_ignores_words_past_length(ctx):
    """A bitset holds exactly wordsNeeded(length) words (bitset.go:89-94,
    ReadFrom): words a caller passes beyond them must not surface when Add
    grows the length (extendSetMaybe exposes zero words).  Checked against the
    oracle's Add from the truncated words."""
    from reflow_amd import capi
    rng = np.random.default_rng(11)
    m, k = 4096, 3
    length = 1000                       # 16 words needed
    words = rng.integers(0, 2**63, size=(m + 63) // 64, dtype=np.uint64)  # junk past word 16
    b = capi.Bloom.load(ctx, m, k, words, length)
    keys = rng.integers(0, 256, size=32 * 200, dtype=np.uint8)
    b.add(keys)
    want = np.zeros((m + 63) // 64, dtype=np.uint64)
    need = (length + 63) // 64
    want[:need] = words[:need]
    ln = np.array([length], dtype=np.uint64)
    O.lib().orc_bloomlive_add_batch(want.ctypes.data, ln.ctypes.data, m, k, keys.tobytes(), 200)
    got = b.words()
    assert b.params()[2] == int(ln[0])
    nw = (int(ln[0]) + 63) // 64
    assert (got[:nw] == want[:nw]).all()
    b.close()
