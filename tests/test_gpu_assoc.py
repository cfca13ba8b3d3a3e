"""HBM assoc: assoc.Assoc (assoc/assoc.go:26-38) with
the in-memory implementation's semantics (test/testutil/assoc.go:34-56) and
dydbassoc's abbreviated-key expansion (assoc/dydbassoc/dydbassoc.go:111-147),
checked op for op against the oracle's restatement (reflow_oracle.InmemoryAssoc)."""
import random

import numpy as np
import pytest

import reflow_oracle as O

pytestmark = pytest.mark.gpu
ZERO = bytes(32)


@pytest.fixture(scope="module")
def ctx():
    from reflow_amd import capi
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


def _status_name(code):
    from reflow_amd import capi
    return {capi.RF_OK: "ok", capi.RF_EPRECONDITION: "precondition"}[int(code)]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_assoc_batches_match_inmemory(ctx, seed):
    """Batches with repeated keys (applied in index order), CAS with matching,
    wrong and zero expects, deletes and re-inserts, two kinds."""
    from reflow_amd import capi
    rng = random.Random(seed)
    pool = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(300)]
    vals = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(50)]
    a = capi.Assoc(ctx, capacity=16)  # forces several rehashes
    ref = O.InmemoryAssoc()
    for b in range(12):
        kind = b % 2
        n = rng.choice([1, 7, 500, 3000])
        keys, vs, exps = [], [], []
        for _ in range(n):
            k = rng.choice(pool)
            v = ZERO if rng.random() < 0.1 else rng.choice(vals)
            r = rng.random()
            cur = ref.get(kind, k)
            e = ZERO if r < 0.5 else (cur or ZERO) if r < 0.7 else rng.choice(vals)
            keys.append(k)
            vs.append(v)
            exps.append(e)
        use_expect = b % 3 != 0
        st = a.put(kind, np.frombuffer(b"".join(keys), np.uint8), np.frombuffer(b"".join(vs), np.uint8),
                   np.frombuffer(b"".join(exps), np.uint8) if use_expect else None)
        want = [ref.put(kind, e if use_expect else None, k, v) for k, v, e in zip(keys, vs, exps)]
        assert [_status_name(x) for x in st] == want, "batch %d" % b
        for kd in (0, 1):
            got, found = a.get(kd, np.frombuffer(b"".join(pool), np.uint8))
            for i, k in enumerate(pool):
                w = ref.get(kd, k)
                assert bool(found[i]) == (w is not None)
                assert got[i].tobytes() == (w or ZERO)
    a.close()


def test_assoc_large_and_growth(ctx):
    from reflow_amd import capi
    rng = np.random.default_rng(5)
    n = 1_000_000
    keys = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    vals = rng.integers(1, 256, size=(n, 32), dtype=np.uint8)
    a = capi.Assoc(ctx, capacity=1000)
    st = a.put(0, keys, vals)
    assert (st == 0).all()
    occ, cap = a.stats()
    assert occ == n and cap >= 2 * n
    probe = np.concatenate([keys[::2], rng.integers(0, 256, size=(n // 2, 32), dtype=np.uint8)])
    got, found = a.get(0, probe)
    assert found[:n // 2].all() and not found[n // 2:].any()
    assert (got[:n // 2] == vals[::2]).all()
    _, found1 = a.get(1, keys[:1000])  # other kind: nothing
    assert not found1.any()
    a.close()


@pytest.mark.parametrize("word", [1, 3, 4, 6])
def test_assoc_keys_differing_in_one_word(ctx, word):
    """A Put batch of 100k keys equal everywhere but one 4-byte word (the
    ADVICE r02 case: the batch dedup's probe run used to exceed its bound and
    the apply kernels then indexed by ~0), with repeats: every op applies in
    index order, a later Get sees the last value per key."""
    rng = np.random.default_rng(100 + word)
    n = 100_000
    keys = np.tile(rng.integers(0, 256, size=(1, 32), dtype=np.uint8), (n, 1))
    keys[:, 4 * word:4 * word + 4] = np.arange(n, dtype=np.uint32).view(np.uint8).reshape(n, 4)
    rep = rng.integers(0, n, size=n // 4)
    batch = np.concatenate([keys, keys[rep]])
    vals = rng.integers(1, 256, size=(len(batch), 32), dtype=np.uint8)
    from reflow_amd import capi
    a = capi.Assoc(ctx, capacity=1024)
    st = a.put(0, batch.reshape(-1), vals.reshape(-1))
    assert (st == 0).all()
    src = np.arange(n)
    for j, r in enumerate(rep.tolist()):  # ops in index order: the last Put per key wins
        src[r] = n + j
    last = vals[src]
    got, found = a.get(0, keys.reshape(-1))
    assert found.all() and (got == last).all()
    assert a.stats()[0] == n
    a.close()


def test_assoc_abbrev_expansion(ctx):
    from reflow_amd import capi
    rng = random.Random(9)
    a = capi.Assoc(ctx)
    ref = O.InmemoryAssoc()
    base = bytes(rng.getrandbits(8) for _ in range(32))
    keys = [base[:4] + bytes(rng.getrandbits(8) for _ in range(28)) for _ in range(5)]  # same ID4
    keys.append(base[:4] + b"\xab" + bytes(27))
    keys.append(base[:4] + b"\xac" + bytes(27))
    keys += [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(200)]
    vals = [bytes([1 + i % 250]) * 32 for i in range(len(keys))]
    a.put(0, np.frombuffer(b"".join(keys), np.uint8), np.frombuffer(b"".join(vals), np.uint8))
    for k, v in zip(keys, vals):
        ref.put(0, None, k, v)
    # delete one of the unique ones: it must not match any more
    a.put(0, np.frombuffer(keys[10], np.uint8), np.frombuffer(ZERO, np.uint8))
    ref.put(0, None, keys[10], ZERO)
    queries = [(keys[0].hex()[:8], 8), (keys[0].hex()[:64], 64), (keys[5].hex()[:9], 9),
               (keys[6].hex()[:10], 10), (keys[10].hex()[:16], 16), (keys[20].hex()[:11], 11),
               ("00000000", 8)]
    qk = b"".join(bytes.fromhex((h + "0" * 64)[:64]) for h, _ in queries)
    ko, vo, st = a.get_abbrev(0, np.frombuffer(qk, np.uint8), [nh for _, nh in queries])
    for j, (h, nh) in enumerate(queries):
        want, hit = ref.get_abbrev(0, h[:nh])
        code = {"ok": capi.RF_OK, "notexist": capi.RF_ENOTFOUND, "invalid": capi.RF_EINVAL}[want]
        assert st[j] == code, (h, nh)
        if want == "ok":
            assert ko[j].tobytes() == hit[0] and vo[j].tobytes() == hit[1]
    a.close()


def capi_assoc(ctx, capacity):
    from reflow_amd import capi
    return capi.Assoc(ctx, capacity=capacity)


def _lookup_case(rng, n_nodes, pool, vals):
    """Nodes with 0..3 cache keys (CacheKeys gives 1-2; 0 and 3 are edges),
    keys shared between nodes (synonyms), some keys present."""
    node_keys = [[rng.choice(pool) for _ in range(rng.choice([0, 1, 2, 2, 2, 3]))] for _ in range(n_nodes)]
    preset = [(k, rng.choice(vals)) for k in rng.sample(pool, len(pool) // 3)]
    return node_keys, preset


@pytest.mark.parametrize("repair", [0, 1, 2])
def test_assoc_lookup_matches_oracle(ctx, repair):
    """Eval.lookup's assoc step (eval.go:1172-1258) for a batch of nodes: one
    Get batch (rf_assoc_lookup, read only); the caller's unmarshal rejects some
    fsids (the next found key wins, :1210-1218) and its missing() check fails
    some nodes; rf_assoc_repair then writes blind (1) or precise (2) repairs
    for the verified nodes only.  The table after each batch equals the
    oracle's, key for key."""
    rng = random.Random(40 + repair)
    pool = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(400)]
    vals = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(40)]
    bad = set(vals[:6])          # fsids that do not unmarshal
    a = capi_assoc(ctx, 64)
    ref = O.InmemoryAssoc()
    for rnd in range(3):  # repairs of one batch feed the next
        node_keys, preset = _lookup_case(rng, 700, pool, vals)
        if rnd == 0:
            for k, v in preset:
                ref.put(0, None, k, v)
            st = a.put(0, np.frombuffer(b"".join(k for k, _ in preset), np.uint8),
                       np.frombuffer(b"".join(v for _, v in preset), np.uint8))
            assert (st == 0).all()
        unverified = set(rng.sample(range(700), 60))  # nodes whose files are missing
        want = O.eval_lookup(ref, 0, node_keys, repair, usable=lambda i, v: v not in bad,
                             verified=lambda i, v: i not in unverified)
        flat = b"".join(k for ks in node_keys for k in ks)
        ptr = np.cumsum([0] + [len(ks) for ks in node_keys]).astype(np.uint64)
        kb = np.frombuffer(flat, np.uint8)
        which, got, kf, kv = a.lookup(0, kb, ptr)
        # the caller's key loop over the per-key results
        w2, v2, rep = [], [], []
        for i, ks in enumerate(node_keys):
            w = next((j for j in range(len(ks)) if kf[ptr[i] + j] and kv[ptr[i] + j].tobytes() not in bad), -1)
            v = kv[ptr[i] + w].tobytes() if w >= 0 else ZERO
            w2.append(w)
            v2.append(v)
            rep.append(w if w >= 0 and i not in unverified else -1)
        assert list(zip(w2, v2)) == want
        first = [next((j for j in range(len(ks)) if kf[ptr[i] + j]), -1) for i, ks in enumerate(node_keys)]
        assert [int(x) for x in which] == first
        if repair:
            a.repair(0, kb, ptr, rep, np.frombuffer(b"".join(v2), np.uint8).reshape(-1, 32),
                     kf if repair == 2 else None)
    allk = np.frombuffer(b"".join(pool), np.uint8)
    gv, gf = a.get(0, allk)
    for i, k in enumerate(pool):
        r = ref.get(0, k)
        assert (r is not None) == bool(gf[i]) and (r is None or gv[i].tobytes() == r)

