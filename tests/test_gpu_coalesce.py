"""Coalescing concurrent callers into device batches (rf_coalescer, SURVEY
§8(b) "Threading"): many threads each asking for one digest / one probe /
one assoc Get -- the reference's <=60 digest goroutines
(local/executor.go:41,522-538) and its goroutine-per-node lookups
(eval.go:402-411) -- get exactly the results of the batched calls (SHA-256
against the oracle), while the coalescer serves them in far fewer device
batches than requests.  Async tickets complete by poll or wait."""
import random
import threading

import numpy as np
import pytest

from reflow_amd import capi

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


def _threads(n, fn):
    errs = []

    def run(i):
        try:
            fn(i)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
    th = [threading.Thread(target=run, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs[0]


def test_coalesce_sha256_many_threads(ctx, oracle):
    co = capi.Coalescer(ctx, capi.RF_COALESCE_SHA256, max_batch=512, max_wait_us=300)
    n_threads, per = 60, 40  # DigestLimiter = 60 (local/executor.go:41)
    msgs = [[oracle.fill_stream(1000 * t + i, random.Random(t * 7 + i).choice([0, 1, 55, 64, 1000, 70000]))
             for i in range(per)] for t in range(n_threads)]
    got = [[None] * per for _ in range(n_threads)]

    def work(t):
        for i, m in enumerate(msgs[t]):
            got[t][i] = co.sha256(m)
    _threads(n_threads, work)
    for t in range(n_threads):
        assert got[t] == [oracle.sha256(m) for m in msgs[t]], t
    batches, reqs, largest = co.stats()
    assert reqs == n_threads * per
    assert batches < reqs // 4 and largest > 8, (batches, reqs, largest)
    co.close()


def test_coalesce_probe_and_assoc_get(ctx):
    rng = np.random.default_rng(4)
    ins = rng.integers(0, 256, size=(20000, 32), dtype=np.uint8)
    qs = np.concatenate([ins[:4000], rng.integers(0, 256, size=(4000, 32), dtype=np.uint8)])
    b = capi.Bloom.new(ctx, 300000, 7)
    b.add(ins)
    want_p = b.probe(qs)
    a = capi.Assoc(ctx, 1 << 16)
    vals = rng.integers(0, 256, size=(20000, 32), dtype=np.uint8)
    a.put(1, ins, vals)
    want_v, want_f = a.get(1, qs)
    cp = capi.Coalescer(ctx, capi.RF_COALESCE_PROBE, target=b, max_batch=1024, max_wait_us=200)
    ca = capi.Coalescer(ctx, capi.RF_COALESCE_ASSOC_GET, target=a, assoc_kind=1, max_batch=1024, max_wait_us=200)
    got_p = np.zeros(len(qs), np.uint8)
    got_f = np.zeros(len(qs), np.uint8)
    got_v = np.zeros((len(qs), 32), np.uint8)

    def work(t):
        for i in range(t, len(qs), 32):
            got_p[i] = cp.probe(qs[i].tobytes())
            f, v = ca.assoc_get(qs[i].tobytes())
            got_f[i] = f
            got_v[i] = np.frombuffer(v, np.uint8)
    _threads(32, work)
    assert (got_p == want_p).all()
    assert (got_f == want_f).all() and (got_v == want_v).all()
    for c in (cp, ca):
        batches, reqs, _ = c.stats()
        assert reqs == len(qs) and batches < reqs // 4, (batches, reqs)
        c.close()
    b.close()


def test_coalesce_async_tickets(ctx, oracle):
    co = capi.Coalescer(ctx, capi.RF_COALESCE_SHA256, max_batch=4096, max_wait_us=100000)
    msgs = [oracle.fill_stream(i, i * 37 % 5000) for i in range(1000)]
    ts = [co.sha256_async(m) for m in msgs]
    # nobody is flushing: the first poll flushes the whole queue at once
    assert co.poll(ts[0])
    assert all(co.poll(t) for t in ts)
    assert [t["out"].raw for t in ts] == [oracle.sha256(m) for m in msgs]
    assert co.stats()[:2] == (1, 1000)
    t = co.sha256_async(b"abc")
    assert co.wait(t) == oracle.sha256(b"abc")
    for x in ts + [t]:
        co.free(x)
    q = co.sha256_async(b"queued at close")
    co.free(q)  # completes it first
    co.close()


def test_coalescer_bad_open(ctx):
    with pytest.raises(capi.RfError):
        capi.Coalescer(ctx, capi.RF_COALESCE_PROBE)  # no filter
    with pytest.raises(capi.RfError):
        capi.Coalescer(ctx, 9)
