"""K1 planner with its host leg: the largest messages of a batch on SHA-NI host
threads (the reference's <=60-goroutine digest pool, local/executor.go:41,
522-538), the rest on the GPU kernels, every digest checked against the
oracle (oracle/oracle.c, scalar FIPS-180-4) -- for HBM-resident sets (host
leg fed by chunked D2H), host-buffer batches (rf_sha256_batch), Fileset
digests and Executor.install, plus configs[1] in full against its committed
fixture (tests/golden/make_c2_fixture.py).

Every other GPU test module pins its context to the GPU kernels
(host_threads=0); this one runs the library default.
"""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

from reflow_amd import capi
from reflow_amd.workloads import GiB, MiB, arena_layout, c2_sizes

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
C2_SEED = 0x5EED0002


@pytest.fixture(scope="module")
def ctx():
    c = capi.Context(0)
    if c.host_info()[0] == 0:
        pytest.skip("host leg unavailable (no SHA extensions)")
    yield c
    c.close()


def _want(oracle, lens, seed):
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    out = np.zeros(32 * max(len(lens), 1), dtype=np.uint8)
    oracle.lib().orc_stream_sha256_batch(seed, lens.ctypes.data, len(lens), out.ctypes.data, os.cpu_count() or 1)
    return out[:32 * len(lens)].reshape(-1, 32)


class DeviceSet:
    def __init__(self, ctx, lens, seed):
        self.lens = np.ascontiguousarray(lens, dtype=np.uint64)
        self.offs, total = arena_layout(self.lens)
        self.arena = ctx.alloc(total)
        self.d_offs, self.d_lens = ctx.upload(self.offs), ctx.upload(self.lens)
        self.out = ctx.alloc(32 * max(len(self.lens), 1))
        ctx.gen_fill(self.arena.ptr, self.d_offs.ptr, self.d_lens.ptr, len(self.lens), seed, total)
        ctx.sync()

    def run(self, ctx, flags=0, reps=1):
        plan = ctx.sha_plan(self.offs, self.lens, flags)
        for _ in range(reps):
            plan.run(self.arena.ptr, self.out.ptr)
        st = plan.stats()
        plan.close()
        ctx.sync()
        return self.out.to_numpy(count=32 * len(self.lens)).reshape(-1, 32), st

    def free(self):
        for b in (self.arena, self.d_offs, self.d_lens, self.out):
            b.free()


# lengths around the SHA-256 padding edges and the host leg's 8 MiB D2H chunks
EDGES = [0, 1, 55, 56, 63, 64, 65, 119, 120, 127, 128, 4095, 8 * MiB - 1, 8 * MiB, 8 * MiB + 1,
         8 * MiB + 55, 8 * MiB + 64, 16 * MiB + 37, 3 * MiB + 56]


def test_host_leg_all_host_edges(ctx, oracle):
    ds = DeviceSet(ctx, EDGES, 0x1234)
    got, st = ds.run(ctx, capi.RF_SHA_ALL_HOST)
    assert st.n_host == len(EDGES) and st.host_threads > 0
    assert (got == _want(oracle, EDGES, 0x1234)).all()
    ds.free()


def test_no_host_flag_pins_gpu(ctx, oracle):
    lens = [64 * MiB, 100, 5000]
    ds = DeviceSet(ctx, lens, 77)
    got, st = ds.run(ctx, capi.RF_SHA_NO_HOST)
    assert st.n_host == 0
    assert (got == _want(oracle, lens, 77)).all()
    ds.free()


def test_flag_conflicts(ctx):
    with pytest.raises(capi.RfError) as e:
        ctx.sha_plan(np.zeros(1, np.uint64), np.ones(1, np.uint64), capi.RF_SHA_ALL_HOST | capi.RF_SHA_NO_HOST)
    assert e.value.code == capi.RF_EINVAL
    c0 = capi.Context(0, host_threads=0)
    with pytest.raises(capi.RfError) as e:
        c0.sha_plan(np.zeros(1, np.uint64), np.ones(1, np.uint64), capi.RF_SHA_ALL_HOST)
    assert e.value.code == capi.RF_EINVAL
    c0.close()


def test_hybrid_split_mixed_set(ctx, oracle):
    """A skewed set: the two long chains go to the host leg, the 3000 short
    ones to the GPU kernels; back-to-back runs (the host digests' upload of
    run 1 still queued when run 2's host leg starts) stay correct."""
    rng = np.random.default_rng(5)
    lens = np.concatenate([[96 * MiB, 72 * MiB], rng.integers(1, 256 * 1024, size=3000)]).astype(np.uint64)
    ds = DeviceSet(ctx, lens, 99)
    got, st = ds.run(ctx, 0, reps=3)
    assert 0 < st.n_host < len(lens), (st.n_host, len(lens))
    assert st.host_bytes >= 72 * MiB
    assert (got == _want(oracle, lens, 99)).all()
    ds.free()


def test_hybrid_host_buffer_batch(ctx, oracle):
    """rf_sha256_batch (host buffers): host-leg messages hashed in place, only
    the GPU messages' bytes uploaded."""
    sizes = [0, 1, 64, 70000, 5 * MiB, 33 * MiB - 1, 12345, 8 * MiB + 7]
    msgs = [oracle.fill_stream(0x77 ^ i, n) for i, n in enumerate(sizes)]
    msgs += [oracle.fill_stream(0x99 ^ i, 3000 + 17 * i) for i in range(2000)]
    got = ctx.sha256_batch(msgs)
    assert got == [hashlib.sha256(m).digest() for m in msgs]


def test_hybrid_fileset_and_install(ctx, oracle, tmp_path):
    """Fileset digests (one long material per set) and Executor.install with a
    large file beside small ones, default host leg."""
    fid = [oracle.from_string("f%d" % i) for i in range(3000)]
    sets = [[[("p%05d" % i, fid[i]) for i in range(3000)]], [[("a", fid[0])]], []]
    want = [oracle.OFileset(map={p: (d, 0) for p, d in g[0]} if g else {}).digest() for g in sets]
    assert ctx.fileset_digest_batch(sets) == want
    (tmp_path / "d").mkdir()
    (tmp_path / "d" / "big.bam").write_bytes(oracle.fill_stream(3, 40 * MiB + 11))
    for i in range(50):
        (tmp_path / "d" / ("s%02d" % i)).write_bytes(oracle.fill_stream(4 + i, 100 * i))
    ents, fsd = ctx.install_dir(str(tmp_path))
    w_ents, w_fsd = oracle.install_dir(str(tmp_path))
    assert [(r, i, s) for r, i, s in ents] == w_ents and fsd == w_fsd


def _c2_fixture():
    meta_p, ids_p = os.path.join(HERE, "golden", "c2_ids.json"), os.path.join(HERE, "golden", "c2_ids.bin")
    if not (os.path.exists(meta_p) and os.path.exists(ids_p)):
        pytest.skip("configs[1] fixture not generated (tests/golden/make_c2_fixture.py)")
    meta = json.load(open(meta_p))
    lens = c2_sizes(total_bytes=64 * GiB, seed=C2_SEED)
    assert hashlib.sha256(lens.tobytes()).hexdigest() == meta["lens_sha256"]
    ids = np.fromfile(ids_p, dtype=np.uint8).reshape(-1, 32)
    assert hashlib.sha256(ids.tobytes()).hexdigest() == meta["ids_sha256"]
    return lens, ids


@pytest.fixture(scope="module")
def c2_set(ctx):
    lens, ids = _c2_fixture()
    ds = DeviceSet(ctx, lens, C2_SEED)
    yield ds, ids
    ds.free()


def test_c2_full_hybrid_vs_fixture(ctx, c2_set):
    """configs[1] in full (64 GiB, 5623 files, 4 KiB - 1.95 GiB): every File ID
    equals the committed fixture; the planner used both legs."""
    ds, ids = c2_set
    got, st = ds.run(ctx, 0)
    assert 0 < st.n_host < len(ds.lens)
    bad = np.nonzero((got != ids).any(axis=1))[0]
    assert len(bad) == 0, "mismatching files: %s" % bad[:10].tolist()


def test_c2_largest_file_on_duo_vs_fixture(ctx, c2_set):
    """The 1.95 GiB file of configs[1] (32.7M-block chain) through
    k1_sha256_duo alone (no host leg): its File ID equals the fixture."""
    ds, ids = c2_set
    i = int(np.argmax(ds.lens))
    plan = ctx.sha_plan(ds.offs[i:i + 1], ds.lens[i:i + 1], capi.RF_SHA_NO_HOST | capi.RF_SHA_ALL_SOLO)
    out = ctx.alloc(32)
    plan.run(ds.arena.ptr, out.ptr)
    st = plan.stats()
    assert st.n_solo == 1 and st.n_host == 0
    assert out.to_numpy().tobytes() == ids[i].tobytes()
    plan.close()
    out.free()


def test_plan_host_leg_does_not_hold_the_context(ctx, oracle):
    """rf_sha_plan_run releases the context mutex while its host leg hashes
    (ADVICE r02): a dedup batch on the same context, issued from another
    thread while a 2 GiB message runs on the host leg, returns before the
    plan does; both results are right."""
    import threading
    import time
    lens = np.array([2 * GiB - 100] + [4096] * 64, dtype=np.uint64)
    ds = DeviceSet(ctx, lens, 77)
    plan = ctx.sha_plan(ds.offs, ds.lens, capi.RF_SHA_ALL_HOST)
    assert plan.stats().n_host == len(lens)
    rng = np.random.default_rng(3)
    dig = rng.integers(0, 256, size=(200_000, 32), dtype=np.uint8)
    dig[100_000:] = dig[:100_000]
    done = {}

    def run_plan():
        plan.run(ds.arena.ptr, ds.out.ptr)
        plan.stats()  # synchronises
        done["plan"] = time.perf_counter()

    th = threading.Thread(target=run_plan)
    th.start()
    time.sleep(0.2)  # the host leg is hashing by now (~0.6 s for 2 GiB on one thread)
    canon, nu = ctx.dedup_digests(dig)
    done["dedup"] = time.perf_counter()
    th.join()
    plan.close()
    assert nu == 100_000 and (canon[100_000:] == np.arange(100_000)).all()
    assert done["dedup"] < done["plan"], done
    got = ds.out.to_numpy().reshape(-1, 32)
    host = ds.arena.to_numpy()
    for i in range(len(lens)):  # hashlib over the device's own bytes (the big one would take the oracle ~7 s)
        o = int(ds.offs[i])
        assert got[i].tobytes() == hashlib.sha256(host[o:o + int(lens[i])].tobytes()).digest(), i
