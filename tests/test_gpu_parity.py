"""GPU parity: every kernel, called through the C-ABI, against the oracle.

Bar: bit-exact (integer/byte work).  Sizes are chosen so the oracle finishes
in seconds; full-size properties are in test_gpu_scale.py (configs[2],
configs[4]) and test_gpu_hybrid.py (configs[1] against its fixture).
"""
import random

import numpy as np
import pytest

import reflow_oracle as O
from flowgen import random_dag
from lowering import Lowerer, walk

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from reflow_amd import capi
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


# ------------------------------------------------------------------ K1 --
EDGE_LENS = [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 32, 33, 54, 55, 56, 57, 63, 64, 65, 100, 118, 119,
             120, 121, 127, 128, 129, 183, 184, 191, 192, 1000, 4095, 4096, 4097]


def test_sha256_batch_edge_lengths(ctx):
    rng = random.Random(1)
    msgs = [bytes(rng.getrandbits(8) for _ in range(n)) for n in EDGE_LENS]
    got = ctx.sha256_batch(msgs)
    for m, g in zip(msgs, got):
        assert g == O.sha256(m), len(m)


def test_sha256_fips_vectors(ctx):
    got = ctx.sha256_batch([b"abc", b"", b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq"])
    assert got[0].hex() == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    assert got[1].hex() == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"
    assert got[2].hex() == "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"


def test_sha256_file_content_kat(ctx):
    # local/s3_test.go:69,149: File.ID == Digester.FromString(contents)
    for s in [b"foo", b"bar", b"a/b/c", b"hello world\n" * 300]:
        assert ctx.sha256_batch([s])[0] == O.sha256(s)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_sha256_batch_random_mix(ctx, seed):
    rng = random.Random(seed)
    lens = [rng.choice([rng.randint(0, 200), rng.randint(0, 5000), rng.randint(0, 70000)])
            for _ in range(300)]
    msgs = [bytes(rng.getrandbits(8) for _ in range(n)) if n < 5000 else O.fill_stream(seed * 1000 + i, n)
            for i, n in enumerate(lens)]
    got = ctx.sha256_batch(msgs)
    assert got == [O.sha256(m) for m in msgs]


def _device_arena(lens, align=256):
    offs, pos = [], 0
    for n in lens:
        offs.append(pos)
        pos += (n + align - 1) // align * align
    return np.array(offs, dtype=np.uint64), max(pos, 16)


@pytest.mark.parametrize("flags", [0, 1, 2, 6, 16, 17, 24, 25])
def test_plan_gen_fill_device(ctx, flags):
    """rf_gen_fill + rf_sha_plan_run on HBM-resident data (the bench path):
    planner mix (lane set on eight-per-wave octo chains for this small set) /
    lane messages only (octo: groups of eight with lengths 0 .. 2 MB) /
    wave-per-message with the two-lane chain (2) / with the one-lane chain (6) /
    the producer/chain pair instead of octo (16, 17) / the lanes kernel (24, 25)."""
    from reflow_amd import capi
    rng = random.Random(10 + flags)
    lens = [rng.choice([0, 1, 55, 56, 64, 4096, rng.randint(1, 300000), rng.randint(1, 3000)])
            for _ in range(120)] + [2_000_000, 1_100_000]
    offs, total = _device_arena(lens)
    d_arena = ctx.alloc(total)
    d_offs = ctx.upload(offs)
    d_lens = ctx.upload(np.array(lens, dtype=np.uint64))
    d_out = ctx.alloc(len(lens) * 32)
    seed = 0x5EED0002
    ctx.gen_fill(d_arena.ptr, d_offs.ptr, d_lens.ptr, len(lens), seed, total)
    plan = ctx.sha_plan(offs, np.array(lens, dtype=np.uint64), flags)
    plan.run(d_arena.ptr, d_out.ptr)
    ctx.sync()
    st = plan.stats()
    if flags & capi.RF_SHA_ALL_SOLO:
        assert st.n_solo == len(lens)
    if flags & capi.RF_SHA_NO_SOLO:
        assert st.n_solo == 0
    out = d_out.to_numpy().reshape(-1, 32)
    arena = d_arena.to_numpy()
    for i, n in enumerate(lens):
        want = O.sha256(O.fill_stream(seed ^ i, n))
        # generator parity too: device bytes == oracle stream
        if n <= 4096:
            assert arena[int(offs[i]):int(offs[i]) + n].tobytes() == O.fill_stream(seed ^ i, n)
        assert out[i].tobytes() == want, (i, n)


# ------------------------------------------------------------ Fileset --
def test_fileset_vlist_golden(ctx):
    # executor_test.go:62-86
    f1, f2, f3 = O.from_string("foo"), O.from_string("bar"), O.from_string("a/b/c")
    v1 = [("foo", f1), ("bar", f2)]
    v2 = [("a/b/c", f3), ("bar", f2)]
    got = ctx.fileset_digest_batch([[v1], [v2], [v1, v2], [], [[]]])
    assert O.digest_string(got[2]) == "sha256:d60e67ce9e89548b502a5ad7968e99caed0d388f0a991b906f41a7ba65adb31f"
    assert got[0] != got[1]
    assert got[3] == O.sha256(b"") == got[4]  # empty Map / empty List


def test_fileset_random(ctx):
    rng = random.Random(5)
    sets, want = [], []
    for _ in range(50):
        groups = []
        for _ in range(rng.randint(1, 3)):
            g = [("p%d/%s" % (rng.randint(0, 9), "q" * rng.randint(0, 20)) + str(j),
                  bytes(rng.getrandbits(8) for _ in range(32))) for j in range(rng.randint(0, 30))]
            groups.append(g)
        sets.append(groups)
        fs = O.OFileset(list=[O.OFileset(map={p: (d, 0) for p, d in g}) for g in groups])
        want.append(fs.digest())
    assert ctx.fileset_digest_batch(sets) == want


def test_fileset_device_ids(ctx):
    """rf_fileset_digest_device (IDs in HBM, placed into the material on the
    device) == rf_fileset_digest_batch == oracle, incl. empty sets/groups and
    unaligned path lengths."""
    rng = random.Random(9)
    sets, flat_ids, want = [], [], []
    for k in range(40):
        groups = []
        for _ in range(rng.randint(0, 3)):
            g = [("d%d/%s%d" % (rng.randint(0, 5), "x" * rng.randint(0, 70), j),
                  bytes(rng.getrandbits(8) for _ in range(32))) for j in range(rng.randint(0, 40))]
            groups.append(g)
        sets.append(groups)
        fs = O.OFileset(list=[O.OFileset(map={p: (d, 0) for p, d in g}) for g in groups])
        want.append(fs.digest())
        flat_ids.extend(d for g in groups for _, d in g)
    host = ctx.fileset_digest_batch(sets)
    fp = ctx.fileset_paths([[[p for p, _ in g] for g in groups] for groups in sets])
    d_ids = ctx.upload(np.frombuffer(b"".join(flat_ids) or b"\0" * 32, dtype=np.uint8).copy())
    try:
        dev = fp.digest_device(d_ids.ptr)
    finally:
        d_ids.free()
    assert host == want
    assert dev == want


# ---------------------------------------------------------- digest DAG --
def _load(ctx, low):
    from reflow_amd import capi
    a = low.L.arrays()
    return capi.Graph(ctx, a["n_slots"], a["out_slot"], a["tmpl_off"], a["tmpl_len"],
                      a["hole_ptr"], a["hole_pos"], a["hole_slot"], a["blob"])


def _stable_flow():
    from test_oracle_golden import stable_flow
    return stable_flow()


def test_graph_stable_flow_v2_v1(ctx):
    for v1, want in [(False, "sha256:02751e46c573a31747a30b05c2b73b2eb556fb45fb4c0aaf88d170f4b5e6d4e7"),
                     (True, "sha256:5a3a916fe9a11b67f9a0dbd67f6fac0f986dd67803267e79f25f866ca9781e2f")]:
        root = _stable_flow()
        low = Lowerer()
        s = low.lower(root, v1=v1)
        g = _load(ctx, low)
        g.recompute(full=True)
        assert O.digest_string(g.get_slots([s])[0].tobytes()) == want


@pytest.mark.parametrize("seed,universe", [(1, b""), (2, b""), (3, b"myuniverse"), (4, b"u")])
def test_graph_random_dag_full(ctx, seed, universe):
    root, nodes = random_dag(seed, n=80)
    low = Lowerer(universe=universe)
    slots, pslots, fl = [], [], []
    for f in walk(root):
        slots.append(low.lower(f))
        pslots.append(low.lower_physical(f))
        fl.append(f)
    g = _load(ctx, low)
    assert g.recompute(full=True) == len(low.L.jobs)
    got = g.get_slots(slots)
    for f, s, d in zip(fl, slots, got):
        assert d.tobytes() == f.digest(universe), f.op
    for f, ps in zip(fl, pslots):
        if ps is not None:
            assert g.get_slots([ps])[0].tobytes() == f.physical_digest()
        else:
            assert f.physical_digest() is None


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_graph_incremental_equals_full(ctx, seed):
    """K3 frontier + early cut-off: after changing File IDs, the incremental
    recompute equals the oracle on the changed graph, and hashes exactly the
    jobs that depend on a changed input."""
    root, nodes = random_dag(seed, n=120)
    low = Lowerer(file_slots=True)
    fl = walk(root)
    slots = [low.lower(f) for f in fl]
    pslots = [low.lower_physical(f) for f in fl]
    g = _load(ctx, low)
    fs_items = list(low.L.file_slot.items())
    g.set_slots([s for _, s in fs_items], np.frombuffer(b"".join(fid for fid, _ in fs_items), np.uint8))
    g.recompute(full=True)
    rng = random.Random(seed)
    for rnd in range(3):
        change = rng.sample(fs_items, max(1, len(fs_items) // 10))
        # mutate oracle values in place: new ID = SHA256(old || "v2")  
        newid = {}
        for fid, s in change:
            newid[fid] = O.sha256(fid + b"v2")
        for f in fl:
            for v in _filesets(f):
                for p, (fid, size) in list((v.map or {}).items()):
                    if fid in newid:
                        v.map[p] = (newid[fid], size)
        g.set_slots([s for _, s in change], np.frombuffer(b"".join(newid[f] for f, _ in change), np.uint8))
        # update the test-side id map so later rounds can change them again
        fs_items = [(newid.get(fid, fid), s) for fid, s in fs_items]
        n = g.recompute(full=False)
        got = g.get_slots(slots)
        for f, d in zip(fl, got):
            assert d.tobytes() == f.digest(), f.op
        for f, ps in zip(fl, pslots):
            if ps is not None:
                assert g.get_slots([ps])[0].tobytes() == f.physical_digest()
        assert 0 < n <= len(low.L.jobs)


def _filesets(f):
    out = []
    if f.value is not None:
        stack = [f.value]
        while stack:
            v = stack.pop()
            out.append(v)
            if v.list:
                stack.extend(v.list)
    return out


def test_graph_rejects_cycle_and_bad_slots(ctx):
    from reflow_amd import capi
    # job0 writes slot0 reading slot1; job1 writes slot1 reading slot0
    mat = b"\x00\x05" + b"\0" * 32
    with pytest.raises(capi.RfError) as e:
        capi.Graph(ctx, 2, [0, 1], [0, 48], [34, 34], [0, 1, 2], [2, 2], [1, 0], mat + b"\0" * 14 + mat)
    assert e.value.code == capi.RF_EINVAL
    low = Lowerer()
    s = low.lower(O.OFlow("OpIntern", url="x"))
    g = _load(ctx, low)
    with pytest.raises(capi.RfError):
        g.set_slots([s], np.zeros(32, np.uint8))  # output slot


def test_graph_wide_fanin(ctx):
    """A wide OpK (fan-in 500: 17,000 B of material, 266 blocks) -- the serial
    Amdahl case of syntax/force.go:180-198."""
    leaves = [O.OFlow("OpIntern", url="s3://x/%d" % i) for i in range(500)]
    k = O.OFlow("OpK", leaves, flow_digest=O.from_string("wide"))
    low = Lowerer()
    s = low.lower(k)
    g = _load(ctx, low)
    g.recompute(full=True)
    assert g.get_slots([s])[0].tobytes() == k.digest()


# --------------------------------------------------------------- bloom --
def _oracle_filter(keys32: bytes, n, p=0.01):
    m, k = O.estimate_parameters(n, p)
    words = np.zeros((m + 63) // 64, dtype=np.uint64)
    length = np.array([m], dtype=np.uint64)
    O.lib().orc_bloomlive_add_batch(words.ctypes.data, length.ctypes.data, m, k, keys32, n)
    return m, k, words, int(length[0])


def _oracle_probe(words, length, m, k, keys32, n):
    out = np.zeros(n, dtype=np.uint8)
    O.lib().orc_bloomlive_contains_batch(words.ctypes.data, length, m, k, keys32, n, out.ctypes.data, 4)
    return out


@pytest.mark.parametrize("n,p", [(1, 0.5), (100, 0.01), (5000, 0.001), (3000, 1e-6)])
def test_bloom_probe_parity(ctx, n, p):
    from reflow_amd import capi
    rng = np.random.default_rng(n)
    keys = rng.integers(0, 256, size=32 * n, dtype=np.uint8).tobytes()
    m, k, words, length = _oracle_filter(keys, n, p)
    b = capi.Bloom.load(ctx, m, k, words, length)
    probes = keys + rng.integers(0, 256, size=32 * 4 * n, dtype=np.uint8).tobytes()
    got = b.probe(np.frombuffer(probes, np.uint8))
    want = _oracle_probe(words, length, m, k, probes, len(probes) // 32)
    assert (got == want).all()
    assert got[:n].all()


def test_bloom_add_bit_exact(ctx):
    from reflow_amd import capi
    rng = np.random.default_rng(3)
    n = 20000
    keys = rng.integers(0, 256, size=32 * n, dtype=np.uint8)
    m, k = O.estimate_parameters(n, 0.001)
    b = capi.Bloom.new(ctx, m, k)
    b.add(keys)
    _, _, words, length = _oracle_filter(keys.tobytes(), n, 0.001)
    assert b.params()[2] == length
    assert (b.words() == words).all()


def test_bloom_wire_formats(ctx):
    """Go JSON {"m","k","b":base64url(BE64 len ‖ BE64 words)} and binary
    (bloom.go:264-325, bitset.go:628-721), probe parity on both."""
    import base64
    import struct
    from reflow_amd import capi
    rng = np.random.default_rng(9)
    n = 700
    keys = rng.integers(0, 256, size=32 * n, dtype=np.uint8).tobytes()
    m, k, words, length = _oracle_filter(keys, n, 0.01)
    bits = struct.pack(">Q", length) + b"".join(struct.pack(">Q", int(w)) for w in words)
    js = b'{"m":%d,"k":%d,"b":"%s"}' % (m, k, base64.urlsafe_b64encode(bits))
    binary = struct.pack(">QQ", m, k) + bits
    probes = np.frombuffer(keys + rng.integers(0, 256, size=32 * n, dtype=np.uint8).tobytes(), np.uint8)
    want = _oracle_probe(words, length, m, k, probes.tobytes(), 2 * n)
    for b in (capi.Bloom.from_json(ctx, js), capi.Bloom.from_binary(ctx, binary)):
        assert (b.probe(probes) == want).all()


def test_bloom_edge_filters(ctx):
    """bloom.New(64,1) (eval.go:843) and a short bitset (loc >= length => false)."""
    from reflow_amd import capi
    rng = np.random.default_rng(4)
    keys = rng.integers(0, 256, size=32 * 50, dtype=np.uint8)
    b = capi.Bloom.new(ctx, 64, 1)
    assert not b.probe(keys).any()
    b.add(keys[:32])
    assert b.probe(keys[:32])[0] == 1
    # filter whose bitset length is shorter than m
    m, k = 1000, 3
    words = np.full(4, np.uint64(0xFFFFFFFFFFFFFFFF), dtype=np.uint64)
    b2 = capi.Bloom.load(ctx, m, k, words, 256)
    want = _oracle_probe(words, 256, m, k, keys.tobytes(), 50)
    assert (b2.probe(keys) == want).all()


# --------------------------------------------------------------- RCCL --
def test_rccl_single_rank_allgather_and_or(ctx):
    """rf_comm_* over RCCL with one rank (the 1-GPU box): all-gather copies the
    boundary digests, the OR all-reduce (all-gather + OR kernel) is identity."""
    from reflow_amd import capi
    uid = capi.Comm.unique_id()
    comm = capi.Comm(ctx, 1, 0, uid)
    rng = np.random.default_rng(2)
    words = rng.integers(0, 2**63, size=1000, dtype=np.uint64)
    d = ctx.upload(words)
    comm.allreduce_or(d.ptr, len(words), ctx.stream)
    ctx.sync()
    assert (d.to_numpy(np.uint64) == words).all()
    src = ctx.upload(rng.integers(0, 256, size=32 * 77, dtype=np.uint8))
    dst = ctx.alloc(32 * 77)
    comm.allgather(src.ptr, dst.ptr, 32 * 77, ctx.stream)
    ctx.sync()
    assert (dst.to_numpy() == src.to_numpy()).all()
    comm.close()
