"""Checkpoint / resume of a loaded digest DAG (rf_graph_save,
rf_graph_restore): a graph saved after a full recompute and an incremental
step, destroyed, and restored in place of a fresh load gives -- after a
further 1% change -- exactly the oracle's digests (the reference's resume is
memoization: runner/runner.go:51-85 persists State per step,
local/executor.go:122-200 restores execs from manifests).  Damaged files are
refused: flipped bytes and truncation with RF_EINTEGRITY (errors.Integrity),
a file that is not a checkpoint with RF_EINVAL, a missing one with RF_EIO."""
import os

import numpy as np
import pytest

import partition_case as PC
import reflow_oracle as O
from reflow_amd import capi
from reflow_amd.workloads import Dag1000, PartitionedDag1000

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


def _load(ctx, dag):
    g = capi.Graph.from_arrays(ctx, dag.arrays())
    g.set_slots(dag.file_slots, dag.leaf_ids)
    return g


def test_save_restore_then_incremental_matches_oracle(ctx, tmp_path):
    dag = Dag1000(12, 6)
    a = dag.arrays()
    every = np.arange(a["n_slots"], dtype=np.uint32)
    g = _load(ctx, dag)
    g.recompute(full=True)
    sa, _, na = dag.change_set(0.1, seed=1)
    g.set_slots(sa, na)
    g.recompute(full=False)
    before = g.get_slots(every)
    path = str(tmp_path / "g.ckpt")
    g.save(path)
    g.close()
    r = capi.Graph.restore(ctx, path)
    assert (r.get_slots(every) == before).all()
    st = r.stats()
    assert st.n_jobs == len(a["out_slot"]) and st.n_slots == a["n_slots"]
    # a second change on the restored graph, against the oracle from scratch
    sb, _, nb = dag.change_set(0.1, seed=2)
    nb = np.frombuffer(bytes(np.asarray(nb).tobytes()[::-1]), np.uint8).reshape(-1, 32)  # not SHA(old||v2)
    r.set_slots(sb, nb)
    n = r.recompute(full=False)
    assert 0 < n < len(a["out_slot"])
    og = O.OGraph(a)
    og.set_inputs(dag.file_slots, dag.leaf_ids)
    og.full()
    og.update(sa, na)
    og.update(sb, nb)
    assert (r.get_slots(every) == og.slots[:a["n_slots"]]).all()
    og.close()
    # input slots stay inputs, job outputs stay refused
    with pytest.raises(capi.RfError):
        r.set_slots(np.array([a["out_slot"][0]], np.uint32), np.zeros((1, 32), np.uint8))
    r.close()


def test_restore_equals_fresh_load_large(ctx, tmp_path):
    """~0.9M nodes: restored + 1% change == fresh load + full recompute of the
    same inputs, slot for slot."""
    dag = Dag1000(2000, 32)
    every = np.arange(dag.n_slots, dtype=np.uint32)
    g = _load(ctx, dag)
    g.recompute(full=True)
    path = str(tmp_path / "big.ckpt")
    g.save(path)
    g.close()
    r = capi.Graph.restore(ctx, path)
    sl, _, nw = dag.change_set(0.01)
    r.set_slots(sl, nw)
    r.recompute(full=False)
    f = _load(ctx, dag)
    f.set_slots(sl, nw)
    f.recompute(full=True)
    assert (r.get_slots(every) == f.get_slots(every)).all()
    r.close()
    f.close()


def test_damaged_checkpoints_refused(ctx, tmp_path):
    dag = Dag1000(3, 4)
    g = _load(ctx, dag)
    g.recompute(full=True)
    path = str(tmp_path / "d.ckpt")
    g.save(path)
    g.close()
    raw = open(path, "rb").read()
    assert not os.path.exists(path + ".tmp")

    def refused(data, code):
        p = str(tmp_path / "x.ckpt")
        open(p, "wb").write(data)
        with pytest.raises(capi.RfError) as e:
            capi.Graph.restore(ctx, p)
        assert e.value.code == code, e.value

    for pos in (200, len(raw) // 2, len(raw) - 50):  # a section byte, the middle, the checksum list
        bad = bytearray(raw)
        bad[pos] ^= 0x40
        refused(bytes(bad), capi.RF_EINTEGRITY)
    refused(raw[:len(raw) // 3], capi.RF_EINTEGRITY)
    refused(raw[:-1], capi.RF_EINTEGRITY)
    refused(b"not a checkpoint" * 20, capi.RF_EINVAL)
    with pytest.raises(capi.RfError) as e:
        capi.Graph.restore(ctx, str(tmp_path / "missing.ckpt"))
    assert e.value.code == capi.RF_EIO
    # the intact file still restores
    open(str(tmp_path / "ok.ckpt"), "wb").write(raw)
    capi.Graph.restore(ctx, str(tmp_path / "ok.ckpt")).close()


def test_restored_pieces_resume_partitioned(tmp_path):
    """Two ranks (threads, one GPU) save their pieces of configs[3]'s layout,
    restore them, re-attach the partition and take an incremental step
    across ranks: the slots equal the oracle's single-rank evaluation."""
    S, P, nr = 8, 4, 2
    G, ga, owner, roots, trees, groot = PC.global_c4(S, P, nr, fanin=4)
    rng = np.random.default_rng(4)
    pick = np.sort(rng.choice(len(G.file_slots), size=9, replace=False))
    new = G.leaf_ids.copy()
    new[pick] = rng.integers(0, 256, size=(len(pick), 32), dtype=np.uint8)
    want = PC.global_digests(G, ga, new)

    def body(r, ag):
        pc = PartitionedDag1000(S, P, nr, r, fanin=4)
        m = PC.c4_local_to_global(pc, G, roots, trees, groot)
        c = capi.Context(0, host_threads=0)
        try:
            g = capi.Graph.from_arrays(c, pc.desc)
            g.set_part(pc.part)
            g.set_slots(pc.dag.file_slots, pc.dag.leaf_ids)
            g.recompute_part(allgather=ag, nranks=nr, full=True)
            path = str(tmp_path / ("piece%d.ckpt" % r))
            g.save(path)
            g.close()
            g = capi.Graph.restore(c, path)
            g.set_part(pc.part)
            f0 = 2 * pc.dag.Q * r
            mine = pick[(pick >= f0) & (pick < f0 + 2 * pc.dag.Q)]
            if len(mine):
                g.set_slots(pc.dag.file_slots[mine - f0], new[mine])
            g.recompute_part(allgather=ag, nranks=nr)
            ok = bool((g.get_slots(np.arange(len(m), dtype=np.uint32)) == want[m]).all())
            g.close()
            return ok
        finally:
            c.close()

    assert all(PC.run_threads(nr, body))


def test_save_refused_with_pending_change(ctx, tmp_path):
    """A slot set but not yet recomputed is a change set the file cannot hold
    (its consumers' queued flags and lists): save refuses with
    RF_EPRECONDITION; after the recompute it saves, and the restored graph
    takes a further change to the oracle's digests."""
    dag = Dag1000(6, 4)
    a = dag.arrays()
    every = np.arange(a["n_slots"], dtype=np.uint32)
    g = _load(ctx, dag)
    g.recompute(full=True)
    sa, _, na = dag.change_set(0.2, seed=5)
    g.set_slots(sa, na)
    path = str(tmp_path / "p.ckpt")
    with pytest.raises(capi.RfError) as e:
        g.save(path)
    assert e.value.code == capi.RF_EPRECONDITION
    assert not os.path.exists(path) and not os.path.exists(path + ".tmp")
    g.recompute(full=False)
    g.save(path)
    g.close()
    r = capi.Graph.restore(ctx, path)
    sb, _, nb = dag.change_set(0.2, seed=6)
    r.set_slots(sb, nb)
    r.recompute(full=False)
    og = O.OGraph(a)
    og.set_inputs(dag.file_slots, dag.leaf_ids)
    og.full()
    og.update(sa, na)
    og.update(sb, nb)
    assert (r.get_slots(every) == og.slots[:a["n_slots"]]).all()
    og.close()
    r.close()


def _sections(raw):
    """(offset, length) of each section of a checkpoint file (graph_io.cpp:
    128-B header, n_sections x {u64 length, bytes}, then the chunk digests,
    the root digest and the end marker)."""
    import struct
    n_sec = struct.unpack_from("<Q", raw, 64)[0]
    out, o = [], 128
    for _ in range(n_sec):
        ln = struct.unpack_from("<Q", raw, o)[0]
        out.append((o + 8, ln))
        o += 8 + ln
    return out, o


def _rechecksum(raw):
    """The same file with every chunk digest and the root recomputed: a
    structurally damaged file whose checksums all match."""
    import hashlib
    import struct
    chunk = 64 << 20
    secs, end = _sections(raw)
    digs = b""
    for o, ln in secs:
        for c in range(0, ln, chunk):
            digs += hashlib.sha256(raw[o + c:o + min(ln, c + chunk)]).digest()
    root = hashlib.sha256(raw[:128] + digs).digest()
    return raw[:end] + struct.pack("<Q", len(digs) // 32) + digs + root + raw[-8:]


def test_structurally_damaged_checkpoints_refused(ctx, tmp_path):
    """Files whose checksums match but whose structure is inconsistent are
    refused before anything reaches a kernel: a reverse edge
    naming a consumer outside its level, the slot-fused flag on an edge that
    is not its input slot's first, and a job numbering that is not a
    permutation.  The untouched file, re-checksummed the same way, restores."""
    import struct
    dag = Dag1000(3, 4)
    g = _load(ctx, dag)
    g.recompute(full=True)
    path = str(tmp_path / "s.ckpt")
    g.save(path)
    g.close()
    raw = open(path, "rb").read()
    secs, _ = _sections(raw)
    names = ["lvl_start", "inc_level", "ext2int", "meta", "holes", "cons_ptr", "cons_job", "tmpl", "slots", "mid"]
    sec = dict(zip(names, secs))
    lvl = np.frombuffer(raw, np.uint32, sec["lvl_start"][1] // 4, sec["lvl_start"][0])
    cons_ptr = np.frombuffer(raw, np.uint32, sec["cons_ptr"][1] // 4, sec["cons_ptr"][0])
    cons = np.frombuffer(raw, np.uint32, sec["cons_job"][1] // 4, sec["cons_job"][0]).reshape(-1, 2)

    def restore(data):
        p = str(tmp_path / "x.ckpt")
        open(p, "wb").write(_rechecksum(data))
        return capi.Graph.restore(ctx, p)

    restore(raw).close()  # the rewriter itself keeps an intact file intact

    def refused(data):
        with pytest.raises(capi.RfError) as e:
            restore(data)
        assert e.value.code == capi.RF_EINTEGRITY, e.value

    # 1. an edge's level word pointing at another level than its consumer's
    e0 = 0
    x, y = int(cons[e0, 0]), int(cons[e0, 1]) & 0x7fffffff
    other = next(lv for lv in range(len(lvl) - 1) if lv != y and not (lvl[lv] <= x < lvl[lv + 1]))
    bad = bytearray(raw)
    struct.pack_into("<I", bad, sec["cons_job"][0] + 8 * e0 + 4, other | (int(cons[e0, 1]) & 0x80000000))
    refused(bytes(bad))
    # 2. the slot-fused flag on an edge that is not the first of its slot's range
    mid_edges = [e for s in range(len(cons_ptr) - 1) for e in range(int(cons_ptr[s]) + 1, int(cons_ptr[s + 1]))]
    assert mid_edges
    e1 = mid_edges[0]
    bad = bytearray(raw)
    struct.pack_into("<I", bad, sec["cons_job"][0] + 8 * e1 + 4, int(cons[e1, 1]) | 0x80000000)
    refused(bytes(bad))
    # 3. two external jobs mapped to one internal id
    bad = bytearray(raw)
    first = struct.unpack_from("<I", bad, sec["ext2int"][0])[0]
    struct.pack_into("<I", bad, sec["ext2int"][0] + 4, first)
    refused(bytes(bad))
    # 4. a fusion target whose one hole sits elsewhere than byte
    # 2, or reads another slot than its producer's output: the chain builds
    # that block 0 in registers from the producer's digest at byte 2
    meta = np.frombuffer(raw, np.uint32, sec["meta"][1] // 4, sec["meta"][0]).reshape(-1, 8)
    j = next(i for i in range(len(meta)) if meta[i, 7] != 0xFFFFFFFF)
    t = int(meta[j, 7])
    hole = int(meta[t, 2])
    assert struct.unpack_from("<II", raw, sec["holes"][0] + 8 * hole) == (2, int(meta[j, 4]))
    bad = bytearray(raw)
    struct.pack_into("<I", bad, sec["holes"][0] + 8 * hole, 40)
    refused(bytes(bad))
    bad = bytearray(raw)
    struct.pack_into("<I", bad, sec["holes"][0] + 8 * hole + 4, int(meta[j, 4]) ^ 1)
    refused(bytes(bad))


def test_older_checkpoint_versions_restore(ctx, tmp_path):
    """ Version-1 checkpoints (round 4) share version 3's layout
    and restore; a version-2 file (round 5) carries four more sections for
    the since-removed flow step (jlv, cout_rng, cout and dstart, sized by the
    header's n_cout), which a restore reads, checks against the checksums and
    drops.  Both then step like the saved graph; an unknown version is
    RF_EINVAL."""
    import struct
    dag = Dag1000(3, 4)
    a = dag.arrays()
    every = np.arange(a["n_slots"], dtype=np.uint32)
    g = _load(ctx, dag)
    g.recompute(full=True)
    path = str(tmp_path / "s.ckpt")
    g.save(path)
    raw = open(path, "rb").read()
    assert struct.unpack_from("<I", raw, 8)[0] == 3
    secs, end = _sections(raw)
    J, L = struct.unpack_from("<I", raw, 16)[0], struct.unpack_from("<I", raw, 24)[0]
    n_cout = 5
    extra = b""
    for ln in (8 * J, 8 * J, 8 * n_cout, 4 * (L + 1)):
        extra += struct.pack("<Q", ln) + bytes((i * 7) & 0xFF for i in range(ln))
    v2 = bytearray(raw[:end] + extra + raw[end:])
    struct.pack_into("<I", v2, 8, 2)
    struct.pack_into("<Q", v2, 64, len(secs) + 4)
    struct.pack_into("<Q", v2, 72, n_cout)
    v1 = bytearray(raw)
    struct.pack_into("<I", v1, 8, 1)
    sl, _, nv = dag.change_set(0.2, seed=9)
    g.set_slots(sl, nv)
    g.recompute(full=False)
    want = g.get_slots(every)
    g.close()
    for name, data in (("v1", v1), ("v2", v2)):
        p = str(tmp_path / (name + ".ckpt"))
        open(p, "wb").write(_rechecksum(bytes(data)))
        r = capi.Graph.restore(ctx, p)
        r.set_slots(sl, nv)
        r.recompute(full=False)
        assert (r.get_slots(every) == want).all(), name
        r.close()
    # a damaged dropped section still fails its checksum
    bad = bytearray(_rechecksum(bytes(v2)))
    bad[end + 8] ^= 1
    p = str(tmp_path / "bad.ckpt")
    open(p, "wb").write(bytes(bad))
    with pytest.raises(capi.RfError) as e:
        capi.Graph.restore(ctx, p)
    assert e.value.code == capi.RF_EINTEGRITY
    v4 = bytearray(raw)
    struct.pack_into("<I", v4, 8, 4)
    open(p, "wb").write(_rechecksum(bytes(v4)))
    with pytest.raises(capi.RfError) as e:
        capi.Graph.restore(ctx, p)
    assert e.value.code == capi.RF_EINVAL


def test_adopt_slots(ctx):
    """rf_graph_adopt_slots (Canonicalize's collapse hand-over, flow.go:814-843):
    a fresh load of the same job table takes a recomputed graph's slot table
    device to device and then steps incrementally exactly like it -- no full
    recompute in between; refused across slot-table sizes, from a graph never
    recomputed, and with a change set pending."""
    dag = Dag1000(12, 6)
    a = dag.arrays()
    every = np.arange(a["n_slots"], dtype=np.uint32)
    src = _load(ctx, dag)
    src.recompute(full=True)
    g = capi.Graph.from_arrays(ctx, a)
    g.adopt_slots(src)
    assert (g.get_slots(every) == src.get_slots(every)).all()
    sl, _, nv = dag.change_set(0.1, seed=3)
    counts = []
    for x in (src, g):
        x.set_slots(sl, nv)
        counts.append(x.recompute(full=False))
    assert counts[0] == counts[1] and 0 < counts[0] < len(a["out_slot"])
    assert (g.get_slots(every) == src.get_slots(every)).all()
    fresh = _load(ctx, dag)
    with pytest.raises(capi.RfError):  # pending change set (the loaded file IDs) and never recomputed
        g.adopt_slots(fresh)
    fresh.recompute(full=True)
    small = Dag1000(4, 6)
    other = _load(ctx, small)
    other.recompute(full=True)
    with pytest.raises(capi.RfError):  # slot tables of different sizes
        g.adopt_slots(other)
    g.set_slots(sl[:1], nv[:1])
    with pytest.raises(capi.RfError):  # a change set pending on the adopter
        g.adopt_slots(fresh)
    for x in (src, g, fresh, other):
        x.close()
