"""The committed golden fixtures (tests/golden/*.json, made by
tests/golden/make_golden.py) against the oracle (CPU) and against the HIP
path through the C-ABI (GPU).

The oracle side re-derives every fixture and pins it to the reference's own
known answers (reference_kats.json); the GPU side must reproduce the same
bytes: bit-exact.
"""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

import reflow_oracle as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import golden_io as G  # noqa: E402
import make_golden as MG  # noqa: E402
from lowering import Lowerer  # noqa: E402

FIXTURES = ["reference_kats.json", "sha256.json", "c1_fileset.json", "filesets.json", "flows.json",
            "murmur3.json", "bloom.json", "fileset_json.json"]


def fileset_groups(v):
    """OFileset -> rf_fileset_digest_batch groups: the material of a List is
    the concatenation of its members' (executor.go:214-233), so a nested
    value flattens into its Map leaves in order."""
    if v.list is not None:
        out = []
        for x in v.list:
            out += fileset_groups(x)
        return out
    return [[(p, fid) for p, (fid, _) in (v.map or {}).items()]]


# --------------------------------------------------------------- CPU side --
def test_fixtures_present():
    for name in FIXTURES:
        assert os.path.exists(G.path(name)), name


def test_reference_kats_reproduced():
    MG.check_reference_kats()
    kats = G.load("reference_kats.json")["kats"]
    assert {k["source"] for k in kats} >= {"flow_test.go:33", "flow_test.go:34", "executor_test.go:77",
                                           "syntax/digest_test.go:25", "values/digest_test.go:28"}


def test_fixtures_regenerate_identically():
    """make_golden.py is deterministic and the committed files are its output."""
    gens = {"sha256.json": MG.gen_sha256, "filesets.json": MG.gen_filesets, "flows.json": MG.gen_flows,
            "fileset_json.json": MG.gen_fileset_json,
            "murmur3.json": MG.gen_murmur3, "bloom.json": MG.gen_bloom}
    for name, fn in gens.items():
        want = json.loads(json.dumps(fn(), sort_keys=True))
        assert want == G.load(name), name


def test_sha256_fixture_oracle():
    d = G.load("sha256.json")
    for c in d["cases"]:
        m = O.fill_stream(d["seed"] ^ c["index"], c["len"])
        assert O.sha256(m).hex() == c["digest"] == hashlib.sha256(m).hexdigest()


def test_c1_fixture_spot_ids_oracle():
    d = G.load("c1_fileset.json")
    for i, h in d["spot_ids"].items():
        assert O.sha256(O.fill_stream(d["seed"] ^ int(i), d["len"])).hex() == h


def test_filesets_fixture_oracle():
    for c in G.load("filesets.json")["cases"]:
        v = G.json_to_fileset(c["value"])
        assert v.material().hex() == c["material"], c["name"]
        assert O.digest_string(v.digest()) == c["digest"], c["name"]


def test_flows_fixture_oracle():
    for c in G.load("flows.json")["cases"]:
        _, nodes = G.json_to_flow(c["flow"])
        U = c["universe"].encode()
        for f, want in zip(nodes, c["nodes"]):
            assert f.digest(U, c["v1"]).hex() == want["digest"], c["name"]
            p = f.physical_digest()
            assert (p.hex() if p else None) == want["physical"], c["name"]
            assert [k.hex() for k in f.cache_keys(U, c["v1"])] == want["cache_keys"], c["name"]


def test_flow_fixture_pins_reference_goldens():
    cases = {c["name"]: c for c in G.load("flows.json")["cases"]}
    v2 = cases["TestDigestStability V2 (flow_test.go:34)"]
    v1 = cases["TestDigestStability V1 (flow_test.go:33)"]
    assert "sha256:" + v2["nodes"][v2["flow"]["root"]]["digest"] == MG.REFERENCE_KATS[0]["digest"]
    assert "sha256:" + v1["nodes"][v1["flow"]["root"]]["digest"] == MG.REFERENCE_KATS[1]["digest"]


def test_murmur3_fixture_oracle():
    d = G.load("murmur3.json")
    for c in d["wd_keys"]:
        h = O.bloom_base_hashes(O.WD(bytes.fromhex(c["digest"])))
        assert ["%016x" % x for x in h] == c["h"]
    for c in d["raw"]:
        assert ["%016x" % x for x in O.mm3_128(bytes.fromhex(c["data"]), c["seed"])] == c["h"]


def _oracle_filter(case):
    m, k = case["m"], case["k"]
    words = np.zeros((m + 63) // 64, dtype=np.uint64)
    length = np.array([m], dtype=np.uint64)
    keys = b"".join(bytes.fromhex(x) for x in case["keys"])
    O.lib().orc_bloomlive_add_batch(words.ctypes.data, length.ctypes.data, m, k, keys, len(case["keys"]))
    return words, int(length[0])


def test_bloom_fixture_oracle():
    for c in G.load("bloom.json")["cases"]:
        words, length = _oracle_filter(c)
        assert length == c["length"]
        assert hashlib.sha256(words.astype("<u8").tobytes()).hexdigest() == c["words_sha256"]
        for key, locs in zip(c["keys"], c["locations_first16"]):
            assert O.bloom_locations(O.WD(bytes.fromhex(key)), c["k"], c["m"]) == locs
        probes = b"".join(bytes.fromhex(x) for x in c["probes"])
        ans = np.zeros(len(c["probes"]), dtype=np.uint8)
        O.lib().orc_bloomlive_contains_batch(words.ctypes.data, length, c["m"], c["k"], probes,
                                             len(c["probes"]), ans.ctypes.data, 1)
        assert ans.tolist() == c["contains"]
        assert all(c["contains"][:len(c["keys"])])  # no false negatives
        js, binary = MG.bloom_wire(c["m"], c["k"], words, length)
        if c["json"] is not None:
            assert js == c["json"]
        assert hashlib.sha256(binary).hexdigest() == c["binary_sha256"]


# --------------------------------------------------------------- GPU side --
@pytest.fixture(scope="module")
def ctx():
    from reflow_amd import capi
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


def _device_set(ctx, seed, lens):
    from reflow_amd.workloads import arena_layout
    lens = np.array(lens, dtype=np.uint64)
    offs, nbytes = arena_layout(lens)
    arena = ctx.alloc(max(nbytes, 256))
    d_offs, d_lens = ctx.upload(offs), ctx.upload(lens)
    ctx.gen_fill(arena.ptr, d_offs.ptr, d_lens.ptr, len(lens), seed, max(nbytes, 256))
    return arena, offs, lens, (d_offs, d_lens)


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_gpu_sha256_fixture(ctx, flags):
    """Device-generated messages (rf_gen_fill = the fixture's stream) through
    every K1 mode: planner default (0), lane messages only (pair kernel),
    wave-per-message only, lanes kernel only."""
    from reflow_amd import capi
    d = G.load("sha256.json")
    lens = [c["len"] for c in d["cases"]]
    arena, offs, lens, keep = _device_set(ctx, d["seed"], lens)
    mode = [0, capi.RF_SHA_NO_SOLO, capi.RF_SHA_ALL_SOLO, capi.RF_SHA_NO_SOLO | capi.RF_SHA_NO_PAIR][flags]
    out = ctx.alloc(32 * len(lens))
    plan = ctx.sha_plan(offs, lens, mode)
    plan.run(arena.ptr, out.ptr)
    ctx.sync()
    got = out.to_numpy().reshape(-1, 32)
    for c, g in zip(d["cases"], got):
        assert g.tobytes().hex() == c["digest"], c["len"]
    plan.close()


@pytest.mark.gpu
def test_gpu_sha256_fixture_host_messages(ctx):
    d = G.load("sha256.json")
    msgs = [O.fill_stream(d["seed"] ^ c["index"], c["len"]) for c in d["cases"]]
    assert [x.hex() for x in ctx.sha256_batch(msgs)] == [c["digest"] for c in d["cases"]]


@pytest.mark.gpu
def test_gpu_c1_fixture(ctx):
    """configs[0] at full size: 4096 x 256 KiB generated in HBM, every File ID
    by K1, then the Fileset digest (a checksum of checksums)."""
    d = G.load("c1_fileset.json")
    arena, offs, lens, keep = _device_set(ctx, d["seed"], [d["len"]] * d["n"])
    out = ctx.alloc(32 * d["n"])
    plan = ctx.sha_plan(offs, lens, 0)
    plan.run(arena.ptr, out.ptr)
    ctx.sync()
    ids = out.to_numpy().reshape(-1, 32)
    plan.close()
    for i, h in d["spot_ids"].items():
        assert ids[int(i)].tobytes().hex() == h
    assert hashlib.sha256(ids.tobytes()).hexdigest() == d["ids_sha256"]
    group = [(MG.c1_path(i), ids[i].tobytes()) for i in range(d["n"])]
    assert O.digest_string(ctx.fileset_digest_batch([[group]])[0]) == d["fileset_digest"]


def test_fileset_json_fixture_oracle_and_capi():
    """json.Marshal bytes: the oracle re-derives them, and the C-ABI's host
    marshaller (no device needed) reproduces them byte for byte."""
    from reflow_amd import capi
    for c in G.load("fileset_json.json")["cases"]:
        v = G.json_to_fs_tree(c["value"])
        assert v.json().hex() == c["json"], c["name"]
        assert capi.fileset_marshal_json(v).hex() == c["json"], c["name"]
        assert O.digest_string(O.sha256(bytes.fromhex(c["json"]))) == c["value_digest"]


@pytest.mark.gpu
def test_gpu_fileset_value_digests_fixture(ctx):
    cases = G.load("fileset_json.json")["cases"]
    got = ctx.fileset_value_digests([G.json_to_fs_tree(c["value"]) for c in cases])
    for c, g in zip(cases, got):
        assert O.digest_string(g) == c["value_digest"], c["name"]


@pytest.mark.gpu
def test_gpu_filesets_fixture(ctx):
    cases = G.load("filesets.json")["cases"]
    sets = [fileset_groups(G.json_to_fileset(c["value"])) for c in cases]
    got = ctx.fileset_digest_batch(sets)
    for c, g in zip(cases, got):
        assert O.digest_string(g) == c["digest"], c["name"]


@pytest.mark.gpu
def test_gpu_flows_fixture(ctx):
    from reflow_amd import capi
    for c in G.load("flows.json")["cases"]:
        _, nodes = G.json_to_flow(c["flow"])
        low = Lowerer(universe=c["universe"].encode())
        slots = [low.lower(f, v1=c["v1"]) for f in nodes]
        pslots = [low.lower_physical(f) for f in nodes]
        a = low.L.arrays()
        g = capi.Graph(ctx, a["n_slots"], a["out_slot"], a["tmpl_off"], a["tmpl_len"], a["hole_ptr"],
                       a["hole_pos"], a["hole_slot"], a["blob"])
        g.recompute(full=True)
        got = g.get_slots(slots)
        for want, d in zip(c["nodes"], got):
            assert d.tobytes().hex() == want["digest"], c["name"]
        for want, ps in zip(c["nodes"], pslots):
            if ps is None:
                assert want["physical"] is None, c["name"]
            else:
                assert g.get_slots([ps])[0].tobytes().hex() == want["physical"], c["name"]
        g.close()


@pytest.mark.gpu
def test_gpu_bloom_fixture(ctx):
    from reflow_amd import capi
    for c in G.load("bloom.json")["cases"]:
        words, length = _oracle_filter(c)
        js, binary = MG.bloom_wire(c["m"], c["k"], words, length)
        probes = np.frombuffer(b"".join(bytes.fromhex(x) for x in c["probes"]), np.uint8)
        for b in (capi.Bloom.from_json(ctx, js.encode()), capi.Bloom.from_binary(ctx, binary),
                  capi.Bloom.load(ctx, c["m"], c["k"], words, length)):
            assert b.probe(probes).tolist() == c["contains"]
            b.close()
        # build side: K4 add over the keys gives the fixture's filter words
        b = capi.Bloom.new(ctx, c["m"], c["k"])
        b.add(np.frombuffer(b"".join(bytes.fromhex(x) for x in c["keys"]), np.uint8))
        assert b.params()[2] == c["length"]
        assert hashlib.sha256(b.words().astype("<u8").tobytes()).hexdigest() == c["words_sha256"]
        b.close()
