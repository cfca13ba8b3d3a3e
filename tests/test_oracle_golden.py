"""Pins the CPU oracle against the reference's own golden vectors.

Every expected digest below is copied from a reference test (file:line cited)
-- these are data (known answers), not reference source.  If the oracle
reproduces them, the byte-level restatement is pinned.
"""
import hashlib
import random

import pytest

import reflow_oracle as O
from reflow_oracle import OFlow, OFileset, WD, from_string

# flow_test.go:33-34
STABLE_V1 = "sha256:5a3a916fe9a11b67f9a0dbd67f6fac0f986dd67803267e79f25f866ca9781e2f"
STABLE_V2 = "sha256:02751e46c573a31747a30b05c2b73b2eb556fb45fb4c0aaf88d170f4b5e6d4e7"
# executor_test.go:77
VLIST = "sha256:d60e67ce9e89548b502a5ad7968e99caed0d388f0a991b906f41a7ba65adb31f"
# syntax/digest_test.go:25
SYNTAX_EXEC = "sha256:ceff79828962397af02d8e2ea30cf6388f2858e0deefbecaa73fad1c6fc88816"
# values/digest_test.go:28
VALUES_MAP = "sha256:c1c3e68de6ccf619538b5810a4feaeac5049505b7719ad67321f62d0c63f52a9"


def stable_flow():
    """The TestDigestStability flow (flow_test.go:24-44), built with the
    test/flow constructors' semantics (test/flow/constructor.go:17-74)."""
    intern = OFlow("OpIntern", url="internurl")
    collect = OFlow("OpCollect", [intern], re=".*", repl="$0")
    groupby = OFlow("OpGroupby", [collect], re="foo-(.*)")
    # Map: MapInit feeds &Flow{Op: OpVal, Value: Fileset{}} (flow.go:315-317)
    val = OFlow("OpVal", value=OFileset(map=None))
    mapflow_exec = OFlow("OpExec", [val], image="image", cmd="command")
    mp = OFlow("OpMap", [groupby], mapflow=mapflow_exec)
    return OFlow("OpExtern", [mp], url="externurl")


def test_stable_v2():
    assert O.digest_string(stable_flow().digest()) == STABLE_V2


def test_stable_v1_after_canonicalize():
    # Canonicalize(Config{HashV1: true}) merges HashV1 into every node,
    # including the re-initialized MapFlow (flow.go:814-843).
    assert O.digest_string(stable_flow().digest(merged=True)) == STABLE_V1


def test_value_digest_vlist():
    file1 = (from_string("foo"), 3)
    file2 = (from_string("bar"), 3)
    file3 = (from_string("a/b/c"), 5)
    v1 = OFileset(map={"foo": file1, "bar": file2})
    v2 = OFileset(map={"a/b/c": file3, "bar": file2})
    vlist = OFileset(list=[v1, v2])
    assert v1.digest() != v2.digest()
    assert O.digest_string(vlist.digest()) == VLIST


def test_syntax_exec_chain():
    intern = OFlow("OpIntern", url="s3://blah")
    c1 = OFlow("OpCoerce", [intern], flow_digest=from_string("file.fs$file"))
    k = OFlow("OpK", [c1], flow_digest=from_string("grail.com/reflow/syntax.Eval.Force"))
    c2 = OFlow("OpCoerce", [k], flow_digest=from_string("grail.com/reflow/syntax.coerceFlowToFileset"))
    ex = OFlow("OpExec", [c2], image="ubuntu", cmd=" cp %s %s ",
               argmap=[(False, 0), (True, 0)])
    c3 = OFlow("OpCoerce", [ex], flow_digest=from_string("grail.com/reflow/syntax.Eval.coerceExecOutput"))
    assert O.digest_string(c3.digest()) == SYNTAX_EXEC


def test_values_map_struct():
    def entry(key, f1, f2):
        return (O.values_string(key),
                O.values_struct({"field1": O.values_int(f1), "field2": O.values_string(f2)}))
    m = O.values_map([entry("hello", 123, "hello world"), entry("world", 321, "foo bar")])
    assert O.digest_string(O.sha256(m)) == VALUES_MAP


def test_wd_is_34_bytes():
    d = from_string("x")
    assert WD(d)[:2] == b"\x00\x05" and len(WD(d)) == 34


def test_opdata_is_maxop():
    # op_string.go:13-21: OpData falls off the end of the stale table.
    assert O.op_digest_string(O.OP["OpData"]) == "maxOp"
    assert O.op_digest_string(O.OP["OpRequirements"]) == "OpRequirements"
    d = OFlow("OpData", data=b"abc")
    assert d.material() == b"maxOpabc"


def test_argmap_neg_zero():
    # Appendix B.5: in(0) and out(0) encode identically.
    a = OFlow("OpExec", image="i", cmd="c", argmap=[(False, 0)])
    b = OFlow("OpExec", image="i", cmd="c", argmap=[(True, 0)])
    assert a.digest() == b.digest()
    c = OFlow("OpExec", image="i", cmd="c", argmap=[(True, 1)])
    assert c.material().endswith(b"\xff" * 8)


def test_universe_twice_for_requirements():
    inner = OFlow("OpIntern", url="u")
    req = OFlow("OpRequirements", [inner])
    assert req.material(b"U") == b"U" + b"U" + b"OpIntern" + b"u"


@pytest.mark.parametrize("n", [0, 1, 3, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 129, 1000, 4096])
def test_sha256_fips_vs_hashlib(n):
    rnd = random.Random(n)
    b = bytes(rnd.getrandbits(8) for _ in range(n))
    assert O.sha256(b) == hashlib.sha256(b).digest()


def test_sha256_fips_known_answers():
    assert O.sha256(b"abc").hex() == \
        "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    assert O.sha256(b"").hex() == \
        "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"


def test_murmur3_smhasher_verification():
    """SMHasher VerificationTest for MurmurHash3_x64_128: hash keys
    {0}, {0,1}, ... {0..254} with seed 256-i, concatenate the 16-byte
    little-endian outputs, hash that with seed 0; the first 4 bytes read
    little-endian must be 0x6384BA69."""
    import struct
    key = bytes(range(256))
    acc = b""
    for i in range(256):
        h1, h2 = O.mm3_128(key[:i], 256 - i)
        acc += struct.pack("<QQ", h1, h2)
    h1, _ = O.mm3_128(acc, 0)
    assert (h1 & 0xFFFFFFFF) == 0x6384BA69


def test_bloom_roundtrip_oracle():
    import numpy as np
    rnd = random.Random(7)
    n = 2000
    m, k = O.estimate_parameters(n, 0.001)
    words = np.zeros((m + 63) // 64, dtype=np.uint64)
    length = np.array([m], dtype=np.uint64)
    keys = bytes(rnd.getrandbits(8) for _ in range(32 * n))
    O.lib().orc_bloomlive_add_batch(words.ctypes.data, length.ctypes.data, m, k, keys, n)
    out = np.zeros(n, dtype=np.uint8)
    O.lib().orc_bloomlive_contains_batch(words.ctypes.data, int(length[0]), m, k, keys, n,
                                         out.ctypes.data, 2)
    assert out.all()  # no false negatives
    fresh = bytes(rnd.getrandbits(8) for _ in range(32 * n))
    O.lib().orc_bloomlive_contains_batch(words.ctypes.data, int(length[0]), m, k, fresh, n,
                                         out.ctypes.data, 2)
    assert out.sum() < n * 0.01  # ~0.1% expected FP rate


def test_estimate_parameters_c5():
    # n = 1e8, p = 0.001
    assert O.estimate_parameters(10**8, 0.001) == (1437758757, 10)


def test_hashv1_is_each_nodes_own_config():
    """flow.go:692-697 reads f.Config.HashV1 of the node being written: a V1
    node inlines a V2 dep's material, and that dep then writes ITS deps as
    WD(digest); a Parent writes with its own config (Canonicalize merges the
    config into copies, never into f.Parent, flow.go:818-843).  Bytes derived
    by hand from the flow.go grammar with hashlib, not the oracle's recursion;
    the same flows are fixture cases (make_golden.mixed_config_flows) that the
    GPU path is checked against in test_golden_fixtures.py."""
    import hashlib
    import struct

    import make_golden as MG

    def H(b):
        return hashlib.sha256(b).digest()

    def WD(d):
        return b"\x00\x05" + d

    cases = {name: (root, u, merged) for name, root, u, merged in MG.mixed_config_flows()}
    c_mat = b"OpIntern" + b"s3://mix"
    b_mat = WD(H(c_mat)) + b"OpCoerce" + WD(H(b"b"))            # V2: dep as WD(digest)
    a_mat = b_mat + b"OpExec" + b"img" + b"cmd" + struct.pack("<q", 0)  # V1: dep inlined
    root, u, merged = cases["HashV1 node over a V2 dep"]
    assert root.digest(u, merged) == H(a_mat)
    root, u, merged = cases["V2 node over a HashV1 dep"]
    assert root.digest(u, merged) == H(WD(H(a_mat)) + b"OpMerge")
    p_mat = WD(H(c_mat)) + b"OpCoerce" + WD(H(b"p"))
    root, u, merged = cases["HashV1 node whose Parent is V2"]
    assert root.digest(u, merged) == H(p_mat)                   # U = "": Parent's own material
    root, u, merged = cases["Canonicalize(HashV1) copy whose Parent is V2, Universe"]
    U = b"U"
    p_mat_u = U + WD(H(U + c_mat)) + b"OpCoerce" + WD(H(b"p"))
    k_mat_u = U + p_mat_u                                       # Parent-forwarded: U written again
    assert merged and root.digest(u, merged) == H(U + k_mat_u + b"OpMerge")  # merged copy inlines its dep
