"""Generates the golden fixtures in tests/golden/ (committed; re-run to
regenerate, the output is deterministic).

    python tests/golden/make_golden.py

Every fixture is computed by the CPU oracle (oracle/), whose byte-level
restatement is pinned by the reference's own known answers (collected in
reference_kats.json and checked first -- generation aborts if any fails).
SHA-256 outputs are cross-checked with hashlib, MurmurHash3 with the SMHasher
verification value.  The fixtures are data: inputs and expected outputs.

  reference_kats.json  known answers quoted from the reference's tests
  sha256.json          seeded messages at padding-edge lengths -> digests
  c1_fileset.json      configs[0] file set (4096 x 256 KiB) -> per-file IDs
                       checksum + Fileset digest (the reference's CPU config)
  filesets.json        Fileset values (Map / List / nested / empty) ->
                       material, digest
  flows.json           flow graphs (every op, V1/V2, Universe) -> digest,
                       physical digest, CacheKeys of every node
  fileset_json.json    Fileset values (nested List + Map, adversarial path
                       bytes) -> json.Marshal bytes, value digest (the assoc
                       value CacheWrite stores; digest JSON text unpinned)
  murmur3.json         murmur3 x64_128 of WD keys and raw strings
  bloom.json           filters (m, k) -> per-key locations, filter words,
                       Contains answers, JSON/binary wire bytes
"""
from __future__ import annotations

import base64
import hashlib
import json
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), HERE]

import numpy as np  # noqa: E402

import reflow_oracle as O  # noqa: E402
from golden_io import fileset_to_json, flow_to_json, topo  # noqa: E402
from reflow_oracle import OFileset, OFlow, from_string  # noqa: E402

# ---------------------------------------------------------------------------
# Known answers quoted from the reference's tests (data, file:line cited).
REFERENCE_KATS = [
    {"source": "flow_test.go:34", "what": "TestDigestStability flow, V2 digest",
     "digest": "sha256:02751e46c573a31747a30b05c2b73b2eb556fb45fb4c0aaf88d170f4b5e6d4e7"},
    {"source": "flow_test.go:33", "what": "TestDigestStability flow after Canonicalize(HashV1)",
     "digest": "sha256:5a3a916fe9a11b67f9a0dbd67f6fac0f986dd67803267e79f25f866ca9781e2f"},
    {"source": "executor_test.go:77", "what": "Fileset{List: [v1, v2]} digest",
     "digest": "sha256:d60e67ce9e89548b502a5ad7968e99caed0d388f0a991b906f41a7ba65adb31f"},
    {"source": "syntax/digest_test.go:25", "what": "Coerce(Exec(Coerce(K(Coerce(Intern)))))",
     "digest": "sha256:ceff79828962397af02d8e2ea30cf6388f2858e0deefbecaa73fad1c6fc88816"},
    {"source": "values/digest_test.go:28", "what": "values.Digest of map[string]struct",
     "digest": "sha256:c1c3e68de6ccf619538b5810a4feaeac5049505b7719ad67321f62d0c63f52a9"},
    {"source": "local/s3_test.go:62-71", "what": "File.ID = Digester.FromString(content) for files a, a/b, d, d/e/f/g, abcdefg",
     "files": {f: O.digest_string(hashlib.sha256(f.encode()).digest())
               for f in ["a", "a/b", "d", "d/e/f/g", "abcdefg"]}},
]


def stable_flow():
    """flow_test.go:24-44 (test/flow/constructor.go:17-74 semantics)."""
    intern = OFlow("OpIntern", url="internurl")
    collect = OFlow("OpCollect", [intern], re=".*", repl="$0")
    groupby = OFlow("OpGroupby", [collect], re="foo-(.*)")
    val = OFlow("OpVal", value=OFileset(map=None))
    mapflow_exec = OFlow("OpExec", [val], image="image", cmd="command")
    mp = OFlow("OpMap", [groupby], mapflow=mapflow_exec)
    return OFlow("OpExtern", [mp], url="externurl")


def syntax_exec_chain():
    """syntax/digest_test.go:14-26."""
    intern = OFlow("OpIntern", url="s3://blah")
    c1 = OFlow("OpCoerce", [intern], flow_digest=from_string("file.fs$file"))
    k = OFlow("OpK", [c1], flow_digest=from_string("grail.com/reflow/syntax.Eval.Force"))
    c2 = OFlow("OpCoerce", [k], flow_digest=from_string("grail.com/reflow/syntax.coerceFlowToFileset"))
    ex = OFlow("OpExec", [c2], image="ubuntu", cmd=" cp %s %s ", argmap=[(False, 0), (True, 0)])
    return OFlow("OpCoerce", [ex], flow_digest=from_string("grail.com/reflow/syntax.Eval.coerceExecOutput"))


def vlist():
    """executor_test.go:62-78."""
    v1 = OFileset(map={"foo": (from_string("foo"), 3), "bar": (from_string("bar"), 3)})
    v2 = OFileset(map={"a/b/c": (from_string("a/b/c"), 5), "bar": (from_string("bar"), 3)})
    return OFileset(list=[v1, v2])


def values_map():
    """values/digest_test.go:14-29."""
    def entry(key, f1, f2):
        return (O.values_string(key),
                O.values_struct({"field1": O.values_int(f1), "field2": O.values_string(f2)}))
    return O.values_map([entry("hello", 123, "hello world"), entry("world", 321, "foo bar")])


def check_reference_kats():
    got = {
        "flow_test.go:34": O.digest_string(stable_flow().digest()),
        "flow_test.go:33": O.digest_string(stable_flow().digest(merged=True)),
        "executor_test.go:77": O.digest_string(vlist().digest()),
        "syntax/digest_test.go:25": O.digest_string(syntax_exec_chain().digest()),
        "values/digest_test.go:28": O.digest_string(O.sha256(values_map())),
    }
    for kat in REFERENCE_KATS:
        if "digest" in kat:
            assert got[kat["source"]] == kat["digest"], (kat["source"], got[kat["source"]])
        else:
            for f, d in kat["files"].items():
                assert O.digest_string(O.sha256(f.encode())) == d
    # SMHasher VerificationTest for MurmurHash3_x64_128
    key = bytes(range(256))
    acc = b""
    for i in range(256):
        h1, h2 = O.mm3_128(key[:i], 256 - i)
        acc += struct.pack("<QQ", h1, h2)
    assert (O.mm3_128(acc, 0)[0] & 0xFFFFFFFF) == 0x6384BA69


# ---------------------------------------------------------------------------
SHA_LENGTHS = [0, 1, 3, 8, 55, 56, 57, 63, 64, 65, 111, 112, 119, 120, 127, 128, 129, 191, 192,
               1000, 4087, 4088, 4095, 4096, 4097, 65527, 65536, 262144, 262151, 1 << 20, (1 << 20) + 55]
SHA_SEED = 0x5EED00F0


def gen_sha256():
    cases = []
    for i, n in enumerate(SHA_LENGTHS):
        m = O.fill_stream(SHA_SEED ^ i, n)
        d = O.sha256(m)
        assert d == hashlib.sha256(m).digest()
        cases.append({"index": i, "len": n, "digest": d.hex()})
    return {"generator": "message i = oracle fill_stream(seed ^ i, len): LE splitmix64 words "
                         "mix64(s + (q+1)*0x9E3779B97F4A7C15), q = word index (oracle/oracle.c orc_fill_stream; "
                         "the device generator rf_gen_fill is the same stream)",
            "seed": SHA_SEED, "cases": cases}


# configs[0]: 4096 x 256 KiB, seed 0x5EED0001 ^ i, paths d%02d/f%04d.fq.gz
C1_N, C1_LEN, C1_SEED = 4096, 262144, 0x5EED0001


def c1_path(i):
    return "d%02d/f%04d.fq.gz" % (i // 64, i)


def gen_c1():
    ids = []
    for i in range(C1_N):
        ids.append(hashlib.sha256(O.fill_stream(C1_SEED ^ i, C1_LEN)).digest())
    # a checksum of the per-file IDs (in file order) and the Fileset digest
    # (executor.go:205-233: sorted paths, path || WD(ID)); one spot ID per 512
    fs = OFileset(map={c1_path(i): (ids[i], C1_LEN) for i in range(C1_N)})
    return {"n": C1_N, "len": C1_LEN, "seed": C1_SEED, "path": "d%02d/f%04d.fq.gz % (i // 64, i)",
            "ids_sha256": hashlib.sha256(b"".join(ids)).hexdigest(),
            "spot_ids": {str(i): ids[i].hex() for i in range(0, C1_N, 512)},
            "fileset_digest": O.digest_string(fs.digest())}


# ---------------------------------------------------------------------------
def gen_filesets():
    rng = random.Random(0xF11E)
    sets = [("vlist executor_test.go:77", vlist()),
            ("empty map", OFileset(map={})), ("nil map", OFileset(map=None)),
            ("empty list", OFileset(list=[])), ("list of empty", OFileset(list=[OFileset(map={})])),
            ("single file '.'", OFileset(map={".": (from_string("x"), 1)})),
            ("list beats map", OFileset(map={"ignored": (from_string("y"), 1)},
                                        list=[OFileset(map={"a": (from_string("a"), 1)})])),
            ("bytewise path order", OFileset(map={"B": (from_string("1"), 1), "a": (from_string("2"), 1),
                                                  "a/b": (from_string("3"), 1), "é": (from_string("4"), 1),
                                                  "A": (from_string("5"), 1)}))]
    for j in range(12):
        groups = []
        for _ in range(rng.randint(1, 3)):
            groups.append(OFileset(map={"p%d/%s%d" % (rng.randint(0, 9), "q" * rng.randint(0, 30), t):
                                        (bytes(rng.getrandbits(8) for _ in range(32)), rng.randint(0, 1 << 40))
                                        for t in range(rng.randint(0, 40))}))
        sets.append(("random %d" % j, groups[0] if len(groups) == 1 else OFileset(list=groups)))
    out = []
    for name, v in sets:
        out.append({"name": name, "value": fileset_to_json(v), "material": v.material().hex(),
                    "digest": O.digest_string(v.digest())})
    return {"cases": out}


def fs_tree_to_json(v: OFileset):
    """Byte-exact form for the JSON fixture: paths as hex (may be invalid UTF-8)."""
    return {"list": None if v.list is None else [fs_tree_to_json(x) for x in v.list],
            "map": None if v.map is None else
            [[O._key_bytes(p).hex(), fid.hex(), size] for p, (fid, size) in v.map.items()]}


# path bytes that exercise every escaping rule of encodeState.string
JSON_PATHS = [b"a", b"", b"dir/file.fq.gz", b'q"uote', b"back\\slash", b"nl\n cr\r tab\t",
              bytes(range(0x00, 0x20)), b"<html>&amp;", b"\x7f del", "é ü 日本".encode(),
              "\u2028\u2029 sep".encode(), b"\xff\xfe bad", b"\xe2\x82 trunc", b"\xed\xa0\x80 surr",
              b"\xf4\x90\x80\x80 >max", b"\xc0\xaf overlong", "\U0001F600 emoji".encode(),
              "\ufffd real".encode(), b"A", b"B", b"a/b"]


def gen_fileset_json():
    rng = random.Random(0x150F)

    def rid():
        return bytes(rng.getrandbits(8) for _ in range(32))
    flat = OFileset(map={p: (rid(), rng.choice([0, 1, -1, 123456789012, -(1 << 63), (1 << 63) - 1]))
                         for p in JSON_PATHS})
    sets = [("empty", OFileset()), ("empty list, empty map", OFileset(list=[], map={})),
            ("escaping + order", flat),
            ("single '.'", OFileset(map={".": (from_string("x"), 1)})),
            ("list and map both", OFileset(list=[OFileset(map={"x": (rid(), 2)})], map={"y": (rid(), 3)})),
            ("nested", OFileset(list=[OFileset(list=[flat, OFileset()]), OFileset(map={"z": (rid(), 0)})])),
            ("vlist executor_test.go:77", vlist())]
    for j in range(8):
        kids = [OFileset(map={"s%d/%s" % (j, "x" * rng.randint(0, 40)) + str(t): (rid(), rng.randint(0, 1 << 40))
                              for t in range(rng.randint(0, 30))}) for _ in range(rng.randint(0, 3))]
        sets.append(("random %d" % j, OFileset(list=kids) if kids and rng.random() < 0.5 else
                     (kids[0] if kids else OFileset(map={}))))
    return {"note": "json.Marshal(Fileset), Go 1.9/1.10 encoding/json; ID text = sha256:<hex> "
                    "(grailbio/base, unvendored: unpinned)",
            "cases": [{"name": n, "value": fs_tree_to_json(v), "json": v.json().hex(),
                       "value_digest": O.digest_string(v.value_digest())} for n, v in sets]}


def flow_case(name, root, universe=b"", v1=False):
    nodes = topo(root)
    per = []
    for f in nodes:
        ck = f.cache_keys(universe, v1)
        p = f.physical_digest()
        per.append({"digest": f.digest(universe, v1).hex(), "physical": p.hex() if p else None,
                    "cache_keys": [k.hex() for k in ck]})
    return {"name": name, "universe": universe.decode(), "v1": v1, "flow": flow_to_json(root), "nodes": per}


def mixed_config_flows():
    """(name, root, universe, merged): flows whose nodes carry different
    HashV1 configs; tests/test_oracle_golden.py pins their bytes by hand."""
    c = OFlow("OpIntern", url="s3://mix")
    b_v2 = OFlow("OpCoerce", [c], flow_digest=from_string("b"))
    a_v1 = OFlow("OpExec", [b_v2], image="img", cmd="cmd", argmap=[(False, 0)], hashv1=True)
    p_v2 = OFlow("OpCoerce", [c], flow_digest=from_string("p"))
    k_v1 = OFlow("OpK", [c], flow_digest=from_string("k"), parent=p_v2, hashv1=True)
    return [("HashV1 node over a V2 dep", a_v1, b"", False),
            ("V2 node over a HashV1 dep", OFlow("OpMerge", [a_v1]), b"", False),
            ("HashV1 node whose Parent is V2", k_v1, b"", False),
            ("Canonicalize(HashV1) copy whose Parent is V2, Universe", OFlow("OpMerge", [k_v1]), b"U", True)]


def gen_flows():
    from flowgen import random_dag
    cases = [flow_case("TestDigestStability V2 (flow_test.go:34)", stable_flow()),
             flow_case("TestDigestStability V1 (flow_test.go:33)", stable_flow(), v1=True),
             flow_case("syntax exec chain (syntax/digest_test.go:25)", syntax_exec_chain()),
             flow_case("syntax exec chain, Universe", syntax_exec_chain(), universe=b"grail/u1")]
    # every op incl. OpData ("maxOp"), OpRequirements (Universe twice), Parent, argmap -0
    inner = OFlow("OpIntern", url="s3://in")
    data = OFlow("OpData", data=b"\x00\x01payload")
    req = OFlow("OpRequirements", [inner])
    par = OFlow("OpCoerce", [inner], flow_digest=from_string("p"))
    child = OFlow("OpMerge", [data], parent=par)
    ex = OFlow("OpExec", [req, child, data], image="img", cmd="c %s %s", argmap=[(False, 0), (True, 0), (True, 2)],
               done=True, value=OFileset(map={".": (from_string("out"), 3)}))
    ext = OFlow("OpExtern", [ex], url="s3://out")
    edge = OFlow("OpMerge", [ext, OFlow("OpPullup", [ex])])
    cases.append(flow_case("edge ops", edge))
    cases.append(flow_case("edge ops, Universe", edge, universe=b"U"))
    # HashV1 is each node's OWN config (flow.go:692-697); Canonicalize merges
    # it into the copies it makes, never into a Parent (flow.go:818-843)
    for name, root, u, merged in mixed_config_flows():
        cases.append(flow_case(name, root, universe=u, v1=merged))
    for seed, u in [(101, b""), (102, b"universe-x"), (103, b"")]:
        root, _ = random_dag(seed, n=40)
        cases.append(flow_case("random_dag seed %d" % seed, root, universe=u))
    return {"cases": cases}


# ---------------------------------------------------------------------------
def gen_murmur3():
    rng = random.Random(0x3A3A)
    wd = []
    for i in range(24):
        d = bytes(rng.getrandbits(8) for _ in range(32)) if i else b"\x00" * 32
        key = O.WD(d)
        h1, h2, h3, h4 = O.bloom_base_hashes(key)
        wd.append({"digest": d.hex(), "h": ["%016x" % x for x in (h1, h2, h3, h4)]})
    raw = []
    for n in list(range(0, 40)) + [64, 100]:
        b = bytes(rng.getrandbits(8) for _ in range(n))
        seed = rng.choice([0, 1, 0x9747B28C])
        h1, h2 = O.mm3_128(b, seed)
        raw.append({"data": b.hex(), "seed": seed, "h": ["%016x" % h1, "%016x" % h2]})
    return {"wd_keys": wd, "raw": raw, "smhasher_verification": "0x6384BA69"}


def bloom_wire(m, k, words, length):
    """bloom.go:263-286 / bitset.go:693-721: compact JSON {"m":M,"k":K,"b":"<base64url of
    BE64 length || BE64 words>"} (BitSet.MarshalJSON uses base64.URLEncoding), and binary
    BE64 m || BE64 k || BE64 length || BE64 words (bloom.go:288-325, bitset.go:628-691)."""
    bits = struct.pack(">Q", length) + b"".join(struct.pack(">Q", int(w)) for w in words)
    js = json.dumps({"m": m, "k": k, "b": base64.urlsafe_b64encode(bits).decode()},
                    separators=(",", ":"))
    binary = struct.pack(">QQ", m, k) + bits
    return js, binary


def gen_bloom():
    rng = random.Random(0xB100)
    L = O.lib()
    out = []
    for n, p in [(1, 0.5), (64, 0.01), (500, 0.001), (200, 1e-6)]:
        m, k = O.estimate_parameters(n, p)
        keys = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(n)]
        words = np.zeros((m + 63) // 64, dtype=np.uint64)
        length = np.array([m], dtype=np.uint64)
        kb = b"".join(keys)
        L.orc_bloomlive_add_batch(words.ctypes.data, length.ctypes.data, m, k, kb, n)
        probes = keys + [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(max(n, 50))]
        pb = b"".join(probes)
        ans = np.zeros(len(probes), dtype=np.uint8)
        L.orc_bloomlive_contains_batch(words.ctypes.data, int(length[0]), m, k, pb, len(probes),
                                       ans.ctypes.data, 1)
        locs = [O.bloom_locations(O.WD(x), k, m) for x in keys[:16]]
        js, binary = bloom_wire(m, k, words, int(length[0]))
        out.append({"n": n, "p": p, "m": m, "k": k, "keys": [x.hex() for x in keys],
                    "locations_first16": locs, "length": int(length[0]),
                    "words_sha256": hashlib.sha256(words.astype("<u8").tobytes()).hexdigest(),
                    "probes": [x.hex() for x in probes], "contains": ans.tolist(),
                    "json": js if m <= 8192 else None, "binary_sha256": hashlib.sha256(binary).hexdigest()})
    return {"key": "WD(d) = 00 05 || d (34 B), eval.go:851 / bloomlive.go:32", "cases": out}


def write(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", name, os.path.getsize(os.path.join(HERE, name)), "bytes")


def main():
    O.lib()
    check_reference_kats()
    write("reference_kats.json", {"kats": REFERENCE_KATS})
    write("sha256.json", gen_sha256())
    write("c1_fileset.json", gen_c1())
    write("filesets.json", gen_filesets())
    write("flows.json", gen_flows())
    write("fileset_json.json", gen_fileset_json())
    write("murmur3.json", gen_murmur3())
    write("bloom.json", gen_bloom())


if __name__ == "__main__":
    main()
