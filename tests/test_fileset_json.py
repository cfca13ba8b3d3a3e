"""Fileset JSON (the assoc value CacheWrite stores, eval.go:1141 -> marshal
eval.go:1961-1967): json.Marshal(Fileset) bytes and their SHA-256.

The reference holds no JSON fixture of a Fileset, so the byte rules are
pinned here by hand-written expectations of Go 1.9/1.10 encoding/json
(struct tags executor.go:25-38, omitempty, sorted map keys, HTML-safe string
escaping) and the oracle and the C-ABI's host marshaller are checked against
them and against each other on random byte strings.  The digest's own JSON
text (grailbio/base/digest, unvendored) is "sha256:<hex>": unpinned.
"""
import random

import pytest

import reflow_oracle as O
from reflow_oracle import OFileset

ID1 = bytes(range(1, 33))
HEX1 = ID1.hex().encode()


# Expected bytes written out by hand from encoding/json's rules.
HAND = [
    (OFileset(), b"{}"),
    (OFileset(list=[], map={}), b"{}"),
    (OFileset(map={"a": (ID1, 7)}), b'{"Fileset":{"a":{"ID":"sha256:' + HEX1 + b'","Size":7}}}'),
    (OFileset(list=[OFileset()]), b'{"List":[{}]}'),
    (OFileset(list=[OFileset()], map={"b": (ID1, -2)}),
     b'{"List":[{}],"Fileset":{"b":{"ID":"sha256:' + HEX1 + b'","Size":-2}}}'),
    (OFileset(map={"b": (ID1, 0), "B": (ID1, 0), "a/b": (ID1, 0)}),
     b'{"Fileset":{"B":{"ID":"sha256:' + HEX1 + b'","Size":0},"a/b":{"ID":"sha256:' + HEX1 +
     b'","Size":0},"b":{"ID":"sha256:' + HEX1 + b'","Size":0}}}'),
]

STRINGS = [
    (b"plain/path.fq", b'"plain/path.fq"'),
    (b'a"b\\c', b'"a\\"b\\\\c"'),
    (b"\n\r\t", b'"\\n\\r\\t"'),
    (b"\x00\x08\x0c\x1f", b'"\\u0000\\u0008\\u000c\\u001f"'),   # Go < 1.22: no \b \f short forms
    (b"<>&", b'"\\u003c\\u003e\\u0026"'),                       # escapeHTML
    (b"\x7f", b'"\x7f"'),                                        # DEL is not escaped
    ("é日\U0001F600".encode(), b'"' + "é日\U0001F600".encode() + b'"'),
    ("  ".encode(), b'"\\u2028\\u2029"'),
    (b"\xff", b'"\\ufffd"'),
    (b"\xe2\x82", b'"\\ufffd\\ufffd"'),                         # truncated: one per byte
    (b"\xed\xa0\x80", b'"\\ufffd\\ufffd\\ufffd"'),              # surrogate half
    (b"\xc0\xaf", b'"\\ufffd\\ufffd"'),                         # overlong
    (b"\xf4\x90\x80\x80", b'"\\ufffd\\ufffd\\ufffd\\ufffd"'),   # > U+10FFFF
    ("�".encode(), b'"\xef\xbf\xbd"'),                 # a real U+FFFD stays raw
]


@pytest.mark.parametrize("v,want", HAND)
def test_oracle_hand_json(v, want):
    assert v.json() == want


@pytest.mark.parametrize("s,want", STRINGS)
def test_oracle_go_string_escaping(s, want):
    assert O.go_json_string(s) == want


@pytest.mark.parametrize("v,want", HAND)
def test_capi_marshal_hand_json(v, want):
    from reflow_amd import capi
    assert capi.fileset_marshal_json(v) == want


@pytest.mark.parametrize("s,want", STRINGS)
def test_capi_marshal_escaping(s, want):
    from reflow_amd import capi
    got = capi.fileset_marshal_json(OFileset(map={s: (ID1, 1)}))
    assert got == b'{"Fileset":{' + want + b':{"ID":"sha256:' + HEX1 + b'","Size":1}}}'


def _random_tree(rng, depth=0):
    def path():
        n = rng.randint(0, 12)
        pool = [rng.randrange(256) for _ in range(n)]
        # bias toward multi-byte sequences and escapes
        if rng.random() < 0.3:
            pool += list(rng.choice(["é", "日", " ", "\U0001F600"]).encode())
        return bytes(pool)
    m = None
    if rng.random() < 0.8:
        m = {}
        for _ in range(rng.randint(0, 6)):
            m[path()] = (bytes(rng.randrange(1, 256) for _ in range(32)), rng.randint(-(1 << 63), (1 << 63) - 1))
    lst = None
    if depth < 3 and rng.random() < 0.4:
        lst = [_random_tree(rng, depth + 1) for _ in range(rng.randint(0, 3))]
    return OFileset(map=m, list=lst)


def test_capi_marshal_matches_oracle_random():
    from reflow_amd import capi
    rng = random.Random(0xB0B)
    for _ in range(300):
        v = _random_tree(rng)
        assert capi.fileset_marshal_json(v) == v.json()


def test_capi_marshal_rejects_duplicates_and_zero_ids():
    from reflow_amd import capi
    with pytest.raises(capi.RfError):
        capi.fileset_marshal_json(OFileset(map={"a": (bytes(32), 1)}))
    b = capi.FilesetTreeBuilder()
    b.paths += [b"x", b"x"]
    b.ids += [ID1, ID1]
    b.sizes += [1, 2]
    b.list_ptr += [None]
    b.entry_ptr += [2]
    b._pending.append((0, []))
    t = b.struct()
    import ctypes
    need = ctypes.c_uint64(0)
    assert capi.lib().rf_fileset_marshal_json(ctypes.byref(t), 0, None, 0, ctypes.byref(need)) == capi.RF_EINVAL


@pytest.mark.gpu
def test_gpu_value_digests_random():
    from reflow_amd import capi
    ctx = capi.Context(0, host_threads=0)
    rng = random.Random(0x7A1)
    sets = [_random_tree(rng) for _ in range(200)]
    # plus a large value: a 20k-file Map (JSON ~2 MB, one long K1 message)
    sets.append(OFileset(map={"d%03d/f%05d.bam" % (i % 97, i): (O.from_string(str(i)), i) for i in range(20000)}))
    got = ctx.fileset_value_digests(sets)
    for v, g in zip(sets, got):
        assert g == O.sha256(v.json())
    ctx.close()
