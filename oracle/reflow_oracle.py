"""CPU restatement (oracle) of Reflow's digest / cache-key / probe path.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module, and only as the checker (or, for the
cpu_baseline, as the timed CPU port).  The product (reflow_amd/, the C-ABI
library) never imports it.

What it restates (reference = LDuderino/reflow @ v0 under /root/reference):
  * digest framing  WD(d) = 0x00 0x05 || d          (grailbio/base/digest, not
    vendored; pinned by the goldens below)
  * Fileset.WriteDigest / Digest                   executor.go:205-233
  * Executor.install over walker.Scan               local/executor.go:514-557, internal/walker/walker.go:33-99
  * json.Marshal(Fileset) -> assoc value digest     executor.go:25-38, eval.go:1961-1967
    (Go 1.9/1.10 encoding/json byte rules; digest JSON text unpinned)
  * Op.DigestString (stale table, OpData->"maxOp")  op_string.go:11-21
  * Flow.WriteDigest / Digest (V1 inline, V2 WD)   flow.go:653-750, writeN :909-913
  * Flow.PhysicalDigest / CacheKeys                flow.go:764-802
  * Canonicalize config merge (HashV1)             flow.go:814-843, 47-50
  * values.WriteDigest (for the values golden)     values/values.go:270-393
  * bloom / murmur3 / SHA-256 arithmetic           oracle.c (via ctypes)

Pinned against the reference's own golden vectors (tests/test_oracle_golden.py):
  flow_test.go:33 (V1), flow_test.go:34 (V2), executor_test.go:77,
  syntax/digest_test.go:25, values/digest_test.go:28.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import struct
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    """Load oracle/liboracle.so (building it with make if absent)."""
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        L = ctypes.CDLL(path)
        u8p = ctypes.c_void_p
        L.orc_sha256.argtypes = [u8p, ctypes.c_uint64, u8p]
        L.orc_sha256_batch.argtypes = [u8p, u8p, u8p, ctypes.c_uint64, u8p, ctypes.c_int]
        # (baseline_openssl.c: the bench's CPU baseline, OpenSSL on native threads)
        L.orc_openssl_sha256_batch.argtypes = [u8p, u8p, u8p, u8p, ctypes.c_uint64, u8p, ctypes.c_int]
        L.orc_openssl_sha256_batch.restype = ctypes.c_int
        L.orc_openssl_sha256_files.argtypes = [u8p, ctypes.c_uint64, u8p, ctypes.c_int]
        L.orc_openssl_sha256_files.restype = ctypes.c_int
        L.orc_fill_stream.argtypes = [ctypes.c_uint64, u8p, ctypes.c_uint64]
        L.orc_mm3_128.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, u8p]
        L.orc_bloom_base_hashes.argtypes = [u8p, ctypes.c_uint64, u8p]
        L.orc_bloom_location.argtypes = [u8p, ctypes.c_uint64]
        L.orc_bloom_location.restype = ctypes.c_uint64
        L.orc_bloom_test.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                     u8p, ctypes.c_uint64]
        L.orc_bloom_test.restype = ctypes.c_int
        L.orc_bloom_add.argtypes = [u8p, u8p, ctypes.c_uint64, ctypes.c_uint64, u8p,
                                    ctypes.c_uint64]
        L.orc_bloomlive_contains_batch.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64,
                                                   ctypes.c_uint64, u8p, ctypes.c_uint64, u8p,
                                                   ctypes.c_int]
        L.orc_bloomlive_add_batch.argtypes = [u8p, u8p, ctypes.c_uint64, ctypes.c_uint64, u8p,
                                              ctypes.c_uint64]
        L.orc_fill_batch.argtypes = [ctypes.c_uint64, u8p, u8p, u8p, ctypes.c_uint64, ctypes.c_int]
        L.orc_stream_sha256.argtypes = [ctypes.c_uint64, ctypes.c_uint64, u8p]
        L.orc_stream_sha256_batch.argtypes = [ctypes.c_uint64, u8p, ctypes.c_uint64, u8p, ctypes.c_int]
        L.orc_graph_new.argtypes = [ctypes.c_uint64, ctypes.c_uint64, u8p, u8p, u8p, u8p, u8p, u8p, u8p]
        L.orc_graph_new.restype = ctypes.c_void_p
        L.orc_graph_free.argtypes = [ctypes.c_void_p]
        L.orc_graph_update.argtypes = [ctypes.c_void_p, u8p, u8p, u8p, ctypes.c_uint64]
        L.orc_graph_update.restype = ctypes.c_uint64
        L.orc_graph_full.argtypes = [ctypes.c_void_p, u8p]
        L.orc_graph_last_blocks.argtypes = [ctypes.c_void_p]
        L.orc_graph_last_blocks.restype = ctypes.c_uint64
        L.orc_graph_eval.argtypes = [ctypes.c_uint64, u8p, u8p, u8p, u8p, u8p, u8p, u8p, u8p, u8p]
        L.orc_graph_check.argtypes = [ctypes.c_uint64, u8p, u8p, u8p, u8p, u8p, u8p, u8p, u8p, ctypes.c_int, u8p]
        L.orc_graph_check.restype = ctypes.c_uint64
        _LIB = L
    return _LIB


class OGraph:
    """The oracle's job graph (orc_graph_*): full and incremental recompute
    over rf_graph_desc-shaped arrays (a dict as Dag1000.arrays() returns)."""

    def __init__(self, a):
        self._a = {k: (np.ascontiguousarray(v) if isinstance(v, np.ndarray) else v) for k, v in a.items()}
        self._blob = np.frombuffer(a["blob"], dtype=np.uint8) if isinstance(a["blob"], (bytes, bytearray)) \
            else np.ascontiguousarray(a["blob"], dtype=np.uint8)
        k = self._a
        self.n_slots = int(k["n_slots"])
        self.slots = np.zeros((max(self.n_slots, 1), 32), dtype=np.uint8)
        hp = np.ascontiguousarray(k["hole_pos"], dtype=np.uint32)
        hs = np.ascontiguousarray(k["hole_slot"], dtype=np.uint32)
        self._keep = (hp, hs)
        self._h = lib().orc_graph_new(len(k["out_slot"]), self.n_slots, k["out_slot"].ctypes.data,
                                      k["tmpl_off"].ctypes.data, k["tmpl_len"].ctypes.data,
                                      k["hole_ptr"].ctypes.data, hp.ctypes.data if len(hp) else None,
                                      hs.ctypes.data if len(hs) else None, self._blob.ctypes.data)

    def set_inputs(self, slots, digests):
        self.slots[np.asarray(slots, dtype=np.int64)] = np.asarray(digests, dtype=np.uint8).reshape(-1, 32)

    def full(self):
        lib().orc_graph_full(self._h, self.slots.ctypes.data)

    def update(self, slots, digests) -> int:
        s = np.ascontiguousarray(slots, dtype=np.uint32)
        d = np.ascontiguousarray(digests, dtype=np.uint8).reshape(-1)
        return int(lib().orc_graph_update(self._h, self.slots.ctypes.data, s.ctypes.data, d.ctypes.data, len(s)))

    def last_blocks(self) -> int:
        return int(lib().orc_graph_last_blocks(self._h))

    def close(self):
        if self._h:
            lib().orc_graph_free(self._h)
            self._h = None

    def __del__(self):
        self.close()


def check_slots(a, slots32, nthreads=1):
    """orc_graph_check: every job of the rf_graph_desc-shaped arrays `a`
    against a whole slot table ([n_slots][32] uint8, e.g. every slot a GPU
    graph holds): (mismatching jobs, lowest such job or None).  Together with
    the input slots' values this is parity with the full evaluation."""
    s = np.ascontiguousarray(slots32, dtype=np.uint8).reshape(-1, 32)
    assert len(s) >= int(a["n_slots"])
    blob = np.frombuffer(a["blob"], dtype=np.uint8) if isinstance(a["blob"], (bytes, bytearray)) \
        else np.ascontiguousarray(a["blob"], dtype=np.uint8)
    arr = {k: np.ascontiguousarray(a[k], dtype=t) for k, t in (
        ("out_slot", np.uint32), ("tmpl_off", np.uint64), ("tmpl_len", np.uint32), ("hole_ptr", np.uint64),
        ("hole_pos", np.uint32), ("hole_slot", np.uint32))}
    first = np.zeros(1, dtype=np.uint64)
    n_jobs = len(arr["out_slot"])
    bad = lib().orc_graph_check(n_jobs, arr["out_slot"].ctypes.data, arr["tmpl_off"].ctypes.data,
                                arr["tmpl_len"].ctypes.data, arr["hole_ptr"].ctypes.data,
                                arr["hole_pos"].ctypes.data if len(arr["hole_pos"]) else None,
                                arr["hole_slot"].ctypes.data if len(arr["hole_slot"]) else None,
                                blob.ctypes.data, s.ctypes.data, int(nthreads), first.ctypes.data)
    return int(bad), (int(first[0]) if bad else None)


def _buf(b: bytes):
    return ctypes.c_char_p(b) if b else ctypes.c_char_p(b"\0")


# --------------------------------------------------------------------------
# SHA-256 and digest framing
# --------------------------------------------------------------------------
def sha256(b: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().orc_sha256(_buf(b), len(b), out)
    return out.raw


def WD(d: bytes) -> bytes:
    """digest.WriteDigest: big-endian uint16(crypto.SHA256 = 5), then the hash."""
    assert len(d) == 32
    return b"\x00\x05" + d


def digest_string(d: bytes) -> str:
    return "sha256:" + d.hex()


def from_string(s: str) -> bytes:
    return sha256(s.encode())


def fill_stream(seed: int, n: int) -> bytes:
    out = ctypes.create_string_buffer(max(n, 1))
    lib().orc_fill_stream(ctypes.c_uint64(seed & (2**64 - 1)), out, n)
    return out.raw[:n]


# --------------------------------------------------------------------------
# Fileset (executor.go:25-38, 205-233)
# --------------------------------------------------------------------------
class OFileset:
    def __init__(self, map=None, list=None):
        self.map = map  # dict path -> (id32, size)
        self.list = list  # list of OFileset or None

    def material(self) -> bytes:
        if self.list is not None:  # List wins when non-nil (executor.go:216-219)
            return b"".join(v.material() for v in self.list)
        out = []
        for path in sorted((self.map or {}).keys(), key=lambda s: s.encode()):
            out.append(path.encode() + WD(self.map[path][0]))
        return b"".join(out)

    def digest(self) -> bytes:
        return sha256(self.material())

    # json.Marshal(Fileset) (executor.go:25-38 struct tags; eval.go:1961-1967
    # marshal -> Repository.Put: the assoc VALUE written under every cache key)
    def json(self) -> bytes:
        parts = []
        if self.list:  # `json:",omitempty"`: nil and empty List both omitted
            parts.append(b'"List":[' + b",".join(v.json() for v in self.list) + b"]")
        if self.map:  # `json:"Fileset,omitempty"`
            items = sorted(((_key_bytes(k), v) for k, v in self.map.items()), key=lambda kv: kv[0])
            ents = []
            for k, (fid, size) in items:
                ents.append(go_json_string(k) + b':{"ID":' + go_json_string(digest_json_text(fid)) +
                            b',"Size":' + str(int(size)).encode() + b"}")
            parts.append(b'"Fileset":{' + b",".join(ents) + b"}")
        return b"{" + b",".join(parts) + b"}"

    def value_digest(self) -> bytes:
        return sha256(self.json())


def install_dir(root):
    """Executor.install (local/executor.go:514-557) over walker.Scan
    (internal/walker/walker.go:33-99): os.Stat follows links and ENOENT skips
    the path (:39-43); directories expand to their bytewise-sorted names,
    prepended to the todo list (:48-55, readDirNames :88-99), so the order is
    depth-first pre-order; every non-directory is Install-ed (ID =
    SHA256(contents), repository/file/repository.go:50-63) with Size = the
    Stat size (executor.go:525) under relpath = filepath.Rel(root, path).
    Returns ([(relpath bytes, id32, size)] in walk order, Fileset digest)."""
    root = os.fsencode(root)
    ents = []
    todo = [(root, b".")]
    while todo:
        path, rel = todo.pop(0)
        try:
            st = os.stat(path)
        except FileNotFoundError:
            continue
        if (st.st_mode & 0o170000) == 0o040000:  # S_ISDIR
            names = sorted(os.listdir(path))
            todo = [(path + b"/" + nm, nm if rel == b"." else rel + b"/" + nm) for nm in names] + todo
            continue
        with open(path, "rb") as f:
            data = f.read()
        ents.append((rel, sha256(data), st.st_size))
    material = b"".join(r + WD(i) for r, i, _ in sorted(ents, key=lambda e: e[0]))
    return ents, sha256(material)


def _key_bytes(k) -> bytes:
    return k if isinstance(k, bytes) else k.encode("utf-8", "surrogateescape")


def digest_json_text(d: bytes) -> bytes:
    """digest.Digest's JSON text (grailbio/base/digest, NOT vendored: parity
    unpinned) -- its String() form "sha256:<64 lowercase hex>"."""
    assert len(d) == 32 and any(d), "zero digests have no pinned text form"
    return b"sha256:" + d.hex().encode()


_HEX = b"0123456789abcdef"


def _utf8_len(s: bytes, i: int) -> int:
    """Length of the valid UTF-8 sequence at s[i] (b >= 0x80), or 0 if invalid:
    unicode/utf8.DecodeRuneInString's acceptance ranges."""
    b0, n = s[i], len(s)

    def cont(j, lo=0x80, hi=0xBF):
        return j < n and lo <= s[j] <= hi
    if 0xC2 <= b0 <= 0xDF:
        return 2 if cont(i + 1) else 0
    if 0xE0 <= b0 <= 0xEF:
        lo, hi = (0xA0, 0xBF) if b0 == 0xE0 else (0x80, 0x9F) if b0 == 0xED else (0x80, 0xBF)
        return 3 if cont(i + 1, lo, hi) and cont(i + 2) else 0
    if 0xF0 <= b0 <= 0xF4:
        lo, hi = (0x90, 0xBF) if b0 == 0xF0 else (0x80, 0x8F) if b0 == 0xF4 else (0x80, 0xBF)
        return 4 if cont(i + 1, lo, hi) and cont(i + 2) and cont(i + 3) else 0
    return 0


def go_json_string(s: bytes) -> bytes:
    """encoding/json encodeState.string(s, escapeHTML=true) as of Go 1.9/1.10
    (.travis.yml:3-5): `"` `\\` -> backslash escapes; \\n \\r \\t short forms;
    other bytes < 0x20 and < > & -> \\u00XX (lowercase hex; Go >= 1.22 writes
    \\b \\f, not used here); invalid UTF-8 -> \\ufffd per bad byte; U+2028/2029 ->
    \\u2028/\\u2029; everything else raw."""
    out = bytearray(b'"')
    i = 0
    while i < len(s):
        b = s[i]
        if b < 0x80:
            if b in (0x22, 0x5C):
                out += bytes([0x5C, b])
            elif b == 0x0A:
                out += b"\\n"
            elif b == 0x0D:
                out += b"\\r"
            elif b == 0x09:
                out += b"\\t"
            elif b < 0x20 or b in (0x3C, 0x3E, 0x26):
                out += b"\\u00" + bytes([_HEX[b >> 4], _HEX[b & 15]])
            else:
                out.append(b)
            i += 1
            continue
        n = _utf8_len(s, i)
        if n == 0:
            out += b"\\ufffd"
            i += 1
            continue
        if s[i:i + n] in (b"\xe2\x80\xa8", b"\xe2\x80\xa9"):
            out += b"\\u202" + bytes([_HEX[s[i + 2] - 0xA0]])
            i += n
            continue
        out += s[i:i + n]
        i += n
    out += b'"'
    return bytes(out)


# --------------------------------------------------------------------------
# Flow (flow.go)
# --------------------------------------------------------------------------
OPS = ["OpExec", "OpIntern", "OpExtern", "OpGroupby", "OpMap", "OpCollect", "OpMerge",
       "OpVal", "OpPullup", "OpK", "OpCoerce", "OpRequirements", "OpData"]
OP = {name: i + 1 for i, name in enumerate(OPS)}
_DIGEST_NAMES = ["OpExec", "OpIntern", "OpExtern", "OpGroupby", "OpMap", "OpCollect",
                 "OpMerge", "OpVal", "OpPullup", "OpK", "OpCoerce", "OpRequirements", "maxOp"]


def op_digest_string(op: int) -> str:
    """op_string.go:15-21: the generated table is one entry stale, so OpData
    digests as "maxOp"."""
    i = op - 1
    if i < 0 or i >= len(_DIGEST_NAMES):
        return "Op(%d)" % op
    return _DIGEST_NAMES[i]


def writeN(n: int) -> bytes:
    return struct.pack("<Q", n & (2**64 - 1))


class OFlow:
    def __init__(self, op, deps=(), **kw):
        self.op = OP[op] if isinstance(op, str) else op
        self.deps = list(deps)
        self.parent = kw.get("parent")
        self.hashv1 = kw.get("hashv1", False)
        self.image = kw.get("image", "")
        self.cmd = kw.get("cmd", "")
        self.url = kw.get("url", "")
        self.re = kw.get("re", "")
        self.repl = kw.get("repl", "")
        self.mapflow = kw.get("mapflow")
        self.argmap = kw.get("argmap")  # None or list of (out: bool, index: int)
        self.flow_digest = kw.get("flow_digest")
        self.value = kw.get("value")  # OFileset or None
        self.done = kw.get("done", False)
        self.data = kw.get("data", b"")
        self.err = kw.get("err", False)

    # Flow.WriteDigest (flow.go:675-750)
    def material(self, universe: bytes = b"", merged=False) -> bytes:
        """Each node's OWN Config.HashV1 decides whether its deps are inlined
        (dep.WriteDigest) or written as WD(dep.Digest()) (flow.go:692-697);
        an inlined dep then follows its own config in turn.  `merged` says
        this node is a Canonicalize copy under Config{HashV1: true}
        (flow.go:820-823: f.Copy() + Config.Merge): its Deps (and OpRequirements'
        dep) are canonical copies merged the same way, and so is its MapFlow
        (MapInit through the canonicalizing MapFunc wrapper, :828-835); its
        Parent is not -- Copy keeps the pointer and canonicalize never visits
        it -- so the Parent writes with its own config (flow.go:680-685)."""
        v1 = self.hashv1 or merged
        w = [universe]
        if self.op == OP["OpRequirements"]:
            return universe + self.deps[0].material(universe, merged)
        if self.parent is not None:
            return universe + self.parent.material(universe, False)
        for d in self.deps:
            w.append(d.material(universe, merged) if v1 else WD(d.digest(universe, merged)))
        w.append(op_digest_string(self.op).encode())
        w.append(self.params(universe, merged))
        return b"".join(w)

    def params(self, universe, merged) -> bytes:
        op = self.op
        if op in (OP["OpIntern"], OP["OpExtern"]):
            return self.url.encode()
        if op == OP["OpExec"]:
            return self.image.encode() + self.cmd.encode() + self.argbytes()
        if op == OP["OpGroupby"]:
            return self.re.encode()
        if op == OP["OpMap"]:
            return self.mapflow.material(universe, merged)
        if op == OP["OpCollect"]:
            return self.re.encode() + self.repl.encode()
        if op == OP["OpVal"]:
            if self.err:
                raise ValueError("error OpVal digests are random (flow.go:722-731)")
            if self.value is not None:
                return self.value.material()
            assert self.flow_digest is not None, "invalid flow digest"
            return WD(self.flow_digest)
        if op in (OP["OpK"], OP["OpCoerce"]):
            assert self.flow_digest is not None, "invalid flow digest"
            return WD(self.flow_digest)
        if op == OP["OpData"]:
            return self.data
        return b""  # OpMerge, OpPullup

    def argbytes(self) -> bytes:
        out = b""
        for is_out, idx in (self.argmap or []):
            out += writeN(-idx if is_out else idx)
        return out

    def digest(self, universe: bytes = b"", merged=False) -> bytes:
        return sha256(self.material(universe, merged))

    # Flow.PhysicalDigest (flow.go:764-792); None == zero digest
    def physical_material(self):
        if self.op not in (OP["OpExtern"], OP["OpExec"]):
            return None
        w = []
        for d in self.deps:
            if not d.done:
                return None
            w.append(d.value.material())
        if self.op == OP["OpExtern"]:
            w.append(self.url.encode())
        else:
            w.append(self.image.encode() + self.cmd.encode() + self.argbytes())
        return b"".join(w)

    def physical_digest(self):
        m = self.physical_material()
        return None if m is None else sha256(m)

    # Flow.CacheKeys (flow.go:796-802)
    def cache_keys(self, universe: bytes = b"", merged=False):
        keys = []
        p = self.physical_digest()
        if p is not None:
            keys.append(p)
        keys.append(self.digest(universe, merged))
        return keys


def eval_dirty(f: OFlow, no_cache_extern: bool, memo=None) -> bool:
    """Eval.dirty (eval.go:874-887), restated: false unless NoCacheExtern; an
    OpExtern is dirty; otherwise dirty iff a Dep is (Deps only -- not MapFlow
    or Parent).  `memo` caches per node (the reference recomputes; the answer
    is the same)."""
    if not no_cache_extern:
        return False
    if memo is None:
        memo = {}
    k = id(f)
    if k not in memo:
        memo[k] = f.op == OP["OpExtern"] or any(eval_dirty(d, True, memo) for d in f.deps)
    return memo[k]


def canonicalize(root: OFlow, hashv1: bool = False, universe: bytes = b""):
    """Flow.Canonicalize (flow.go:814-843) with flowMap.Get/Put (:881-907),
    restated node for node: Get by the ORIGINAL node's digest before recursing,
    copy + Config.Merge, canonicalize the deps (then the map flow, which
    MapInit re-derives through the wrapped MapFunc right after the deps), Put
    by the copy's digest (first Put wins).  Returns {id(original): original
    whose copy is canonical for it}; copies are represented by their originals
    (a copy's digest is its original's under the merged config)."""
    m = {}       # digest -> original whose copy was Put
    out = {}
    memo = {}

    def dig(f, merged):  # Flow.Digest is sync.Once-memoized per node (flow.go:653-664)
        key = (id(f), merged)
        if key not in memo:
            memo[key] = f.digest(universe, merged)
        return memo[key]

    def rec(f):
        hit = m.get(dig(f, False))  # the original node's own digest
        if hit is not None:
            out.setdefault(id(f), hit)
            return hit
        for d in f.deps:
            rec(d)
        if f.mapflow is not None:
            rec(f.mapflow)
        d = dig(f, hashv1)  # the copy's, Config merged
        got = m.setdefault(d, f)
        out.setdefault(id(f), got)
        return got
    rec(root)
    return out


class InmemoryAssoc:
    """test/testutil/assoc.go:16-56 (NewInmemoryAssoc): (kind, key) -> value;
    Put with a nonzero expect is a compare-and-set (errors.Precondition), a
    zero value deletes; Get of a missing key is errors.NotExist.  Abbreviated
    keys follow assoc/dydbassoc/dydbassoc.go:111-147 (ID4 narrowing, then
    Digest.Expands = the full key's hex starts with the abbreviation's)."""
    ZERO = bytes(32)

    def __init__(self):
        self.m = {}

    def put(self, kind, expect, k, v):
        key = (kind, k)
        if expect is not None and expect != self.ZERO and self.m.get(key, self.ZERO) != expect:
            return "precondition"
        if v == self.ZERO:
            self.m.pop(key, None)
        else:
            self.m[key] = v
        return "ok"

    def get(self, kind, k):
        return self.m.get((kind, k))  # None = NotExist

    def get_abbrev(self, kind, prefix_hex: str):
        hits = [(k, v) for (kd, k), v in self.m.items() if kd == kind and k.hex().startswith(prefix_hex)]
        if not hits:
            return "notexist", None
        if len(hits) > 1:
            return "invalid", None  # "more than one key matched"
        return "ok", hits[0]


def assoc_lookup(assoc, kind, node_keys):
    """The Gets of Eval.lookup's key loop for a batch of nodes (eval.go:1202-1209),
    all against the table as it is before the batch: per node (which, value,
    per-key values) with which = the first key that has a value (-1 if none)."""
    res = []
    for keys in node_keys:
        got = [assoc.get(kind, k) for k in keys]
        which = next((j for j, v in enumerate(got) if v is not None), -1)
        res.append((which, got[which] if which >= 0 else bytes(32), got))
    return res


def assoc_repair(assoc, kind, node_keys, which, vals, got=None):
    """Read repair (eval.go:1247-1258) of the nodes with which >= 0, in node
    order: Put(zero expect, key, value) under every other key (blind, the
    reference), or with got (per-key Get results) only under the keys that
    were missing (precise, the TODO at eval.go:1199-1201)."""
    for i, keys in enumerate(node_keys):
        if which[i] < 0:
            continue
        for j, k in enumerate(keys):
            if j != which[i] and (got is None or got[i][j] is None):
                assoc.put(kind, None, k, vals[i])


def eval_lookup(assoc, kind, node_keys, repair=0, usable=None, verified=None):
    """Eval.lookup (eval.go:1172-1258) for a batch of nodes: keys in CacheKeys
    order; a key counts if Get finds a value that `usable(node, fsid)` accepts
    (the unmarshal, :1210-1218 -- otherwise the loop goes on to the next key);
    read repair (1 blind, 2 precise) only for nodes whose value passes
    `verified(node, fsid)` (missing() / RecomputeEmpty, :1227-1246).  Returns
    [(which, fsid)] (-1 and zero when no key counts)."""
    snap = assoc_lookup(assoc, kind, node_keys)
    out, which, vals, got = [], [], [], []
    for i, (_, _, g) in enumerate(snap):
        w = next((j for j, v in enumerate(g) if v is not None and (usable is None or usable(i, v))), -1)
        v = g[w] if w >= 0 else bytes(32)
        out.append((w, v))
        ok = w >= 0 and (verified is None or verified(i, v))
        which.append(w if ok else -1)
        vals.append(v)
        got.append(g)
    if repair:
        assoc_repair(assoc, kind, node_keys, which, vals, got if repair == 2 else None)
    return out


# --------------------------------------------------------------------------
# values.WriteDigest subset (values/values.go:290-393) for the values golden
# --------------------------------------------------------------------------
KIND = {"Int": 2, "String": 3, "Struct": 12, "Map": 9}


def values_int(n: int) -> bytes:
    # big.Int.Bytes(): big-endian magnitude, no leading zeros
    return bytes([KIND["Int"]]) + (n.to_bytes((n.bit_length() + 7) // 8, "big") if n else b"")


def values_string(s: str) -> bytes:
    return bytes([KIND["String"]]) + s.encode()


def values_struct(fields: dict) -> bytes:
    """fields: name -> material; sorted by name, LE64 length prefix."""
    out = bytes([KIND["Struct"]]) + writeN(len(fields))
    for k in sorted(fields, key=lambda s: s.encode()):
        out += fields[k]
    return out


def values_map(entries) -> bytes:
    """entries: list of (key material, value material); sorted by key digest."""
    out = bytes([KIND["Map"]]) + writeN(len(entries))
    for km, vm in sorted(entries, key=lambda e: sha256(e[0])):
        out += km + vm
    return out


# --------------------------------------------------------------------------
# Bloom / murmur3 wrappers
# --------------------------------------------------------------------------
def mm3_128(data: bytes, seed: int = 0):
    out = (ctypes.c_uint64 * 2)()
    lib().orc_mm3_128(_buf(data), len(data), seed, out)
    return out[0], out[1]


def bloom_base_hashes(data: bytes):
    out = (ctypes.c_uint64 * 4)()
    lib().orc_bloom_base_hashes(_buf(data), len(data), out)
    return tuple(out)


def bloom_locations(data: bytes, k: int, m: int):
    h = (ctypes.c_uint64 * 4)(*bloom_base_hashes(data))
    return [lib().orc_bloom_location(h, i) % m for i in range(k)]


def estimate_parameters(n: int, p: float):
    """bloom.go:120-124 (float64 math; filters carry m,k -- never recompute)."""
    import math
    m = int(math.ceil(-1 * float(n) * math.log(p) / math.pow(math.log(2), 2)))
    k = int(math.ceil(math.log(2) * float(m) / float(n)))
    return m, k


def sha256_hashlib(b: bytes) -> bytes:
    """Independent FIPS-180 implementation used to cross-check oracle.c."""
    return hashlib.sha256(b).digest()
