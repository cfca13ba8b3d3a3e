"""Synthetic workloads of BASELINE.json's configs.

  c2_sizes     64 GiB FASTQ/BAM-like Fileset: 98% of files log-uniform in
               [4 KiB, 1 MiB], 2% log-uniform in [64 MiB, 2 GiB] (seed 0x5EED0002)
  Dag1000      1000align-shaped Flow DAG (doc/1000align/1000align.rf:36-47,
               align.rf:54-97, bam.rf:12-42) lowered straight to rf_graph jobs,
               vectorised so 10M-100M nodes build in seconds; 1% of leaf
               File IDs change per step (seed 0x5EED0003): new = SHA256(old||"v2")
  c5_keys      probe keys for the bloomlive filter (seed 0x5EED0005)

The digest grammar is SURVEY App. A (flow.go:675-792).  Dag1000.oflow()
builds the same graph as oracle flows for small S so tests can check the
vectorised lowering against the oracle.
"""
from __future__ import annotations

import hashlib
import math
import struct

import numpy as np

KiB, MiB, GiB = 1 << 10, 1 << 20, 1 << 30


# --------------------------------------------------------------------- C2 --
def c2_sizes(total_bytes=64 * GiB, seed=0x5EED0002, small=(4 * KiB, 1 * MiB),
             big=(64 * MiB, 2 * GiB), big_frac=0.02):
    """File sizes until their sum reaches total_bytes (last file trimmed)."""
    rng = np.random.default_rng(seed)
    out, acc = [], 0
    while acc < total_bytes:
        lo, hi = big if rng.random() < big_frac else small
        n = int(math.exp(rng.uniform(math.log(lo), math.log(hi))))
        n = min(n, total_bytes - acc)
        out.append(n)
        acc += n
    return np.array(out, dtype=np.uint64)


def arena_layout(lens, align=256):
    """Offsets of messages packed at `align`-byte boundaries; total bytes."""
    lens = np.asarray(lens, dtype=np.uint64)
    padded = (lens + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    offs = np.zeros(len(lens), dtype=np.uint64)
    if len(lens) > 1:
        offs[1:] = np.cumsum(padded[:-1])
    total = int(padded.sum()) if len(lens) else 16
    return offs, max(total, 16)


# --------------------------------------------------------------------- C5 --
def c5_keys(n, seed=0x5EED0005):
    return np.random.default_rng(seed).integers(0, 256, size=(n, 32), dtype=np.uint8)


# --------------------------------------------------------------------- C3 --
def _h(s: bytes) -> bytes:
    return hashlib.sha256(s).digest()


def _le64(n: int) -> bytes:
    return struct.pack("<q", n)


WD0 = b"\x00\x05" + b"\0" * 32  # WD prefix + hole placeholder

FD_COERCE_FILE = _h(b"file.fs$file")
FD_FORCE = _h(b"grail.com/reflow/syntax.Eval.Force")
FD_TO_FILESET = _h(b"grail.com/reflow/syntax.coerceFlowToFileset")
FD_EXEC_OUT = _h(b"grail.com/reflow/syntax.Eval.coerceExecOutput")
FD_MERGE = _h(b"grail.com/reflow/syntax.Eval.Force.merge")
BWA = b"biocontainers/bwa"
SAMTOOLS = b"biocontainers/samtools"
REF_URL = b"s3://1000genomes/technical/reference/human_g1k_v37.fasta.gz"
INDEX_CMD = (b"\n\tgunzip -c %s > %s/g1k_v37.fa || true\n\tcd %s\n\tbwa index -a bwtsw g1k_v37.fa\n")
INDEX_FILES = [b"g1k_v37.fa", b"g1k_v37.fa.amb", b"g1k_v37.fa.ann", b"g1k_v37.fa.bwt",
               b"g1k_v37.fa.pac", b"g1k_v37.fa.sa"]


def _argmap(n_in):
    """in(0..n_in-1), out(0): writeN(index) / writeN(-index) (flow.go:707-712)."""
    return b"".join(_le64(i) for i in range(n_in)) + _le64(-0)


def _digits(a: np.ndarray, width: int) -> np.ndarray:
    """[n, width] ASCII decimal digits of a (zero padded)."""
    a = np.asarray(a, dtype=np.int64)
    out = np.empty((len(a), width), dtype=np.uint8)
    x = a.copy()
    for j in range(width - 1, -1, -1):
        out[:, j] = 48 + (x % 10)
        x //= 10
    return out


_GOLD = np.uint64(0x9E3779B97F4A7C15)


def _mix64(z):
    """splitmix64's finaliser over a uint64 array (wrapping arithmetic)."""
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _ids_vec(domain: bytes, seed: int, idx) -> np.ndarray:
    """[n, 32] uint8: four splitmix64 outputs per global index, keyed by
    SHA256(domain || seed)."""
    key = np.uint64(int.from_bytes(_h(domain + b":%d" % seed)[:8], "little"))
    idx = np.asarray(idx, dtype=np.int64).astype(np.uint64)
    with np.errstate(over="ignore"):
        base = key + idx * np.uint64(4) * _GOLD
        out = np.empty((len(idx), 4), dtype=np.uint64)
        for k in range(4):
            out[:, k] = _mix64(base + np.uint64(k + 1) * _GOLD)
    return out.view(np.uint8).reshape(len(idx), 32)


class _Kind:
    """One node kind: a template of fixed length, per-instance digit fields,
    per-instance literal byte fields and holes."""

    def __init__(self, name, tmpl: bytes, count: int):
        self.name, self.tmpl, self.count = name, tmpl, count
        self.digit_fields = []   # (pos, width, values[count])
        self.byte_fields = []    # (pos, values[count, k])
        self.holes = []          # (pos, slot[count])
        self.out_slot = None

    def digits(self, pos, width, values):
        self.digit_fields.append((pos, width, np.asarray(values)))

    def bytes_at(self, pos, values):
        self.byte_fields.append((pos, np.asarray(values, dtype=np.uint8)))

    def hole(self, pos, slots):
        self.holes.append((pos, np.asarray(slots, dtype=np.uint32)))


def _kind_blocks(kk):
    """Blocks an incremental recompute of one job of kind kk must hash: its
    padded material's, less the constant leading blocks before its first hole
    (hashed once at load, the midstate)."""
    nb = (len(kk.tmpl) + 9 + 63) // 64
    return nb - (min(p for p, _ in kk.holes) // 64 if kk.holes else 0)


class Dag1000:
    """1000align-shaped DAG: S samples x P read pairs (~S*(14P+5) nodes).

    Per pair: V1,V2 = Val(Fileset{".": File}) leaves (File IDs are input slots)
      C1,C2 = Coerce ; E1 = Exec(bwa mem, [R2,C1,C2]) ; C3 ; K1 ; C4 ;
      E2 = Exec(samtools view) ; C5 ; K2 ; C6 ; E3 = Exec(samtools sort) ; C7
    Per sample: KS = K(C7 x P) (wide fan-in) ; CS1 ; ES = Exec(merge) ; CS2 ;
      XS = Extern(s3://out/...)
    Shared: R0 = Intern(ref) ; R1 = Exec(bwa index) ; R2 = Coerce
    Physical keys (flow.go:764-792) for every Exec/Extern whose deps are done.
    """

    PAIR_KINDS = ["V1", "V2", "C1", "C2", "E1", "C3", "K1", "C4", "E2", "C5", "K2", "C6", "E3", "C7"]
    SAMPLE_KINDS = ["KS", "CS1", "ES", "CS2", "XS"]

    def __init__(self, S: int, P: int = 32, seed=0x5EED0003, sample0=0):
        """sample0: global index of this DAG's first sample -- Dag1000(S,
        sample0=r*S) is samples [r*S, (r+1)*S) of the global Dag1000 with the
        same seed, node for node (rank r's piece of a partitioned DAG)."""
        self.S, self.P, self.seed, self.sample0 = S, P, seed, sample0
        self.Q = S * P
        self.n_nodes = 3 + self.Q * 14 + S * 5
        self._build()

    # deterministic "previous run" values: 32 bytes per (domain, seed, global
    # index) from a keyed splitmix64 stream, vectorised (hashlib per node took
    # ~35 s of Python at 100M nodes); any fixed values serve, what matters is
    # that a rank's piece and the global DAG agree (global indices)
    def file_id(self, i):  # File ID of leaf file i (2 per pair)
        return _ids_vec(b"file", self.seed, np.array([i + 2 * self.P * self.sample0]))[0].tobytes()

    def out_id(self, tag, i):  # output File ID of exec instance i (per pair; "es" per sample)
        return self._out_ids(tag, np.array([i]))[0].tobytes()

    def _out_ids(self, tag, idx):
        off = self.sample0 if tag == b"es" else self.P * self.sample0
        return _ids_vec(b"out:" + tag, self.seed, np.asarray(idx, dtype=np.int64) + off)

    def _build(self):
        S, P, Q = self.S, self.P, self.Q
        kinds = {}
        # slots: [file slots 2Q][logical slots per kind][physical slots]
        next_slot = [2 * Q]

        def alloc(n):
            b = next_slot[0]
            next_slot[0] += n
            return np.arange(b, b + n, dtype=np.uint32)

        q = np.arange(Q)
        s_of_q = q // P + self.sample0
        p_of_q = q % P
        sidx = np.arange(S) + self.sample0

        # shared
        k = _Kind("R0", b"OpIntern" + REF_URL, 1)
        k.out_slot = alloc(1)
        kinds["R0"] = k
        idx_cmd = INDEX_CMD % (b"%s", b"%s", b"%s")
        k = _Kind("R1", WD0 + b"OpExec" + BWA + idx_cmd + _argmap(1), 1)
        k.hole(2, kinds["R0"].out_slot)
        k.out_slot = alloc(1)
        kinds["R1"] = k
        k = _Kind("R2", WD0 + b"OpCoerce" + b"\x00\x05" + FD_EXEC_OUT, 1)
        k.hole(2, kinds["R1"].out_slot)
        k.out_slot = alloc(1)
        kinds["R2"] = k

        def coerce(name, dep_slots, fd, count):
            kk = _Kind(name, WD0 + b"OpCoerce" + b"\x00\x05" + fd, count)
            kk.hole(2, dep_slots)
            kk.out_slot = alloc(count)
            kinds[name] = kk
            return kk

        def kcont(name, dep_slots, fd, count):
            kk = _Kind(name, WD0 + b"OpK" + b"\x00\x05" + fd, count)
            kk.hole(2, dep_slots)
            kk.out_slot = alloc(count)
            kinds[name] = kk
            return kk

        # leaves: material "OpVal" + "." + WD(file id)
        for j, name in enumerate(["V1", "V2"]):
            kk = _Kind(name, b"OpVal" + b"." + WD0, Q)
            kk.hole(8, 2 * q + j)
            kk.out_slot = alloc(Q)
            kinds[name] = kk
        coerce("C1", kinds["V1"].out_slot, FD_COERCE_FILE, Q)
        coerce("C2", kinds["V2"].out_slot, FD_COERCE_FILE, Q)
        # E1: bwa mem, deps [R2, C1, C2]
        cmd1 = (b'\n\t\tbwa mem -R "@RG\\tID:S0000000_P000\\tSM:S0000000" -t 32 \\\n'
                b'\t\t\t%s/g1k_v37.fa %s %s > %s\n\t')
        pre = 3 * 34 + len(b"OpExec") + len(BWA)
        k = _Kind("E1", WD0 * 3 + b"OpExec" + BWA + cmd1 + _argmap(3), Q)
        k.hole(2, np.repeat(kinds["R2"].out_slot, Q))
        k.hole(36, kinds["C1"].out_slot)
        k.hole(70, kinds["C2"].out_slot)
        c = cmd1.index(b"S0000000_P000")
        k.digits(pre + c + 1, 7, s_of_q)
        k.digits(pre + c + 10, 3, p_of_q)
        c2 = cmd1.index(b"SM:S0000000")
        k.digits(pre + c2 + 4, 7, s_of_q)
        k.out_slot = alloc(Q)
        kinds["E1"] = k
        coerce("C3", kinds["E1"].out_slot, FD_EXEC_OUT, Q)
        kcont("K1", kinds["C3"].out_slot, FD_FORCE, Q)
        coerce("C4", kinds["K1"].out_slot, FD_TO_FILESET, Q)
        cmd2 = b"\n\t\t< %s samtools view -Sb - > %s # S0000000_P000\n\t"
        pre2 = 34 + len(b"OpExec") + len(SAMTOOLS)
        k = _Kind("E2", WD0 + b"OpExec" + SAMTOOLS + cmd2 + _argmap(1), Q)
        k.hole(2, kinds["C4"].out_slot)
        c = cmd2.index(b"S0000000_P000")
        k.digits(pre2 + c + 1, 7, s_of_q)
        k.digits(pre2 + c + 10, 3, p_of_q)
        k.out_slot = alloc(Q)
        kinds["E2"] = k
        coerce("C5", kinds["E2"].out_slot, FD_EXEC_OUT, Q)
        kcont("K2", kinds["C5"].out_slot, FD_FORCE, Q)
        coerce("C6", kinds["K2"].out_slot, FD_TO_FILESET, Q)
        cmd3 = b"\n\t\tsamtools sort --threads 64 -o %s %s # S0000000_P000\n\t"
        k = _Kind("E3", WD0 + b"OpExec" + SAMTOOLS + cmd3 + _argmap(1), Q)
        k.hole(2, kinds["C6"].out_slot)
        c = cmd3.index(b"S0000000_P000")
        k.digits(pre2 + c + 1, 7, s_of_q)
        k.digits(pre2 + c + 10, 3, p_of_q)
        k.out_slot = alloc(Q)
        kinds["E3"] = k
        coerce("C7", kinds["E3"].out_slot, FD_EXEC_OUT, Q)
        # per sample: wide K over the P sorted BAMs
        k = _Kind("KS", WD0 * P + b"OpK" + b"\x00\x05" + FD_MERGE, S)
        c7 = kinds["C7"].out_slot.reshape(S, P)
        for j in range(P):
            k.hole(34 * j + 2, c7[:, j])
        k.out_slot = alloc(S)
        kinds["KS"] = k
        coerce("CS1", kinds["KS"].out_slot, FD_TO_FILESET, S)
        cmdm = b"\n\t\tsamtools merge -@64 %s %s # S0000000\n\t"
        k = _Kind("ES", WD0 + b"OpExec" + SAMTOOLS + cmdm + _argmap(1), S)
        k.hole(2, kinds["CS1"].out_slot)
        k.digits(pre2 + cmdm.index(b"S0000000") + 1, 7, sidx)
        k.out_slot = alloc(S)
        kinds["ES"] = k
        coerce("CS2", kinds["ES"].out_slot, FD_EXEC_OUT, S)
        url = b"s3://1000genomes-out/S0000000.bam"
        k = _Kind("XS", WD0 + b"OpExtern" + url, S)
        k.hole(2, kinds["CS2"].out_slot)
        k.digits(34 + len(b"OpExtern") + url.index(b"S0000000") + 1, 7, sidx)
        k.out_slot = alloc(S)
        kinds["XS"] = k
        self.n_logical_slots = next_slot[0] - 2 * Q

        # ---- physical keys: concat FM(dep values) || suffix ------------------
        # values: R0 -> {".": ref}; R1/R2 -> index dir; V*/C1/C2 -> {".": file};
        # E1..C7 outputs -> {".": out}; KS/CS1 -> list of P bams; ES/CS2 -> {".": merged}
        self.ref_id = _h(b"ref:%d" % self.seed)
        self.index_ids = [_h(b"index:%d:%s" % (self.seed, f)) for f in INDEX_FILES]
        fm_index = b"".join(f + b"\x00\x05" + i for f, i in zip(INDEX_FILES, self.index_ids))
        fm_dot = lambda: b"." + WD0  # noqa: E731  ("." + WD(hole/literal))

        k = _Kind("pR1", b"." + b"\x00\x05" + self.ref_id + BWA + idx_cmd + _argmap(1), 1)
        k.out_slot = alloc(1)
        kinds["pR1"] = k
        # E1: FM(R2 value = index dir) + FM(C1 value) + FM(C2 value) + suffix
        e1_suffix = kinds["E1"].tmpl[3 * 34 + len(b"OpExec"):]
        k = _Kind("pE1", fm_index + fm_dot() + fm_dot() + e1_suffix, Q)
        k.hole(len(fm_index) + 3, 2 * q)
        k.hole(len(fm_index) + 35 + 3, 2 * q + 1)
        for pos, width, vals in kinds["E1"].digit_fields:
            k.digits(pos - 3 * 34 - len(b"OpExec") + len(fm_index) + 70, width, vals)
        k.out_slot = alloc(Q)
        kinds["pE1"] = k
        # E2: dep C4's value = E1's output {".": out_e1}; E3: C6 -> out_e2
        for name, src, tag in [("pE2", "E2", b"e1"), ("pE3", "E3", b"e2")]:
            suffix = kinds[src].tmpl[34 + len(b"OpExec"):]
            kk = _Kind(name, b"." + b"\x00\x05" + b"\0" * 32 + suffix, Q)
            kk.bytes_at(3, self._out_ids(tag, np.arange(Q)))
            for pos, width, vals in kinds[src].digit_fields:
                kk.digits(pos - 34 - len(b"OpExec") + 35, width, vals)
            kk.out_slot = alloc(Q)
            kinds[name] = kk
        # ES: dep CS1's value = list of P sorted bams (paths "." each)
        suffix = kinds["ES"].tmpl[34 + len(b"OpExec"):]
        kk = _Kind("pES", (b"." + b"\x00\x05" + b"\0" * 32) * P + suffix, S)
        bam_ids = self._out_ids(b"e3", np.arange(Q)).reshape(S, P, 32)
        for j in range(P):
            kk.bytes_at(35 * j + 3, bam_ids[:, j, :])
        for pos, width, vals in kinds["ES"].digit_fields:
            kk.digits(pos - 34 - len(b"OpExec") + 35 * P, width, vals)
        kk.out_slot = alloc(S)
        kinds["pES"] = kk
        # XS extern: dep CS2 value = {".": merged} + URL
        kk = _Kind("pXS", b"." + b"\x00\x05" + b"\0" * 32 + url, S)
        kk.bytes_at(3, self._out_ids(b"es", np.arange(S)))
        kk.digits(35 + url.index(b"S0000000") + 1, 7, sidx)
        kk.out_slot = alloc(S)
        kinds["pXS"] = kk

        self.kinds = kinds
        self.n_slots = next_slot[0]
        self.n_jobs = sum(kk.count for kk in kinds.values())
        self.file_slots = np.arange(2 * Q, dtype=np.uint32)
        self.leaf_ids = _ids_vec(b"file", self.seed, np.arange(2 * Q, dtype=np.int64) + 2 * P * self.sample0)

    # -------------------------------------------------------------- lowering
    def arrays(self):
        """rf_graph_desc arrays (out_slot, tmpl_off, tmpl_len, hole_ptr,
        hole_pos, hole_slot, blob).  The blob is allocated once and each
        kind's rows are written into their view on a thread of their own
        (numpy releases the GIL for the copies): ~15 GB at 100M nodes."""
        from concurrent.futures import ThreadPoolExecutor
        kinds = list(self.kinds.values())
        L16 = [(len(kk.tmpl) + 15) // 16 * 16 for kk in kinds]
        sizes = [kk.count * l16 for kk, l16 in zip(kinds, L16)]
        bases = np.concatenate([[0], np.cumsum(sizes, dtype=np.int64)]).astype(np.int64)
        blob = np.empty(int(bases[-1]), dtype=np.uint8)

        def fill(x):
            kk, l16, b = kinds[x], L16[x], int(bases[x])
            L = len(kk.tmpl)
            arr = blob[b:b + kk.count * l16].reshape(kk.count, l16)
            arr[:, :L] = np.frombuffer(kk.tmpl, dtype=np.uint8)
            arr[:, L:] = 0
            for pos, width, vals in kk.digit_fields:
                arr[:, pos:pos + width] = _digits(vals, width)
            for pos, vals in kk.byte_fields:
                arr[:, pos:pos + vals.shape[1]] = vals

        with ThreadPoolExecutor(min(8, len(kinds))) as ex:
            list(ex.map(fill, range(len(kinds))))
        out_slot = np.concatenate([kk.out_slot for kk in kinds]).astype(np.uint32)
        off = np.concatenate([bases[x] + np.arange(kk.count, dtype=np.int64) * L16[x]
                              for x, kk in enumerate(kinds)]).astype(np.uint64)
        ln = np.concatenate([np.full(kk.count, len(kk.tmpl), dtype=np.uint32) for kk in kinds])
        nh = np.concatenate([np.full(kk.count, len(kk.holes), dtype=np.uint64) for kk in kinds])
        hpos = [np.tile(np.array([p for p, _ in kk.holes], dtype=np.uint32), kk.count) for kk in kinds if kk.holes]
        hslot = [np.stack([sl for _, sl in kk.holes], axis=1).reshape(-1).astype(np.uint32)
                 for kk in kinds if kk.holes]
        hole_ptr = np.zeros(self.n_jobs + 1, dtype=np.uint64)
        hole_ptr[1:] = np.cumsum(nh)
        return dict(n_slots=self.n_slots, out_slot=out_slot, tmpl_off=off, tmpl_len=ln, hole_ptr=hole_ptr,
                    hole_pos=np.concatenate(hpos), hole_slot=np.concatenate(hslot), blob=blob)

    def critical_path(self, file_slots):
        """The longest chain of dependent compressions a change of leaf-file
        slots `file_slots` starts: Val -> Coerce -> the pair's ten-job chain
        (E1 .. C7) -> the sample's tail (KS .. XS), in blocks (0 if nothing
        changed).  Every dirty pair's chain has this shape, so the maximum is
        over the two leaf parities present."""
        f = np.asarray(file_slots, dtype=np.int64)
        if not len(f):
            return 0
        b = {k: _kind_blocks(kk) for k, kk in self.kinds.items()}
        lead = max([b["V1"] + b["C1"]] * bool((f % 2 == 0).any()) + [b["V2"] + b["C2"]] * bool((f % 2).any()))
        chain = ("E1", "C3", "K1", "C4", "E2", "C5", "K2", "C6", "E3", "C7")
        return lead + sum(b[k] for k in chain) + sum(b[k] for k in self.SAMPLE_KINDS)

    def change_set(self, frac=0.01, seed=0x5EED0003, n_global=None):
        """File slots to change (1% of leaf files) and their two versions:
        v_old = current IDs, v_new = SHA256(old || "v2").  n_global: this DAG
        is the slice (sample0) of a global DAG with n_global leaf files -- the
        change set is the global one's, restricted to this slice (so every
        partition of one global DAG changes the same files)."""
        nf = len(self.file_slots)
        f0 = 2 * self.P * self.sample0 if n_global is not None else 0
        n_all = nf if n_global is None else n_global
        rng = np.random.default_rng(seed)
        n = max(1, int(round(frac * n_all)))
        pick = np.sort(rng.choice(n_all, size=n, replace=False)).astype(np.int64)
        pick = (pick[(pick >= f0) & (pick < f0 + nf)] - f0).astype(np.uint32)
        old = self.leaf_ids[pick]
        new = np.frombuffer(b"".join(_h(o.tobytes() + b"v2") for o in old), dtype=np.uint8).reshape(len(pick), 32)
        return self.file_slots[pick], old, new

    # ------------------------------------------------ oracle twin (small S)
    def oflow(self, file_ids=None):
        """The same graph as reflow_oracle.OFlow objects (test infrastructure).
        Returns (nodes by kind name -> list, physical-bearing nodes)."""
        from reflow_oracle import OFileset, OFlow  # noqa: imported only by tests
        S, P, Q = self.S, self.P, self.Q
        fid = (lambda i: self.leaf_ids[i].tobytes()) if file_ids is None else file_ids
        T = {name: [] for name in self.kinds}
        one = lambda i: OFileset(map={".": (i, 0)})  # noqa: E731
        idx_cmd = INDEX_CMD % (b"%s", b"%s", b"%s")
        r0 = OFlow("OpIntern", url=REF_URL.decode(), done=True, value=one(self.ref_id))
        r1 = OFlow("OpExec", [r0], image=BWA.decode(), cmd=idx_cmd.decode(), argmap=[(False, 0), (True, 0)],
                   done=True, value=OFileset(map={f.decode(): (i, 0) for f, i in zip(INDEX_FILES, self.index_ids)}))
        r2 = OFlow("OpCoerce", [r1], flow_digest=FD_EXEC_OUT, done=True, value=r1.value)
        T["R0"], T["R1"], T["R2"] = [r0], [r1], [r2]

        def cmd_of(kind, i):
            kk = self.kinds[kind]
            L = len(kk.tmpl)
            arr = np.frombuffer(kk.tmpl, dtype=np.uint8).copy()
            for pos, width, vals in kk.digit_fields:
                arr[pos:pos + width] = _digits(vals[i:i + 1], width)[0]
            return arr[:L].tobytes()

        def exec_cmd(kind, i, ndeps, image):
            t = cmd_of(kind, i)
            body = t[ndeps * 34 + len(b"OpExec") + len(image):]
            return body[:len(body) - 8 * (ndeps + 1)].decode()

        c7s = []
        for i in range(Q):
            v1 = OFlow("OpVal", value=one(fid(2 * i)), done=True)
            v2 = OFlow("OpVal", value=one(fid(2 * i + 1)), done=True)
            c1 = OFlow("OpCoerce", [v1], flow_digest=FD_COERCE_FILE, done=True, value=v1.value)
            c2 = OFlow("OpCoerce", [v2], flow_digest=FD_COERCE_FILE, done=True, value=v2.value)
            e1 = OFlow("OpExec", [r2, c1, c2], image=BWA.decode(), cmd=exec_cmd("E1", i, 3, BWA),
                       argmap=[(False, 0), (False, 1), (False, 2), (True, 0)], done=True,
                       value=one(self.out_id(b"e1", i)))
            c3 = OFlow("OpCoerce", [e1], flow_digest=FD_EXEC_OUT, done=True, value=e1.value)
            k1 = OFlow("OpK", [c3], flow_digest=FD_FORCE, done=True, value=e1.value)
            c4 = OFlow("OpCoerce", [k1], flow_digest=FD_TO_FILESET, done=True, value=e1.value)
            e2 = OFlow("OpExec", [c4], image=SAMTOOLS.decode(), cmd=exec_cmd("E2", i, 1, SAMTOOLS),
                       argmap=[(False, 0), (True, 0)], done=True, value=one(self.out_id(b"e2", i)))
            c5 = OFlow("OpCoerce", [e2], flow_digest=FD_EXEC_OUT, done=True, value=e2.value)
            k2 = OFlow("OpK", [c5], flow_digest=FD_FORCE, done=True, value=e2.value)
            c6 = OFlow("OpCoerce", [k2], flow_digest=FD_TO_FILESET, done=True, value=e2.value)
            e3 = OFlow("OpExec", [c6], image=SAMTOOLS.decode(), cmd=exec_cmd("E3", i, 1, SAMTOOLS),
                       argmap=[(False, 0), (True, 0)], done=True, value=one(self.out_id(b"e3", i)))
            c7 = OFlow("OpCoerce", [e3], flow_digest=FD_EXEC_OUT, done=True, value=e3.value)
            for name, f in zip(self.PAIR_KINDS, [v1, v2, c1, c2, e1, c3, k1, c4, e2, c5, k2, c6, e3, c7]):
                T[name].append(f)
            c7s.append(c7)
        for s in range(S):
            deps = c7s[s * P:(s + 1) * P]
            ks = OFlow("OpK", deps, flow_digest=FD_MERGE, done=True,
                       value=OFileset(list=[d.value for d in deps]))
            cs1 = OFlow("OpCoerce", [ks], flow_digest=FD_TO_FILESET, done=True, value=ks.value)
            es = OFlow("OpExec", [cs1], image=SAMTOOLS.decode(), cmd=exec_cmd("ES", s, 1, SAMTOOLS),
                       argmap=[(False, 0), (True, 0)], done=True, value=one(self.out_id(b"es", s)))
            cs2 = OFlow("OpCoerce", [es], flow_digest=FD_EXEC_OUT, done=True, value=es.value)
            xs = OFlow("OpExtern", [cs2], url="s3://1000genomes-out/S%07d.bam" % s)
            for name, f in zip(self.SAMPLE_KINDS, [ks, cs1, es, cs2, xs]):
                T[name].append(f)
        return T


# --------------------------------------------------------------------- C4 --
def merge_tmpl(k):
    """A Merge over k deps (the shape of KS: k WD holes, "OpK", FD_MERGE)."""
    return WD0 * k + b"OpK" + b"\x00\x05" + FD_MERGE


def append_jobs(a, jobs):
    """Append jobs to rf_graph_desc arrays: jobs = [(tmpl bytes, [(pos,
    slot)...])], each given the next fresh output slot.  Returns (arrays,
    out slots).  One concatenation of the blob (it is ~15 GB at 100M nodes):
    callers that append in stages collect the jobs first (merge_tree_jobs)."""
    old = np.asarray(a["blob"], dtype=np.uint8)
    pad = (-len(old)) % 16
    base = len(old) + pad
    n = int(a["n_slots"])
    parts, offs, lens, hp, pos, sl, outs = [], [], [], [], [], [], []
    h = int(a["hole_ptr"][-1])
    cur = base
    for tmpl, holes in jobs:
        offs.append(cur)
        lens.append(len(tmpl))
        t = tmpl + bytes((-len(tmpl)) % 16)
        parts.append(t)
        cur += len(t)
        h += len(holes)
        hp.append(h)
        pos += [p for p, _ in holes]
        sl += [x for _, x in holes]
        outs.append(n)
        n += 1
    blob = np.concatenate([old, np.zeros(pad, np.uint8), np.frombuffer(b"".join(parts), dtype=np.uint8)])
    out = dict(n_slots=n,
               out_slot=np.concatenate([a["out_slot"], np.array(outs, np.uint32)]).astype(np.uint32),
               tmpl_off=np.concatenate([a["tmpl_off"], np.array(offs, np.uint64)]).astype(np.uint64),
               tmpl_len=np.concatenate([a["tmpl_len"], np.array(lens, np.uint32)]).astype(np.uint32),
               hole_ptr=np.concatenate([a["hole_ptr"], np.array(hp, np.uint64)]).astype(np.uint64),
               hole_pos=np.concatenate([a["hole_pos"], np.array(pos, np.uint32)]).astype(np.uint32),
               hole_slot=np.concatenate([a["hole_slot"], np.array(sl, np.uint32)]).astype(np.uint32),
               blob=blob)
    return out, np.array(outs, dtype=np.uint32)


def merge_tree_jobs(next_slot, leaves, fanin=32):
    """The jobs of a fan-in-`fanin` Merge tree over `leaves` slots whose
    outputs will be numbered from next_slot on (as append_jobs numbers them).
    Returns (jobs, root slot, [tree slots in job order])."""
    cur, made, jobs = np.asarray(leaves, dtype=np.uint32), [], []
    while len(cur) > 1:
        lvl = [(merge_tmpl(len(g)), [(34 * j + 2, int(x)) for j, x in enumerate(g)])
               for g in (cur[i:i + fanin] for i in range(0, len(cur), fanin))]
        cur = np.arange(next_slot, next_slot + len(lvl), dtype=np.uint32)
        next_slot += len(lvl)
        jobs += lvl
        made.append(cur)
    return jobs, int(cur[0]), (np.concatenate(made) if made else np.zeros(0, np.uint32))


def merge_tree(a, leaves, fanin=32):
    """Fan-in-`fanin` Merge tree over `leaves` slots, appended to arrays a.
    Returns (arrays, root slot, [tree slots in job order])."""
    jobs, root, made = merge_tree_jobs(int(a["n_slots"]), leaves, fanin)
    if jobs:
        a, _ = append_jobs(a, jobs)
    return a, root, made


class PartitionedDag1000:
    """configs[3]'s DAG, one rank's piece.  The global DAG is a 1000align DAG
    of nparts*S samples cut into nparts parts of S samples; each part's
    sample roots (XS) are merged by a fan-in-32 Merge tree into a part root,
    and the global root merges the nparts part roots (none when nparts = 1).
    Rank r of nranks owns k = nparts/nranks consecutive parts (samples [r*k*S,
    (r+1)*k*S)) -- SURVEY §8(e): partition by sample subtree, the shared
    reference-index chain replicated on every rank, the global root on rank
    0, which imports the other ranks' part roots (one 32-B boundary digest per
    part, so the exchange per step is nparts bits + 32*nparts bytes).  The
    global DAG is the same for every nranks dividing nparts (strong scaling:
    nranks = 1 holds all of it, no exchange), node for node.
    desc: this piece's rf_graph_desc arrays; part: its rf_graph_part (exports
    = the rank's part roots on ranks > 0; boundary id of part q = q).  Slot
    layout: the rank's Dag1000 slots, its tree slots (part by part), then
    (rank 0) the global root and the import slots of the other ranks' parts."""

    def __init__(self, S, P, nranks, rank, seed=0x5EED0003, fanin=32, nparts=None):
        nparts = nranks if nparts is None else nparts
        if nparts % nranks:
            raise ValueError("nparts (%d) must be a multiple of nranks (%d)" % (nparts, nranks))
        k = nparts // nranks
        self.nranks, self.rank, self.nparts, self.k = nranks, rank, nparts, k
        self.dag = Dag1000(k * S, P, seed, sample0=rank * k * S)
        a = self.dag.arrays()
        xs = self.dag.kinds["XS"].out_slot
        nxt = int(a["n_slots"])
        jobs, roots, trees = [], [], []
        for p in range(k):
            jb, root, tree = merge_tree_jobs(nxt, xs[p * S:(p + 1) * S], fanin)
            nxt += len(jb)
            jobs += jb
            roots.append(root)
            trees.append(tree)
        self.part_roots = np.array(roots, dtype=np.uint32)
        self.tree_slots = np.concatenate(trees) if trees else np.zeros(0, np.uint32)
        self.rank_root = roots[0] if k == 1 else None
        self.import_slot = np.zeros(0, np.uint32)
        self.global_root = None
        if rank == 0 and nparts > 1:
            # the global root takes the next slot, the imports the ones after
            # it, so every appended job goes in one append (one blob copy)
            self.global_root = nxt
            self.import_slot = np.arange(nxt + 1, nxt + 1 + nparts - k, dtype=np.uint32)
            holes = roots + self.import_slot.tolist()
            jobs.append((merge_tmpl(nparts), [(34 * j + 2, int(x)) for j, x in enumerate(holes)]))
        if jobs:
            a, outs = append_jobs(a, jobs)
        if self.global_root is not None:
            assert int(outs[-1]) == self.global_root
            a["n_slots"] = int(a["n_slots"]) + nparts - k
        self.desc = a
        self.n_nodes = self.dag.n_nodes + len(self.tree_slots) + (1 if self.global_root is not None else 0)
        multi = nranks > 1
        self.part = dict(nranks=nranks, rank=rank, max_export=k if multi else 0,
                         export_slot=self.part_roots if rank > 0 else np.zeros(0, np.uint32),
                         import_slot=self.import_slot,
                         import_bid=np.arange(k, nparts, dtype=np.uint32) if rank == 0 and multi
                         else np.zeros(0, np.uint32),
                         any_import=multi, rounds=1 if multi else 0)

    def dirty_work(self, file_slots, global_changed=True):
        """(jobs, nodes, material blocks) a change of the local leaf-file slots
        `file_slots` makes this piece hash -- the dirty closure, counted on the
        host from the layout: per changed file its Val + Coerce, per changed
        pair its ten-node chain + the pE1 physical key, per changed sample its
        five-node tail, the Merge-tree ancestors, and (rank 0, when anything
        anywhere changed) the global root.  Blocks are the full materials'
        (ceil((len + 9) / 64)), as the reference hashes them.  self.last_twice:
        the jobs the partitioned recompute hashes twice -- none: rank 0 holds
        the imports and no exports, so the library defers the levels from its
        import readers up until after the exchange (GraphPart::defer_lvl) and
        hashes the global root once; the device's count is jobs +
        last_twice."""
        d, a = self.dag, self.desc
        blk = {k: (len(kk.tmpl) + 9 + 63) // 64 for k, kk in d.kinds.items()}
        f = np.asarray(file_slots, dtype=np.int64)
        odd = int((f % 2).sum())
        even = len(f) - odd
        jobs = 2 * len(f)
        blocks = even * (blk["V1"] + blk["C1"]) + odd * (blk["V2"] + blk["C2"])
        pairs = np.unique(f // 2)
        chain = ("E1", "C3", "K1", "C4", "E2", "C5", "K2", "C6", "E3", "C7", "pE1")
        jobs += len(pairs) * len(chain)
        blocks += len(pairs) * sum(blk[k] for k in chain)
        samples = np.unique(pairs // d.P)
        tail = ("KS", "CS1", "ES", "CS2", "XS")
        jobs += len(samples) * len(tail)
        blocks += len(samples) * sum(blk[k] for k in tail)
        # the Merge trees (and the global root): the jobs appended after the DAG's
        dirty = set(d.kinds["XS"].out_slot[samples].tolist())
        hp, hs, osl, tl = a["hole_ptr"], a["hole_slot"], a["out_slot"], a["tmpl_len"]
        imports = set(self.import_slot.tolist())
        self.last_twice = 0
        for j in range(d.n_jobs, len(osl)):
            deps = hs[int(hp[j]):int(hp[j + 1])].tolist()
            local = any(x in dirty for x in deps)
            imported = global_changed and any(x in imports for x in deps)
            if local or imported:
                dirty.add(int(osl[j]))
                jobs += 1
                blocks += (int(tl[j]) + 9 + 63) // 64
        return jobs, jobs - len(pairs), blocks

    def critical_path(self, file_slots):
        """The longest chain of dependent compressions in this piece for a
        change of its leaf-file slots: the Dag1000 chain to a dirty sample
        root, then the Merge tree above it and (rank 0) the global root --
        blocks, each job's constant leading blocks excluded."""
        d, a = self.dag, self.desc
        f = np.asarray(file_slots, dtype=np.int64)
        base = d.critical_path(f)
        if not base:
            return 0
        dirty_xs = set(d.kinds["XS"].out_slot[np.unique(f // 2 // d.P)].tolist())
        hp, hs, hpos = a["hole_ptr"], a["hole_slot"], a["hole_pos"]
        osl, tl = a["out_slot"], a["tmpl_len"]
        path = {s: base for s in dirty_xs}
        best = base
        for j in range(d.n_jobs, len(osl)):  # the appended jobs, in dependency order
            deps = [path[x] for x in hs[int(hp[j]):int(hp[j + 1])].tolist() if x in path]
            if deps:
                lead = int(hpos[int(hp[j])]) // 64 if hp[j + 1] > hp[j] else 0
                path[int(osl[j])] = max(deps) + (int(tl[j]) + 9 + 63) // 64 - lead
                best = max(best, path[int(osl[j])])
        return best
