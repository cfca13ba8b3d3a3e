"""Test helper: lower oracle flows (reflow_oracle.OFlow) into rf_graph jobs.

Used only by the tests to drive the C-ABI graph engine with graphs whose
digests the oracle computes independently.  Byte grammar: SURVEY App. A /
flow.go:675-792.  File IDs of Fileset values can be bound to input slots
(file_slots=True) so tests can change them through rf_graph_set_slots.
"""
from __future__ import annotations

import numpy as np

from reflow_oracle import OP, OFlow, OFileset, op_digest_string, writeN


class Lowered:
    def __init__(self):
        self.jobs = []          # (out_slot, material bytearray, holes[(pos, slot)])
        self.n_slots = 0
        self.logical = {}       # id(flow) -> slot
        self.physical = {}      # id(flow) -> slot
        self.file_slot = {}     # file id bytes -> slot (only with file_slots)
        self.file_value = {}    # slot -> current id bytes

    def new_slot(self):
        s = self.n_slots
        self.n_slots += 1
        return s

    def arrays(self):
        out_slot, off, ln, hptr, hpos, hslot = [], [], [], [0], [], []
        blob = bytearray()
        for slot, mat, holes in self.jobs:
            out_slot.append(slot)
            off.append(len(blob))
            ln.append(len(mat))
            blob += mat
            while len(blob) % 16:
                blob.append(0)
            for pos, hs in holes:
                hpos.append(pos)
                hslot.append(hs)
            hptr.append(len(hpos))
        return dict(n_slots=self.n_slots, out_slot=np.array(out_slot, dtype=np.uint32),
                    tmpl_off=np.array(off, dtype=np.uint64), tmpl_len=np.array(ln, dtype=np.uint32),
                    hole_ptr=np.array(hptr, dtype=np.uint64), hole_pos=np.array(hpos, dtype=np.uint32),
                    hole_slot=np.array(hslot, dtype=np.uint32), blob=bytes(blob))


class Lowerer:
    def __init__(self, universe=b"", file_slots=False):
        self.U = universe
        self.file_slots = file_slots
        self.L = Lowered()

    # pieces: list of bytes | ("hole", slot)
    def _wd_hole(self, slot):
        return [b"\x00\x05", ("hole", slot)]

    def _fileset_pieces(self, v: OFileset):
        if v.list is not None:
            out = []
            for x in v.list:
                out += self._fileset_pieces(x)
            return out
        out = []
        for path in sorted((v.map or {}).keys(), key=lambda s: s.encode()):
            fid = v.map[path][0]
            out.append(path.encode())
            if self.file_slots:
                s = self.L.file_slot.get(fid)
                if s is None:
                    s = self.L.new_slot()
                    self.L.file_slot[fid] = s
                    self.L.file_value[s] = fid
                out += self._wd_hole(s)
            else:
                out.append(b"\x00\x05" + fid)
        return out

    def _material(self, f: OFlow, merged: bool):
        """Flow.WriteDigest (flow.go:675-750) with WD(dep.Digest()) as holes:
        the node's own HashV1 (or the Canonicalize merge) decides inlining;
        the Parent keeps its own config (see reflow_oracle.OFlow.material)."""
        v1 = merged or f.hashv1
        U = self.U
        if f.op == OP["OpRequirements"]:
            return [U] + self._material(f.deps[0], merged)
        if f.parent is not None:
            return [U] + self._material(f.parent, False)
        out = [U]
        for d in f.deps:
            if v1:
                out += self._material(d, merged)
            else:
                out += self._wd_hole(self.lower(d, merged))
        out.append(op_digest_string(f.op).encode())
        op = f.op
        if op in (OP["OpIntern"], OP["OpExtern"]):
            out.append(f.url.encode())
        elif op == OP["OpExec"]:
            out.append(f.image.encode() + f.cmd.encode() + f.argbytes())
        elif op == OP["OpGroupby"]:
            out.append(f.re.encode())
        elif op == OP["OpMap"]:
            out += self._material(f.mapflow, merged)
        elif op == OP["OpCollect"]:
            out.append(f.re.encode() + f.repl.encode())
        elif op == OP["OpVal"]:
            if f.value is not None:
                out += self._fileset_pieces(f.value)
            else:
                out.append(b"\x00\x05" + f.flow_digest)
        elif op in (OP["OpK"], OP["OpCoerce"]):
            out.append(b"\x00\x05" + f.flow_digest)
        elif op == OP["OpData"]:
            out.append(f.data)
        return out

    def _emit(self, slot, pieces):
        mat = bytearray()
        holes = []
        for p in pieces:
            if isinstance(p, tuple):
                holes.append((len(mat), p[1]))
                mat += b"\0" * 32
            else:
                mat += p
        self.L.jobs.append((slot, mat, holes))

    def lower(self, f: OFlow, v1=False) -> int:
        """Logical digest slot of f (jobs for its deps are emitted first);
        v1 = f is a Canonicalize copy under Config{HashV1: true}."""
        key = (id(f), bool(v1))
        if key in self.L.logical:
            return self.L.logical[key]
        pieces = self._material(f, bool(v1))
        slot = self.L.new_slot()
        self.L.logical[key] = slot
        self._emit(slot, pieces)
        return slot

    def lower_physical(self, f: OFlow):
        """Physical digest slot of f or None (flow.go:764-792)."""
        if f.op not in (OP["OpExtern"], OP["OpExec"]):
            return None
        if any(not d.done for d in f.deps):
            return None
        key = id(f)
        if key in self.L.physical:
            return self.L.physical[key]
        pieces = []
        for d in f.deps:
            pieces += self._fileset_pieces(d.value)
        if f.op == OP["OpExtern"]:
            pieces.append(f.url.encode())
        else:
            pieces.append(f.image.encode() + f.cmd.encode() + f.argbytes())
        slot = self.L.new_slot()
        self.L.physical[key] = slot
        self._emit(slot, pieces)
        return slot


def walk(root):
    seen, order, stack = set(), [], [root]
    while stack:
        f = stack.pop()
        if id(f) in seen:
            continue
        seen.add(id(f))
        order.append(f)
        stack.extend(f.deps)
        if f.mapflow is not None:
            stack.append(f.mapflow)
        if f.parent is not None:
            stack.append(f.parent)
    return order
