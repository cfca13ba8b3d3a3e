"""Test helper: a global job graph partitioned over ranks.

A 1000align DAG (reflow_amd.workloads.Dag1000) split by sample, the shared
reference-index chain replicated (owner -1), plus two jobs that make the
exchange real: a global root Merge over every sample's Extern (owned by rank
0, so it imports every other rank's sample roots) and a consumer of that root
owned by the last rank (so a change crosses ranks twice: two supersteps).

superstep_oracle() runs the protocol of rf_graph_recompute_part with the
oracle (reflow_oracle.OGraph) as each rank's local engine -- test
infrastructure for the CPU checks of the splitter and the exchange."""
import numpy as np

import reflow_oracle as O
from reflow_amd.workloads import Dag1000

WD0 = b"\x00\x05" + bytes(32)


def global_case(S=6, P=4, nranks=2):
    dag = Dag1000(S, P)
    a = dag.arrays()
    roots = dag.kinds["XS"].out_slot
    n_slots = a["n_slots"]
    tmpl_root = WD0 * S + b"OpMerge"
    tmpl_tail = WD0 + b"OpCoerce" + b"\x00\x05" + O.sha256(b"global tail")
    blob = bytearray(bytes(a["blob"]))
    while len(blob) % 16:
        blob.append(0)
    off_root = len(blob)
    blob += tmpl_root + bytes((-len(tmpl_root)) % 16)
    off_tail = len(blob)
    blob += tmpl_tail + bytes((-len(tmpl_tail)) % 16)
    root_slot, tail_slot = n_slots, n_slots + 1
    out = dict(n_slots=n_slots + 2,
               out_slot=np.concatenate([a["out_slot"], [root_slot, tail_slot]]).astype(np.uint32),
               tmpl_off=np.concatenate([a["tmpl_off"], [off_root, off_tail]]).astype(np.uint64),
               tmpl_len=np.concatenate([a["tmpl_len"], [len(tmpl_root), len(tmpl_tail)]]).astype(np.uint32),
               hole_ptr=np.concatenate([a["hole_ptr"], [a["hole_ptr"][-1] + S, a["hole_ptr"][-1] + S + 1]])
               .astype(np.uint64),
               hole_pos=np.concatenate([a["hole_pos"], 34 * np.arange(S) + 2, [2]]).astype(np.uint32),
               hole_slot=np.concatenate([a["hole_slot"], roots, [root_slot]]).astype(np.uint32),
               blob=np.frombuffer(bytes(blob), dtype=np.uint8))
    # owner: by sample; shared kinds replicated; global root rank 0, tail last rank
    owner = []
    for name, kk in dag.kinds.items():
        if name in ("R0", "R1", "R2", "pR1"):
            owner.append(np.full(kk.count, -1))
        elif kk.count == dag.Q:
            owner.append((np.arange(kk.count) // dag.P) % nranks)
        else:
            owner.append(np.arange(kk.count) % nranks)
    owner = np.concatenate(owner + [[0, nranks - 1]]).astype(np.int32)
    return dag, out, owner, root_slot, tail_slot


def global_digests(dag, arrays, file_ids):
    g = O.OGraph(arrays)
    g.set_inputs(dag.file_slots, file_ids)
    g.full()
    d = g.slots[:arrays["n_slots"]].copy()
    g.close()
    return d


def superstep_oracle(piece, dag, file_ids, allgather, changed=None, state=None):
    """Rank's side of rf_graph_recompute_part with the oracle as local engine.
    allgather(bytes) -> [bytes per rank].  First call (state None): load +
    full; later calls: `changed` = (global file slots, new IDs).  Returns
    (state, supersteps)."""
    part, g2l = piece.part, {int(gs): i for i, gs in enumerate(piece.global_of_local)}
    nr, me, mx = part["nranks"], part["rank"], part["max_export"]
    if state is None:
        og = O.OGraph(piece.desc)
        local_files = [(g2l[int(s)], file_ids[k]) for k, s in enumerate(dag.file_slots) if int(s) in g2l]
        if local_files:
            og.set_inputs([s for s, _ in local_files], np.stack([d for _, d in local_files]))
        og.full()
        state = {"og": og, "snap": np.zeros((len(part["export_slot"]), 32), np.uint8)}
    else:
        og = state["og"]
        sl, ids = changed
        loc = [(g2l[int(s)], ids[k]) for k, s in enumerate(sl) if int(s) in g2l]
        if loc:
            og.update([s for s, _ in loc], np.stack([d for _, d in loc]))
    steps = 0
    nbits = nr * mx
    while True:
        steps += 1
        if nbits == 0:
            break
        cur = og.slots[part["export_slot"]] if len(part["export_slot"]) else np.zeros((0, 32), np.uint8)
        bits = np.zeros(nbits, np.uint8)
        ch = (cur != state["snap"]).any(axis=1) if len(cur) else np.zeros(0, bool)
        bits[me * mx + np.nonzero(ch)[0]] = 1
        state["snap"] = cur.copy()
        ored = np.bitwise_or.reduce(np.stack([np.frombuffer(b, np.uint8) for b in allgather(bits.tobytes())]), axis=0)
        if part["any_import"] and not ored.any():
            break
        send = np.zeros((mx, 32), np.uint8)
        send[:len(cur)] = cur
        gathered = np.concatenate([np.frombuffer(b, np.uint8).reshape(mx, 32) for b in allgather(send.tobytes())])
        if not part["any_import"]:
            break
        sel = [i for i, b in enumerate(part["import_bid"]) if ored[b]]
        if sel:
            og.update(part["import_slot"][sel], gathered[part["import_bid"][sel]])
    return state, steps
