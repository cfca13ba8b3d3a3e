"""Test helper: a global job graph partitioned over ranks.

global_case: a 1000align DAG (reflow_amd.workloads.Dag1000) split by
sample with rf_graph_split, the shared
reference-index chain replicated (owner -1), plus two jobs that make the
exchange real: a global root Merge over every sample's Extern (owned by rank
0, so it imports every other rank's sample roots) and a consumer of that root
owned by the last rank (so a change crosses ranks twice: two supersteps).
global_c4: configs[3]'s DAG as bench.py lays it out per rank
(workloads.PartitionedDag1000), with the map from each piece to it.

superstep_oracle() runs the protocol of rf_graph_recompute_part with the
oracle (reflow_oracle.OGraph) as each rank's local engine -- test
infrastructure for the CPU checks of the splitter and the exchange."""
import threading

import numpy as np

import reflow_oracle as O
from reflow_amd.workloads import Dag1000, PartitionedDag1000, merge_tree_jobs

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


def piece_inputs(piece, dag, file_ids, pick=None):
    """(local slots, IDs) of a GraphPiece's leaf files among global file
    indices `pick` (default all)."""
    g2l = {int(s): i for i, s in enumerate(piece.global_of_local)}
    ks = range(len(dag.file_slots)) if pick is None else pick
    mine = [k for k in ks if int(dag.file_slots[k]) in g2l]
    return (np.array([g2l[int(dag.file_slots[k])] for k in mine], np.uint32),
            file_ids[mine] if len(mine) else np.zeros((0, 32), np.uint8))


def global_digests(dag, arrays, file_ids):
    g = O.OGraph(arrays)
    g.set_inputs(dag.file_slots, file_ids)
    g.full()
    d = g.slots[:arrays["n_slots"]].copy()
    g.close()
    return d


SHARED = ("R0", "R1", "R2", "pR1")


class ThreadGather:
    """All-gather between threads of one process (ranks as threads)."""

    def __init__(self, n):
        self.n, self.bar, self.buf = n, threading.Barrier(n, timeout=600), [None] * n

    def fn(self, rank):
        def allgather(b):
            self.buf[rank] = b
            self.bar.wait()
            out = list(self.buf)
            self.bar.wait()
            return out
        return allgather


def run_threads(nranks, body):
    """body(rank, allgather) on nranks threads; returns the results by rank
    (re-raises the first failure)."""
    tg = ThreadGather(nranks)
    res, errs = [None] * nranks, []

    def main(r):
        try:
            res[r] = body(r, tg.fn(r))
        except BaseException as e:  # noqa: BLE001
            errs.append((r, e))
            tg.bar.abort()

    th = [threading.Thread(target=main, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    if errs:
        raise errs[0][1]
    return res


def global_c4(S, P, nranks, seed=0x5EED0003, fanin=32):
    """The whole configs[3] DAG that PartitionedDag1000(S, P, nranks, r)
    pieces -- itself the one-rank piece of nranks parts -- with an owner per
    job (part r -> rank r).  Returns (G, arrays, owner, part roots, part tree
    slots, global root)."""
    whole = PartitionedDag1000(S, P, 1, 0, seed=seed, fanin=fanin, nparts=nranks)
    G, a = whole.dag, whole.desc
    sizes = [len(merge_tree_jobs(0, np.zeros(S, np.uint32), fanin)[0])] * nranks
    trees = np.split(whole.tree_slots, np.cumsum(sizes)[:-1])
    owner = []
    for name, kk in G.kinds.items():
        if name in SHARED:
            owner.append(np.full(kk.count, -1))
        elif kk.count == G.Q:
            owner.append(np.arange(kk.count) // (P * S))
        else:
            owner.append(np.arange(kk.count) // S)
    for r in range(nranks):
        owner.append(np.full(len(trees[r]), r))
    if whole.global_root is not None:
        owner.append([0])
    return G, a, np.concatenate(owner).astype(np.int32), whole.part_roots.tolist(), trees, whole.global_root


def c4_local_to_global(piece, G, roots, trees, groot):
    """Global slot of every slot of a PartitionedDag1000 piece."""
    d, r, k = piece.dag, piece.rank, piece.k
    m = np.full(int(piece.desc["n_slots"]), -1, dtype=np.int64)
    m[d.file_slots] = G.file_slots[2 * d.Q * r:2 * d.Q * (r + 1)]
    for name, kk in d.kinds.items():
        off = 0 if name in SHARED else r * kk.count
        m[kk.out_slot] = G.kinds[name].out_slot[off:off + kk.count]
    m[piece.tree_slots] = np.concatenate(trees[r * k:(r + 1) * k])
    if piece.global_root is not None:
        m[piece.import_slot] = roots[k:]
        m[piece.global_root] = groot
    assert (m >= 0).all()
    return m


def superstep_oracle(desc, part, allgather, inputs=None, changed=None, state=None):
    """Rank's side of rf_graph_recompute_part with the oracle as local engine.
    allgather(bytes) -> [bytes per rank].  First call (state None): inputs =
    (local slots, IDs) loaded, full recompute; later calls: `changed` = (local
    slots, new IDs).  part["rounds"] > 0: the fixed-round protocol (every
    export digest gathered each round, imports that differ written), else
    supersteps until nothing changed.  Returns (state, supersteps)."""
    nr, me, mx = part["nranks"], part["rank"], part["max_export"]
    if state is None:
        og = O.OGraph(desc)
        if inputs is not None and len(inputs[0]):
            og.set_inputs(inputs[0], inputs[1])
        og.full()
        state = {"og": og, "snap": np.zeros((len(part["export_slot"]), 32), np.uint8)}
    else:
        og = state["og"]
        if changed is not None and len(changed[0]):
            og.update(changed[0], changed[1])
    rounds = part.get("rounds", 0)
    if rounds and nr > 1:
        for _ in range(rounds):
            cur = og.slots[part["export_slot"]] if len(part["export_slot"]) else np.zeros((0, 32), np.uint8)
            send = np.zeros((mx, 32), np.uint8)
            send[:len(cur)] = cur
            gathered = np.concatenate([np.frombuffer(b, np.uint8).reshape(mx, 32) for b in allgather(send.tobytes())])
            if len(part["import_slot"]):
                imp = np.asarray(part["import_slot"])
                new = gathered[np.asarray(part["import_bid"])]
                diff = (og.slots[imp] != new).any(axis=1)
                if diff.any():
                    og.update(imp[diff], new[diff])
        return state, 1 + rounds
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
