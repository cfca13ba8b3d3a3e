"""configs[3]'s partitioned DAG on the CPU: the per-rank pieces
bench.py builds (workloads.PartitionedDag1000: samples [r*S, (r+1)*S), the
shared reference chain replicated, per-rank Merge tree, global root on rank
0) together compute exactly the digests of the one global DAG, slot for slot,
through the superstep exchange of rf_graph_recompute_part (ranks as threads,
the oracle as each rank's local engine); and rf_graph_split of that global
DAG (the library's splitter) finds the same boundary."""
import numpy as np
import pytest

import partition_case as PC
from reflow_amd import capi
from reflow_amd.workloads import Dag1000, PartitionedDag1000


def test_sample0_slices_the_global_dag():
    G = Dag1000(6, 3)
    for r in range(3):
        d = Dag1000(2, 3, sample0=2 * r)
        assert (d.leaf_ids == G.leaf_ids[12 * r:12 * (r + 1)]).all()
        a, ga = d.arrays(), G.arrays()
        for name in ("E1", "ES", "pE2", "pXS"):
            k, gk = d.kinds[name], G.kinds[name]
            gi = np.arange(k.count) + r * k.count
            for i in range(k.count):
                j = int(np.nonzero(a["out_slot"] == k.out_slot[i])[0][0])
                gj = int(np.nonzero(ga["out_slot"] == gk.out_slot[gi[i]])[0][0])
                assert bytes(a["blob"][a["tmpl_off"][j]:a["tmpl_off"][j] + a["tmpl_len"][j]]) == \
                    bytes(ga["blob"][ga["tmpl_off"][gj]:ga["tmpl_off"][gj] + ga["tmpl_len"][gj]])


@pytest.mark.parametrize("protocol", ["supersteps", "rounds"])
@pytest.mark.parametrize("nranks,S,P,fanin", [(2, 5, 3, 32), (3, 40, 4, 8), (4, 9, 2, 4)])
def test_c4_pieces_equal_global_dag(nranks, S, P, fanin, protocol):
    G, ga, owner, roots, trees, groot = PC.global_c4(S, P, nranks, fanin=fanin)
    rng = np.random.default_rng(nranks)
    nf = len(G.file_slots)
    ids = [G.leaf_ids.copy()]
    picks = []
    for frac, ranks in ((0.01, range(nranks)), (0.2, range(1, nranks))):  # then: rank 0's samples unchanged
        pick = np.sort(rng.choice([k for k in range(nf) if k // (2 * P * S) in ranks], size=max(1, int(nf * frac)),
                                  replace=False))
        new = ids[-1].copy()
        new[pick] = rng.integers(0, 256, size=(len(pick), 32), dtype=np.uint8)
        ids.append(new)
        picks.append(pick)
    wants = [PC.global_digests(G, ga, x) for x in ids]

    def body(r, ag):
        pc = PartitionedDag1000(S, P, nranks, r, fanin=fanin)
        if protocol == "supersteps":
            pc.part = dict(pc.part, rounds=0)
        m = PC.c4_local_to_global(pc, G, roots, trees, groot)
        f0 = 2 * pc.dag.Q * r
        out = []
        st, n = PC.superstep_oracle(pc.desc, pc.part, ag, inputs=(pc.dag.file_slots, ids[0][f0:f0 + 2 * pc.dag.Q]))
        out.append((st["og"].slots[:len(m)].copy(), n))
        for pick, x in zip(picks, ids[1:]):
            mine = pick[(pick >= f0) & (pick < f0 + 2 * pc.dag.Q)]
            st, n = PC.superstep_oracle(pc.desc, pc.part, ag, changed=(pc.dag.file_slots[mine - f0], x[mine]),
                                        state=st)
            out.append((st["og"].slots[:len(m)].copy(), n))
        st["og"].close()
        return m, out

    res = PC.run_threads(nranks, body)
    for r, (m, out) in enumerate(res):
        for step, ((slots, n), want) in enumerate(zip(out, wants)):
            assert (slots == want[m]).all(), (r, step)
            assert n == 2  # rank roots -> global root, then quiet
    assert (wants[2][groot] != wants[1][groot]).any()  # rank 0 saw only imported changes


@pytest.mark.parametrize("nranks", [1, 2, 4])
def test_strong_layout_fixed_global_dag(nranks):
    """bench.py's strong-scaling layout: ONE global DAG of nparts = 4 parts,
    nranks | nparts, rank r holding parts [r*k, (r+1)*k) -- every rank count
    computes the same digests (nranks = 1: the whole DAG, no exchange)."""
    S, P, nparts, fanin = 6, 3, 4, 4
    G, ga, owner, roots, trees, groot = PC.global_c4(S, P, nparts, fanin=fanin)
    rng = np.random.default_rng(3)
    nf = len(G.file_slots)
    pick = np.sort(rng.choice(nf, size=7, replace=False))
    new = G.leaf_ids.copy()
    new[pick] = rng.integers(0, 256, size=(len(pick), 32), dtype=np.uint8)
    wants = [PC.global_digests(G, ga, x) for x in (G.leaf_ids, new)]

    def body(r, ag):
        pc = PartitionedDag1000(S, P, nranks, r, fanin=fanin, nparts=nparts)
        assert pc.k == nparts // nranks
        m = PC.c4_local_to_global(pc, G, roots, trees, groot)
        f0, nfl = 2 * pc.dag.Q * r, 2 * pc.dag.Q
        st, _ = PC.superstep_oracle(pc.desc, pc.part, ag, inputs=(pc.dag.file_slots, G.leaf_ids[f0:f0 + nfl]))
        out = [st["og"].slots[:len(m)].copy()]
        mine = pick[(pick >= f0) & (pick < f0 + nfl)]
        st, _ = PC.superstep_oracle(pc.desc, pc.part, ag, changed=(pc.dag.file_slots[mine - f0], new[mine]), state=st)
        out.append(st["og"].slots[:len(m)].copy())
        st["og"].close()
        return m, out, pc.part

    res = PC.run_threads(nranks, body)
    for r, (m, out, part) in enumerate(res):
        for step, (slots, want) in enumerate(zip(out, wants)):
            assert (slots == want[m]).all(), (r, step)
        if nranks > 1:
            assert part["max_export"] == nparts // nranks and part["rounds"] == 1
            assert len(part["import_slot"]) == (nparts - nparts // nranks if r == 0 else 0)
    assert (wants[1][groot] != wants[0][groot]).any()
    with pytest.raises(ValueError):
        PartitionedDag1000(S, P, 3, 0, nparts=nparts)


def test_split_finds_the_same_boundary():
    nranks, S, P = 3, 10, 2
    G, ga, owner, roots, trees, groot = PC.global_c4(S, P, nranks, fanin=4)
    for r in range(nranks):
        piece = capi.GraphPiece(ga, nranks, r, owner)
        pc = PartitionedDag1000(S, P, nranks, r, fanin=4)
        gl = piece.global_of_local
        assert sorted(gl[piece.part["export_slot"]].tolist()) == ([roots[r]] if r else [])
        assert sorted(gl[piece.part["import_slot"]].tolist()) == (sorted(roots[1:]) if r == 0 else [])
        assert len(piece.desc["out_slot"]) == len(pc.desc["out_slot"])
        assert piece.part["any_import"]
        assert piece.part["rounds"] == pc.part["rounds"] == 1  # rank roots -> global root


def test_split_counts_boundary_crossings():
    """rf_graph_split's rounds: the most rank-boundary crossings on any path."""
    dag, arrays, owner, root_slot, tail_slot = PC.global_case(S=6, P=2, nranks=3)
    assert capi.GraphPiece(arrays, 3, 1, owner).part["rounds"] == 2  # sample roots -> root (0) -> tail (2)
    one = np.zeros_like(owner)  # everything on rank 0 (replicated kinds stay replicated)
    one[owner < 0] = -1
    p = capi.GraphPiece(arrays, 2, 0, one).part
    assert p["rounds"] == 0 and not p["any_import"]
    rep = owner.copy()  # the tail replicated: still read across ranks once more
    rep[-1] = -1
    assert capi.GraphPiece(arrays, 3, 0, rep).part["rounds"] == 2


@pytest.mark.parametrize("nparts,fanin", [(1, 32), (4, 4)])
def test_dirty_work_matches_oracle(nparts, fanin):
    """PartitionedDag1000.dirty_work (bench.py's dirty-node and block counts
    for the 100M leg, where the oracle is too slow) equals the oracle's
    incremental update: jobs hashed and material blocks."""
    import reflow_oracle as O
    pc = PartitionedDag1000(10, 3, 1, 0, fanin=fanin, nparts=nparts)
    slots, old, new = pc.dag.change_set(0.1)
    og = O.OGraph(pc.desc)
    og.set_inputs(pc.dag.file_slots, pc.dag.leaf_ids)
    og.full()
    jobs = og.update(slots, new)
    blocks = og.last_blocks()
    og.close()
    assert pc.dirty_work(slots)[0] == jobs
    assert pc.dirty_work(slots)[2] == blocks


@pytest.mark.parametrize("nranks", [2, 4])
def test_persample_layout_pieces_equal_global_dag(nranks):
    """bench.py's per-sample-root layout at N ranks (bench_persample: SURVEY
    §8(d) C3/C4 as written -- samples independent, one module per sample in
    /root/reference/doc/1000align/1000align.rf:37-47 -- so no exchange): rank
    r holds samples [r S/N, (r+1) S/N) (Dag1000 sample0), the global change
    set restricted to its slice (change_set n_global).  Together the pieces'
    change sets are exactly the global one, and each piece's oracle
    incremental update gives its samples' digests of the global DAG (every
    per-sample kind, root included); the bench's dirty-node count sums to
    the global count."""
    import reflow_oracle as O
    S, P = 8, 3
    G = Dag1000(S, P)
    gsl, _, gnew = G.change_set(0.1)
    og = O.OGraph(G.arrays())
    og.set_inputs(G.file_slots, G.leaf_ids)
    og.full()
    og.update(gsl, gnew)

    def n_dirty(f):
        f = np.asarray(f, dtype=np.int64)
        return int(2 * len(f) + 10 * len(np.unique(f // 2)) + 5 * len(np.unique(f // 2 // P)))

    s_rank = S // nranks
    got_changes, dirty_sum = {}, 0
    for r in range(nranks):
        d = Dag1000(s_rank, P, sample0=r * s_rank)
        sl, _, new = d.change_set(0.1, n_global=2 * P * S)
        for s, v in zip(sl.tolist(), new):
            got_changes[s + 2 * P * s_rank * r] = bytes(v)  # local file slot -> global file index
        dirty_sum += n_dirty(sl)
        o = O.OGraph(d.arrays())
        o.set_inputs(d.file_slots, d.leaf_ids)
        o.full()
        if len(sl):
            o.update(sl, new)
        for name in ("KS", "CS1", "ES", "CS2", "XS", "pES", "pXS"):
            k, gk = d.kinds[name], G.kinds[name]
            gi = np.arange(k.count) + r * k.count
            assert (o.slots[k.out_slot] == og.slots[gk.out_slot[gi]]).all(), (r, name)
        o.close()
    og.close()
    assert got_changes == {int(s): bytes(v) for s, v in zip(gsl.tolist(), gnew)}
    assert dirty_sum == n_dirty(gsl)
