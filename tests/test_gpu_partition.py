"""One job DAG partitioned over ranks on the GPU (rf_graph_set_part +
rf_graph_recompute_part): each rank holds its piece in its own
rf_ctx and runs the superstep exchange through a host all-gather; every
rank's slots equal the oracle's single-rank recompute of the whole graph,
slot for slot, after a full recompute and after incremental changes that
cross ranks -- with both exchange protocols: the supersteps until nothing
changes (rf_graph_part.rounds = 0) and the fixed rounds the splitter counts
(the most rank-boundary crossings on any path; no host round trip).  Pieces come from the library's splitter (rf_graph_split of
partition_case.global_case: a change crosses ranks twice) and from bench.py's
per-rank layout of configs[3] (workloads.PartitionedDag1000).  Ranks are
threads of one process sharing the GPU (RCCL needs one GPU per rank; bench.py
--gpus N uses it)."""
import numpy as np
import pytest

import partition_case as PC
from reflow_amd import capi
from reflow_amd.workloads import PartitionedDag1000

pytestmark = pytest.mark.gpu


def _changes(nf, rng, fracs):
    changes = []
    for frac in fracs:
        pick = np.sort(rng.choice(nf, size=max(1, int(nf * frac)), replace=False))
        changes.append((pick, rng.integers(0, 256, size=(len(pick), 32), dtype=np.uint8)))
    changes.append((np.zeros(0, np.int64), np.zeros((0, 32), np.uint8)))  # nothing changed
    return changes


def _states(ids, changes):
    out = [ids]
    for pick, new in changes:
        x = out[-1].copy()
        x[pick] = new
        out.append(x)
    return out


def _run(ctx_rank_setup, nranks, changes):
    """ctx_rank_setup(r, ctx) -> (graph, n_local, local inputs (slots, ids),
    change mapper (pick, new) -> (slots, ids))."""
    def body(r, ag):
        ctx = capi.Context(0, host_threads=0)
        try:
            g, n_local, inputs, to_local = ctx_rank_setup(r, ctx)
            if len(inputs[0]):
                g.set_slots(inputs[0], inputs[1])
            every = np.arange(n_local, dtype=np.uint32)
            out = [(g.recompute_part(allgather=ag, nranks=nranks, full=True), g.get_slots(every),
                    g.part_gathered()[2])]
            for pick, new in changes:
                sl, ids = to_local(pick, new)
                if len(sl):
                    g.set_slots(sl, ids)
                out.append((g.recompute_part(allgather=ag, nranks=nranks), g.get_slots(every), g.part_gathered()[2]))
            g.close()
            return out
        finally:
            ctx.close()
    return PC.run_threads(nranks, body)


def _part(part, protocol):
    return part if protocol == "rounds" else dict(part, rounds=0)


@pytest.mark.parametrize("protocol", ["supersteps", "rounds"])
@pytest.mark.parametrize("nranks,S,P", [(2, 6, 4), (3, 40, 8), (4, 64, 16)])
def test_split_pieces_match_single_rank(nranks, S, P, protocol):
    dag, arrays, owner, root_slot, tail_slot = PC.global_case(S=S, P=P, nranks=nranks)
    changes = _changes(len(dag.file_slots), np.random.default_rng(nranks), (0.01, 0.3))
    pieces = [capi.GraphPiece(arrays, nranks, r, owner) for r in range(nranks)]
    assert all(pc.part["rounds"] == 2 for pc in pieces)  # sample roots -> global root -> tail

    def setup(r, ctx):
        pc = pieces[r]
        g = capi.Graph.from_arrays(ctx, pc.desc)
        g.set_part(_part(pc.part, protocol))
        return (g, len(pc.global_of_local), PC.piece_inputs(pc, dag, dag.leaf_ids),
                lambda pick, new: PC.piece_inputs(pc, dag, _scatter(dag, pick, new), pick))

    res = _run(setup, nranks, changes)
    wants = [PC.global_digests(dag, arrays, x) for x in _states(dag.leaf_ids, changes)]
    covered = set()
    for r, out in enumerate(res):
        gl = pieces[r].global_of_local
        covered |= set(gl.tolist())
        for step, ((n, slots, supersteps), want) in enumerate(zip(out, wants)):
            assert (slots == want[gl]).all(), (r, step)
        if protocol == "rounds":
            assert all(st == 3 for _, _, st in out)  # a local pass + two exchange rounds, always
            assert out[3][0] == 0  # nothing changed: nothing hashed
        else:
            assert out[2][2] >= 3  # 30% change: sample roots -> global root -> tail
            assert out[3][0] == 0 and out[3][2] == 1  # nothing changed: one quiet superstep
    assert covered == set(range(arrays["n_slots"]))


def _scatter(dag, pick, new):
    x = np.zeros((len(dag.file_slots), 32), np.uint8)
    x[pick] = new
    return x


@pytest.mark.parametrize("protocol", ["supersteps", "rounds"])
@pytest.mark.parametrize("nranks,S,P,fanin", [(2, 30, 8, 32), (4, 100, 4, 8)])
def test_bench_layout_pieces_match_global_dag(nranks, S, P, fanin, protocol):
    G, ga, owner, roots, trees, groot = PC.global_c4(S, P, nranks, fanin=fanin)
    changes = _changes(len(G.file_slots), np.random.default_rng(7), (0.01, 0.25))
    pcs = [PartitionedDag1000(S, P, nranks, r, fanin=fanin) for r in range(nranks)]

    def setup(r, ctx):
        pc = pcs[r]
        f0, nf = 2 * pc.dag.Q * r, 2 * pc.dag.Q
        g = capi.Graph.from_arrays(ctx, pc.desc)
        g.set_part(_part(pc.part, protocol))

        def to_local(pick, new):
            sel = (pick >= f0) & (pick < f0 + nf)
            return pc.dag.file_slots[pick[sel] - f0], new[sel]
        return g, int(pc.desc["n_slots"]), (pc.dag.file_slots, G.leaf_ids[f0:f0 + nf]), to_local

    res = _run(setup, nranks, changes)
    wants = [PC.global_digests(G, ga, x) for x in _states(G.leaf_ids, changes)]
    for r, out in enumerate(res):
        m = PC.c4_local_to_global(pcs[r], G, roots, trees, groot)
        for step, ((n, slots, supersteps), want) in enumerate(zip(out, wants)):
            assert (slots == want[m]).all(), (r, step)
            assert supersteps == (2 if protocol == "rounds" or step != 3 else 1)
        # ranks > 0 have no imports: their second superstep launches nothing
        assert r == 0 or out[1][0] > 0


@pytest.mark.parametrize("nranks,nparts", [(2, 4), (4, 4), (2, 2)])
def test_strong_layout_counts_match_dirty_work(nranks, nparts):
    """bench.py's strong layout (nparts fixed, nranks | nparts): each rank's
    jobs hashed by an incremental step equal the layout's dirty closure
    (PartitionedDag1000.dirty_work) plus the jobs hashed twice (rank 0's
    global root: local pass, then after the exchange).  A part cannot be
    re-attached while a change set is pending."""
    S, P = 12, 4
    nf = 2 * P * S * nparts

    def setup(r, ctx):
        pc = PartitionedDag1000(S, P, nranks, r, fanin=4, nparts=nparts)
        g = capi.Graph.from_arrays(ctx, pc.desc)
        g.set_part(pc.part)
        return g, pc

    def body(r, ag):
        ctx = capi.Context(0, host_threads=0)
        try:
            g, pc = setup(r, ctx)
            g.set_slots(pc.dag.file_slots, pc.dag.leaf_ids)
            g.recompute_part(allgather=ag, nranks=nranks, full=True)
            sl, _, nw = pc.dag.change_set(0.05, n_global=nf)
            if len(sl):
                g.set_slots(sl, nw)
                #  no part attached inside a step: the change set is pending
                with pytest.raises(capi.RfError) as e:
                    g.set_part(pc.part)
                assert e.value.code == capi.RF_EPRECONDITION
            got = g.recompute_part(allgather=ag, nranks=nranks)
            jobs, _, _ = pc.dirty_work(sl)
            g.close()
            return got, jobs + pc.last_twice
        finally:
            ctx.close()

    for got, want in PC.run_threads(nranks, body):
        assert got == want
