"""configs[3]'s 100M-node DAG at full size on the one GPU a box has.

The DAG is the one bench.py partitions (workloads.PartitionedDag1000, SURVEY
§8(e)): a 1000align DAG of 8 x 27,594 samples (P = 32, 100M nodes, 121.6M
jobs, 15.5 GB of templates), each rank's sample roots merged by a fan-in-32
Merge tree, the global root merging the 8 rank roots
(partition_case.global_c4 builds the whole of it).

  (a) one rank holds all of it: after 1% of the leaf File IDs change, the
      incremental recompute equals a full recompute slot for slot (121.6M
      jobs), and it hashes exactly the dirty closure (per changed leaf, pair
      and sample, plus the Merge-tree ancestors and the global root).
  (b) the same DAG as bench.py's 8 per-rank pieces, 8 ranks as threads with a
      context each on the one GPU, the boundary exchanged through a host
      all-gather (RCCL needs one GPU per rank): every rank's slots equal
      (a)'s, before and after the change.

  (c) the oracle ((a) and (b) alone compare the engine with
      itself): after the change, every one of the 121.6M jobs re-derived on
      the host from its own hole digests in the table (the oracle's job-local
      check, orc_graph_check, 16 threads) -- and the input slots hold the
      changed File IDs.

The oracle's CPU evaluator would take minutes per full pass at this size; the
job-local check takes seconds, and the oracle pins the same generator and
protocol end to end at small sizes (test_gpu_partition.py, test_gpu_dag.py,
test_gpu_scale.py's configs[2])."""
import numpy as np
import pytest

import partition_case as PC
import reflow_oracle as O
from reflow_amd import capi
from reflow_amd.workloads import PartitionedDag1000

pytestmark = pytest.mark.gpu

S_RANK, P, NR, FANIN = 27594, 32, 8, 32


@pytest.fixture(scope="module")
def c4():
    G, ga, owner, roots, trees, groot = PC.global_c4(S_RANK, P, NR, fanin=FANIN)
    assert G.n_nodes + sum(len(t) for t in trees) + 1 >= 100_000_000
    slots, old, new = G.change_set(0.01)
    return dict(G=G, a=ga, roots=roots, trees=trees, groot=groot, change=(slots, old, new))


def _expected_dirty(G, slots):
    """The dirty closure's job count for the changed leaf files `slots`."""
    pair = slots // 2
    sample = np.unique(pair // P)
    n = 2 * len(slots) + len(np.unique(pair)) * 11 + len(sample) * 5
    # Merge-tree ancestors, per rank (fan-in FANIN over the rank's samples)
    for r in range(NR):
        loc = sample[(sample >= r * S_RANK) & (sample < (r + 1) * S_RANK)] - r * S_RANK
        width = S_RANK
        while width > 1:
            loc = np.unique(loc // FANIN)
            n += len(loc)
            width = (width + FANIN - 1) // FANIN
    return n + 1  # the global root


def test_configs3_single_rank_incremental_equals_full(c4):
    G, a = c4["G"], c4["a"]
    slots, old, new = c4["change"]
    ctx = capi.Context(0, host_threads=0)
    try:
        g = capi.Graph.from_arrays(ctx, a)
        g.set_slots(G.file_slots, G.leaf_ids)
        assert g.recompute(full=True) == len(a["out_slot"])
        every = np.arange(a["n_slots"], dtype=np.uint32)
        c4["base"] = g.get_slots(every)
        g.set_slots(slots, new)
        n_inc = g.recompute(full=False)
        inc = g.get_slots(every)
        assert n_inc == _expected_dirty(G, slots), n_inc
        g.recompute(full=True)
        assert (g.get_slots(every) == inc).all(), "incremental != full recompute"
        c4["after"] = inc
        # (c) the oracle, job by job over the whole table, and the inputs
        ids = G.leaf_ids.copy()
        order = np.argsort(G.file_slots, kind="stable")
        pos = order[np.searchsorted(G.file_slots[order], slots)]
        assert (G.file_slots[pos] == slots).all()
        ids[pos] = new
        assert (inc[G.file_slots] == ids).all(), "input slots"
        bad, first = O.check_slots(a, inc, 16)
        assert bad == 0, ("oracle: jobs whose digest is not the hash of their material", bad, first)
        # and back: the old IDs restore the original digests
        g.set_slots(slots, old)
        g.recompute(full=False)
        assert (g.get_slots(c4["trees"][0]) == c4["base"][c4["trees"][0]]).all()
        assert (g.get_slots([c4["groot"]]) == c4["base"][[c4["groot"]]]).all()
        g.close()
    finally:
        ctx.close()


def test_configs3_eight_pieces_match_single_rank(c4):
    if "after" not in c4:
        pytest.skip("needs the single-rank result")
    G = c4["G"]
    slots, old, new = c4["change"]
    Q = S_RANK * P

    def body(r, ag):
        pc = PartitionedDag1000(S_RANK, P, NR, r, fanin=FANIN)
        m = PC.c4_local_to_global(pc, G, c4["roots"], c4["trees"], c4["groot"])
        f0 = 2 * Q * r
        sel = (slots >= f0) & (slots < f0 + 2 * Q)
        ctx = capi.Context(0, host_threads=0)
        try:
            g = capi.Graph.from_arrays(ctx, pc.desc)
            g.set_part(pc.part)
            g.set_slots(pc.dag.file_slots, pc.dag.leaf_ids)
            every = np.arange(int(pc.desc["n_slots"]), dtype=np.uint32)
            g.recompute_part(allgather=ag, nranks=NR, full=True)
            ok0 = bool((g.get_slots(every) == c4["base"][m]).all())
            g.set_slots(pc.dag.file_slots[slots[sel] - f0], new[sel])
            g.recompute_part(allgather=ag, nranks=NR)
            ok1 = bool((g.get_slots(every) == c4["after"][m]).all())
            steps = g.part_gathered()[2]
            g.close()
            return ok0, ok1, steps
        finally:
            ctx.close()

    res = PC.run_threads(NR, body)
    for r, (ok0, ok1, steps) in enumerate(res):
        assert ok0, (r, "full recompute")
        assert ok1, (r, "incremental")
        assert steps == 2  # the local pass + the layout's one fixed exchange round
