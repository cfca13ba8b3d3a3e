"""Multi-rank host logic on the CPU (gloo, world_size 2).

The GPU data path (RCCL inside libreflow_hip.so) cannot run here; these tests
cover what every rank does around it: rendezvous on 127.0.0.1, barrier,
max-over-ranks timing, the RCCL unique-id broadcast, the LPT sharding of the
global Fileset, and -- the partitioned DAG -- the product's splitter
(rf_graph_split, host code in libreflow_hip.so) with the superstep exchange
protocol of rf_graph_recompute_part (boundary-bitset OR all-reduce +
all-gather of boundary digests over gloo), each rank's local recompute done by
the oracle, checked slot for slot against a single-rank recompute."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from reflow_amd.workloads import Dag1000, c2_sizes
    d = bench.Dist(world)
    d.barrier()
    mx = d.max(1.0 + rank)
    sm = d.sum(10.0 * (rank + 1))
    uid = d.bcast_bytes(b"U" * 128 if rank == 0 else None)
    ag = d.all_gather_bytes(np.full(3, 7 + rank, dtype=np.uint8)).tolist()  # root-digest exchange without RCCL
    class A:
        sha_gib = 1.0
    lens, _, glob = bench.rank_sizes(A, d)  # LPT shard of the global Fileset
    allsz = np.concatenate([c2_sizes(total_bytes=1 << 30, seed=0x5EED0004 + g) for g in range(world)])
    dag = Dag1000(3, 4, seed=0x5EED0003 + 1000003 * rank)
    q.put((rank, mx, sm, uid, int(lens.sum()), sorted(lens.tolist()), dag.leaf_ids[:2].tobytes(), ag,
           glob["files"], int(allsz.sum()), sorted(allsz.tolist())))
    d.dist.destroy_process_group()


def test_gloo_world2_bench_dist():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, mx0, sm0, uid0, b0, l0, ids0, ag0, n0, tot0, all0), (r1, mx1, sm1, uid1, b1, l1, ids1, ag1, n1, tot1, _) = res
    assert ag0 == ag1 == [7, 7, 7, 8, 8, 8]  # rank order
    assert mx0 == mx1 == 2.0  # max over ranks
    assert sm0 == sm1 == 30.0  # whole-job aggregate
    assert uid0 == uid1 == b"U" * 128  # RCCL id reaches every rank
    # the LPT shards partition the global Fileset and balance its bytes
    assert sorted(l0 + l1) == all0 and b0 + b1 == tot0 and n0 == n1 == len(all0)
    assert abs(b0 - b1) <= max(l0 + l1)
    assert ids0 != ids1  # per-rank DAG seeds differ


def _part_worker(rank, world, port, q, protocol="rounds"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "oracle"), os.path.join(root, "tests")]
    import torch
    import torch.distributed as dist

    import partition_case as PC
    from reflow_amd import capi
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(b):
        t = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        return [o.numpy().tobytes() for o in out]

    dag, arrays, owner, root_slot, tail_slot = PC.global_case(S=6, P=4, nranks=world)
    piece = capi.GraphPiece(arrays, world, rank, owner)
    if protocol == "supersteps":
        piece.part = dict(piece.part, rounds=0)
    ids = dag.leaf_ids.copy()
    state, steps1 = PC.superstep_oracle(piece.desc, piece.part, allgather, inputs=PC.piece_inputs(piece, dag, ids))
    first = state["og"].slots[:len(piece.global_of_local)].copy()
    # change 1/3 of the leaf files, including ones of every sample
    rng = np.random.default_rng(3)
    pick = np.sort(rng.choice(len(dag.file_slots), size=len(dag.file_slots) // 3, replace=False))
    new = ids.copy()
    new[pick] = rng.integers(0, 256, size=(len(pick), 32), dtype=np.uint8)
    state, steps2 = PC.superstep_oracle(piece.desc, piece.part, allgather,
                                        changed=PC.piece_inputs(piece, dag, new, pick), state=state)
    second = state["og"].slots[:len(piece.global_of_local)].copy()
    q.put((rank, piece.global_of_local.tolist(), first.tobytes(), second.tobytes(), steps1, steps2,
           len(piece.part["import_slot"]), len(piece.part["export_slot"]), piece.part["any_import"]))
    dist.destroy_process_group()


@pytest.mark.parametrize("protocol", ["supersteps", "rounds"])
def test_gloo_world2_partitioned_dag(protocol):
    """One DAG over 2 ranks: every rank's local slots equal the single-rank
    recompute, before and after an incremental change, and the change crosses
    ranks twice (global root on rank 0, its consumer on rank 1) -- with the
    superstep exchange and with the splitter's fixed rounds."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import partition_case as PC
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_part_worker, args=(r, 2, port, q, protocol)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dag, arrays, owner, root_slot, tail_slot = PC.global_case(S=6, P=4, nranks=2)
    want1 = PC.global_digests(dag, arrays, dag.leaf_ids)
    rng = np.random.default_rng(3)
    pick = np.sort(rng.choice(len(dag.file_slots), size=len(dag.file_slots) // 3, replace=False))
    new = dag.leaf_ids.copy()
    new[pick] = rng.integers(0, 256, size=(len(pick), 32), dtype=np.uint8)
    want2 = PC.global_digests(dag, arrays, new)
    covered = set()
    for rank, g, first, second, steps1, steps2, n_imp, n_exp, any_imp in res:
        g = np.array(g)
        assert (np.frombuffer(first, np.uint8).reshape(-1, 32) == want1[g]).all(), rank
        assert (np.frombuffer(second, np.uint8).reshape(-1, 32) == want2[g]).all(), rank
        assert any_imp and n_imp > 0 and n_exp > 0
        assert steps2 >= 3  # sample roots -> global root (rank 0) -> tail (rank 1) -> quiet
        covered |= set(g.tolist())
    assert covered == set(range(arrays["n_slots"]))  # every slot lives on some rank
