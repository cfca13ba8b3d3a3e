"""Multi-rank host logic of bench.py on the CPU (gloo, world_size 2).

The GPU data path (RCCL inside libreflow_hip.so) cannot run here; these tests
cover what every rank does around it: rendezvous on 127.0.0.1, barrier,
max-over-ranks timing, the RCCL unique-id broadcast, and that ranks get
disjoint weak-scaling shards (distinct seeds -> distinct files / DAGs)."""
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
    seed = 0x5EED0004 + rank
    lens = c2_sizes(total_bytes=1 << 30, seed=seed)
    dag = Dag1000(3, 4, seed=0x5EED0003 + 1000003 * rank)
    q.put((rank, mx, sm, uid, int(lens.sum()), lens[:8].tolist(), dag.leaf_ids[:2].tobytes(), ag))
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
    (r0, mx0, sm0, uid0, b0, l0, ids0, ag0), (r1, mx1, sm1, uid1, b1, l1, ids1, ag1) = res
    assert ag0 == ag1 == [7, 7, 7, 8, 8, 8]  # rank order
    assert mx0 == mx1 == 2.0  # max over ranks
    assert sm0 == sm1 == 30.0  # whole-job aggregate
    assert uid0 == uid1 == b"U" * 128  # RCCL id reaches every rank
    assert b0 == b1 == 1 << 30  # equal per-rank work (weak scaling)
    assert l0 != l1 and ids0 != ids1  # disjoint shards


def test_or_allreduce_semantics():
    """rf_comm_allreduce_or = all-gather + OR (RCCL has no bitwise OR); the
    CPU restatement over 4 simulated ranks."""
    rng = np.random.default_rng(0)
    ranks = [rng.integers(0, 2**63, size=17, dtype=np.uint64) for _ in range(4)]
    gathered = np.stack(ranks)
    want = ranks[0] | ranks[1] | ranks[2] | ranks[3]
    assert (np.bitwise_or.reduce(gathered, axis=0) == want).all()
