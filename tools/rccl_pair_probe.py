"""Probe: can RCCL build a communicator of two ranks that share one GPU?
(The 1-GPU box is the only place rf_comm_* can run with > 1 rank.)
Launch: python -m torch.distributed.run --nnodes=1 --nproc-per-node 2
        --master-addr 127.0.0.1 --master-port 29511 tools/rccl_pair_probe.py
Each rank all-gathers 32 B x 5 of its own pattern and OR-reduces a bitset
through the engine's rf_comm_*; rank 0 prints one JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch.distributed as dist
    from reflow_amd import capi
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = capi.Context(0, host_threads=0)
    obj = [capi.Comm.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    res = {"rank": rank, "world": world}
    try:
        comm = capi.Comm(ctx, world, rank, obj[0])
    except Exception as e:  # noqa: BLE001 - the probe reports whatever RCCL says
        res["init"] = "failed: %s" % e
        comm = None
    if comm is not None:
        res["init"] = "ok"
        mine = np.full(32 * 5, rank + 1, dtype=np.uint8)
        src, dst = ctx.upload(mine), ctx.alloc(32 * 5 * world)
        comm.allgather(src.ptr, dst.ptr, 32 * 5, ctx.stream)
        ctx.sync()
        got = dst.to_numpy().reshape(world, -1)
        res["allgather_ok"] = bool(all((got[r] == r + 1).all() for r in range(world)))
        words = np.zeros(64, dtype=np.uint64)
        words[rank] = np.uint64(1) << np.uint64(rank)
        d = ctx.upload(words)
        comm.allreduce_or(d.ptr, len(words), ctx.stream)
        ctx.sync()
        w = d.to_numpy(np.uint64)
        want = np.zeros(64, dtype=np.uint64)
        for r in range(world):
            want[r] = np.uint64(1) << np.uint64(r)
        res["or_ok"] = bool((w == want).all())
        comm.close()
    out = [None] * world
    dist.all_gather_object(out, res)
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
