#!/usr/bin/env python3
"""bench.py -- Reflow memoization hot path on MI355X (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W

Primary line (value): SHA-256 digest GB/s of configs[1], the 64 GiB
FASTQ/BAM-like skewed Fileset (4 KiB-2 GiB files), HBM-resident, on each GPU
(weak scaling: every rank digests its own 64 GiB set).  A step = one
rf_sha_plan_run over the whole set (all File IDs of the Fileset).

Secondary, in the same JSON line:
  "incremental"  configs[2]: 10M-node 1000align DAG, 1% of leaf File IDs
                 changed per step -> K3 frontier + K2 recompute (Mnodes/s of
                 dirty nodes, and effective graph nodes/s); RCCL all-gather of
                 the per-rank root digests when N > 1.
  "probe"        configs[4]: 1e9 bloomlive probes against a 1e8-key filter.
  "cpu_baseline" the oracle's C port on the host cores (rank 0, N=1).

The only process-wide runtime is the engine's own (libreflow_hip.so); torch is
used only for torch.distributed (gloo, CPU) to bootstrap RCCL and to take the
max over ranks.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from reflow_amd import capi  # noqa: E402
from reflow_amd.workloads import Dag1000, GiB, arena_layout, c2_sizes  # noqa: E402

# ---- hardware constants (MI355X_MICROARCH.md) ------------------------------
CLOCK_HZ = 2.4e9
N_CU = 256
VALU_LANE_OPS = N_CU * 4 * 32 * CLOCK_HZ      # int32 VALU lane-ops/s (= FP32 FMA rate)
SHA_OPS_PER_BLOCK = 1464                        # canonical ops per 64-B block
SHA_VALU_PEAK_GBS = VALU_LANE_OPS / SHA_OPS_PER_BLOCK * 64 / 1e9
# A message's blocks are a serial chain (Merkle-Damgard).  One round's critical
# path is 3 dependent VALU ops (rotate -> xor3 -> add3 into e/a); the
# dependent-issue latency of one wave is 4 cycles (MI355X_MICROARCH.md,
# "Dependent-chain latency"; tools/micro.py lat: 4-5).  So no implementation
# can finish a message of B blocks in less than B * 64 * 3 * 4 cycles.
CHAIN_CYCLES_PER_BLOCK = 64 * 3 * 4
HBM_PEAK_GBS = 8000.0


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3
    --pmc FETCH_SIZE/WRITE_SIZE summary (tools/pmc_summary.py, corrected as
    MI355X_MICROARCH.md prescribes), or None.  The PMC passes run the same
    default workloads as this script."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")))
    if not paths:
        return None, None
    d = json.load(open(paths[-1]))
    v = d.get("rf::" + kernel)
    if not v:
        return None, None
    # the bench prices the kernel's largest launch (the mean over dispatches
    # would mix in small launches of other workloads)
    return v.get("traffic_bytes_largest_launch", v["traffic_bytes_per_launch"]), os.path.relpath(paths[-1], ROOT)


class Dist:
    def __init__(self, n_gpus):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # gloo prints "[Gloo] Rank r is connected ..." on the C-level
            # stdout: keep stdout for the one JSON line (send it to stderr)
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
                dist.barrier()
            finally:
                os.dup2(saved, 1)
                os.close(saved)
            self.dist = dist
        if n_gpus != self.world and self.world > 1:
            log("warning: --gpus %d but WORLD_SIZE %d" % (n_gpus, self.world))

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, x):
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x):
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def bcast_bytes(self, b):
        if self.world == 1:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def all_gather_bytes(self, arr):
        """Host all-gather over gloo (the exchange when no RCCL communicator
        could be created)."""
        import torch
        t = torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).copy())
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return np.concatenate([o.numpy() for o in out])


def timed_steps(dist, ctx, fn, steps, warmup):
    for _ in range(warmup):
        fn()
    ctx.sync()
    dist.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for i in range(steps):
        fn()
        if steps > 2:
            pass
    ctx.sync()
    dist.barrier()
    t1 = time.perf_counter()
    return dist.max(t1 - t0)


# ---------------------------------------------------------------- C2: SHA --
def bench_sha(args, dist, ctx):
    seed = 0x5EED0002 if dist.world == 1 else 0x5EED0004 + dist.rank
    total = int(args.sha_gib * GiB)
    lens = c2_sizes(total_bytes=total, seed=seed)
    offs, arena_bytes = arena_layout(lens)
    arena = ctx.alloc(arena_bytes)
    d_offs, d_lens = ctx.upload(offs), ctx.upload(lens)
    out = ctx.alloc(32 * len(lens))
    ctx.gen_fill(arena.ptr, d_offs.ptr, d_lens.ptr, len(lens), seed, arena_bytes)
    ctx.sync()
    plan = ctx.sha_plan(offs, lens, 0)
    st = plan.stats()
    log("C2: %d files, %.1f GiB, %d wave-per-message, max file %.2f GiB"
        % (len(lens), lens.sum() / GiB, st.n_solo, lens.max() / GiB))
    solo_ms, lanes_ms = [], []

    def step():
        plan.run(arena.ptr, out.ptr)
        s = plan.stats()  # synchronises: per-kernel HIP-event times of this run
        solo_ms.append(s.last_ms_solo)
        lanes_ms.append(s.last_ms_lanes)
        log("  sha step: total %.1f ms (solo %.1f, lanes %.1f)" % (s.last_ms_total, s.last_ms_solo,
                                                                    s.last_ms_lanes))

    t = timed_steps(dist, ctx, step, args.steps, args.warmup)
    solo_ms, lanes_ms = solo_ms[args.warmup:], lanes_ms[args.warmup:]
    bytes_all = dist.sum(float(lens.sum())) * args.steps
    gbs = bytes_all / t / 1e9
    # roofline of the dominant kernel (the longer of solo / lanes)
    order = np.argsort(-lens.astype(np.int64), kind="stable")
    solo_ids = order[:st.n_solo]
    lane_ids = order[st.n_solo:]
    nblk = (lens.astype(np.int64) + 9 + 63) // 64
    # dominant kernel: the one that holds the largest message (its chain is the
    # critical path); wave-per-message runs k1_sha256_duo by default
    wave_mode = st.n_solo > 0
    dom = "k1_sha256_duo" if wave_mode else "k1_sha256_lanes"
    ids = solo_ids if wave_mode else lane_ids
    dom_ms = float(np.mean(solo_ms if wave_mode else lanes_ms))
    dom_bytes = float(lens[ids].sum())
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    # skew-aware floor: the longest serial chain (critical-path latency) vs
    # chip VALU throughput
    t_chain = float(nblk[ids].max()) * CHAIN_CYCLES_PER_BLOCK / CLOCK_HZ
    t_valu = float(nblk[ids].sum()) * SHA_OPS_PER_BLOCK / VALU_LANE_OPS
    t_floor = max(t_chain, t_valu)
    peak = dom_bytes / t_floor / 1e9
    traffic, tsrc = pmc_traffic(dom)
    roof = {"bound": "valu", "kernel": dom, "achieved": round(achieved, 3), "peak": round(peak, 3),
            "unit": "GB/s", "frac": round(achieved / peak, 4), "traffic": traffic,
            "traffic_source": tsrc, "traffic_over_algorithmic": (round(traffic / dom_bytes, 3)
                                                                 if traffic else None),
            "peak_kind": "skew-aware floor: max(longest message's blocks x 64 rounds x 3 dependent VALU"
                         " x 4 cyc @2.4GHz (round critical path), sum blocks x 1464 ops / INT32 VALU peak)",
            "floor_s": round(t_floor, 3), "chain_floor_s": round(t_chain, 3),
            "valu_peak_GBps": round(SHA_VALU_PEAK_GBS, 1),
            "frac_of_valu_peak": round(achieved / SHA_VALU_PEAK_GBS, 6),
            "launch_ms": round(dom_ms, 3), "bytes_per_launch": dom_bytes,
            "critical_chain_blocks": int(nblk[ids].max())}
    res = dict(value=gbs, ms_per_step=t / args.steps * 1e3, roofline=roof,
               files=int(len(lens)), bytes_per_gpu=int(lens.sum()), n_solo=int(st.n_solo),
               lanes_ms=float(np.mean(lanes_ms)) if lanes_ms else 0.0)
    # keep digests of a host-checkable sample for the cpu_baseline cross-check
    res["_digests"] = out.to_numpy().reshape(-1, 32)
    res["_lens"], res["_seed"] = lens, seed
    plan.close()
    for b in (arena, d_offs, d_lens, out):
        b.free()
    return res


# -------------------------------------------------- C1: reference config --
C1_N, C1_LEN, C1_SEED = 4096, 262144, 0x5EED0001


def c1_path(i):
    return ("d%02d/f%04d.fq.gz" % (i // 64, i)).encode()


def bench_c1(args, dist, ctx):
    """configs[0], the reference's own CPU-runnable case, on the GPU: digest
    1 GiB = 4096 x 256 KiB files (HBM-resident, File IDs on K1), the Fileset
    digest of the 4096-entry map (executor.go:205-233; host material + K1,
    File IDs read back), and CacheKeys of a ~10k-node 1000align DAG (K2 full
    recompute).  Checked against the committed fixture tests/golden/c1_fileset.json."""
    lens = np.full(C1_N, C1_LEN, dtype=np.uint64)
    offs, arena_bytes = arena_layout(lens)
    arena = ctx.alloc(arena_bytes)
    d_offs, d_lens = ctx.upload(offs), ctx.upload(lens)
    out = ctx.alloc(32 * C1_N)
    ctx.gen_fill(arena.ptr, d_offs.ptr, d_lens.ptr, C1_N, C1_SEED, arena_bytes)
    ctx.sync()
    plan = ctx.sha_plan(offs, lens, 0)
    plan.run(arena.ptr, out.ptr)
    ctx.sync()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        plan.run(arena.ptr, out.ptr)
    ctx.sync()
    ids_ms = (time.perf_counter() - t0) / reps * 1e3
    # Fileset digest over the IDs where K1 left them (rf_fileset_digest_device:
    # path material from the host, IDs placed on the device); the paths are
    # marshalled once, outside the timed region
    fp = ctx.fileset_paths([[[c1_path(i) for i in range(C1_N)]]])
    fp.digest_device(out.ptr)
    t0 = time.perf_counter()
    for _ in range(reps):
        fsd = fp.digest_device(out.ptr)[0]
    fs_ms = (time.perf_counter() - t0) / reps * 1e3
    # the host-ID form (IDs read back, rf_fileset_digest_batch), for comparison
    t0 = time.perf_counter()
    ids = out.to_numpy().reshape(-1, 32)
    d2h_ms = (time.perf_counter() - t0) * 1e3
    group = [[[(c1_path(i), ids[i].tobytes()) for i in range(C1_N)]]]  # harness-side argument building
    ctx.fileset_digest_batch(group)
    t0 = time.perf_counter()
    fsd_host = ctx.fileset_digest_batch(group)[0]
    fs_host_ms = (time.perf_counter() - t0) * 1e3 + d2h_ms
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "c1_fileset.json")))
    ok = ("sha256:" + fsd.hex() == want["fileset_digest"] and fsd_host == fsd and
          __import__("hashlib").sha256(ids.tobytes()).hexdigest() == want["ids_sha256"])
    inst = (bench_c1_install(ctx, arena, offs, fsd, cpu_leg=dist.world == 1 and "cpu" not in args.skip)
            if "install" not in args.skip and dist.rank == 0 else None)
    plan.close()
    for b in (arena, d_offs, d_lens, out):
        b.free()
    # CacheKeys over a ~10k-node DAG (S*(14P+5) nodes at P=32)
    small = Dag1000(22, 32)
    a = small.arrays()
    g = capi.Graph(ctx, a["n_slots"], a["out_slot"], a["tmpl_off"], a["tmpl_len"], a["hole_ptr"],
                   a["hole_pos"], a["hole_slot"], a["blob"])
    g.set_slots(small.file_slots, small.leaf_ids)
    g.recompute(full=True)  # captures the hipGraph
    ctx.timer_start()
    for _ in range(reps):
        g.recompute(full=True)
    dag_ms = ctx.timer_stop() / reps
    g.close()
    return {"workload": "configs[0]: 4096 x 256 KiB files (1 GiB) -> File IDs + Fileset digest; CacheKeys "
                        "of a %d-node 1000align DAG (%d jobs)" % (small.n_nodes, small.n_jobs),
            "file_ids_ms": ids_ms, "file_ids_gbps": C1_N * C1_LEN / (ids_ms * 1e-3) / 1e9,
            "fileset_digest_ms": fs_ms, "fileset_digest_note": "rf_fileset_digest_device: bytewise sort and path "
            "material on the host, IDs placed from HBM, one %d-block message on the duo chain" % ((C1_N * 49 + 9 + 63) // 64),
            "fileset_digest_host_ids_ms": fs_host_ms,
            "fixture_match": ok,
            "dag_nodes": small.n_nodes, "dag_full_recompute_ms": dag_ms,
            "total_ms": ids_ms + fs_ms + dag_ms,
            "install": inst,
            "note": "4096 messages on 512 k1_sha256_octo chain waves (eight files per wave): the per-file "
                    "chain (4097 blocks x ~1.2 us) bounds the file-ID time, not chip throughput"}


def bench_c1_install(ctx, arena, offs, want_fsd, cpu_leg=False):
    """configs[0] from files: the same 4096 x 256 KiB contents written as a
    tree d%02d/f%04d.fq.gz, then Executor.install over it (rf_install_dir:
    walk, read on <=60 host threads into pinned memory, H2D, K1, Fileset
    digest) -- page-cache-warm reads, so storage speed is not measured."""
    import shutil
    import tempfile
    host = arena.to_numpy()
    root = tempfile.mkdtemp(prefix="rf_c1_")
    try:
        for i in range(C1_N):
            p = os.path.join(root, c1_path(i).decode())
            os.makedirs(os.path.dirname(p), exist_ok=True)
            with open(p, "wb") as f:
                f.write(host[int(offs[i]):int(offs[i]) + C1_LEN].tobytes())
        del host
        ctx.install_dir(root)  # warm-up (stage allocation, plan)
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            ents, fsd = ctx.install_dir(root)
        ms = (time.perf_counter() - t0) / reps * 1e3
        res = {"what": "rf_install_dir over the configs[0] tree on local disk (page cache warm)",
               "ms": ms, "gbps": C1_N * C1_LEN / (ms * 1e-3) / 1e9, "entries": len(ents),
               "fileset_digest_match": fsd == want_fsd}
        if cpu_leg:  # the same install on the host: read + hashlib (OpenSSL) SHA-256, 16 threads
            import hashlib
            from concurrent.futures import ThreadPoolExecutor
            paths = [os.path.join(root, c1_path(i).decode()) for i in range(C1_N)]

            def one(p):
                with open(p, "rb") as f:
                    return hashlib.sha256(f.read()).digest()
            with ThreadPoolExecutor(16) as ex:
                t0 = time.perf_counter()
                cpu_ids = list(ex.map(one, paths))
                cms = (time.perf_counter() - t0) * 1e3
            res["cpu_openssl_16t"] = {"ms": cms, "gbps": C1_N * C1_LEN / (cms * 1e-3) / 1e9, "cores": 16,
                                      "ids_match": cpu_ids == [e[1] for e in ents]}
    finally:
        shutil.rmtree(root, ignore_errors=True)
    return res


# ------------------------------------------------------- C3: incremental --
def bench_dag(args, dist, ctx, comm):
    S = args.dag_samples
    t0 = time.perf_counter()
    dag = Dag1000(S, args.dag_pairs, seed=0x5EED0003 + 1000003 * dist.rank)
    a = dag.arrays()
    g = capi.Graph(ctx, a["n_slots"], a["out_slot"], a["tmpl_off"], a["tmpl_len"], a["hole_ptr"],
                   a["hole_pos"], a["hole_slot"], a["blob"])
    del a
    g.set_slots(dag.file_slots, dag.leaf_ids)
    log("C3: %d nodes, %d jobs built+loaded in %.1f s" % (dag.n_nodes, dag.n_jobs, time.perf_counter() - t0))
    g.recompute(full=True)  # first call also captures the hipGraphs (host work): untimed
    ctx.timer_start()
    g.recompute(full=True)
    full_ms = ctx.timer_stop()
    slots, old, new = dag.change_set(0.01)
    d_slots = ctx.upload(slots)
    d_old, d_new = ctx.upload(old), ctx.upload(new)
    roots = dag.kinds["XS"].out_slot
    d_roots_idx = ctx.upload(roots)
    d_gather = ctx.alloc(32 * len(roots) * max(dist.world, 1))
    d_local = ctx.alloc(32 * len(roots))
    # one counted step to learn the dirty-set size
    g.set_slots(slots, new)
    n_dirty_jobs = g.recompute(full=False)
    g.set_slots(slots, old)
    g.recompute(full=False)
    pairs = np.unique(slots // 2)
    n_dirty_nodes = n_dirty_jobs - len(pairs)  # minus the pE1 physical keys
    state = {"v": 0}

    def step():
        ver = d_new if state["v"] == 0 else d_old
        state["v"] ^= 1
        g.set_slots_device(d_slots.ptr, ver.ptr, len(slots), ctx.stream)
        g.recompute_async(False, ctx.stream)
        if dist.world > 1:  # boundary digests (per-sample roots) to every rank
            g.gather_device(d_roots_idx.ptr, len(roots), d_local.ptr, ctx.stream)
            if comm is not None:
                comm.allgather(d_local.ptr, d_gather.ptr, 32 * len(roots), ctx.stream)
            else:  # no RCCL communicator (see main): same exchange through the host
                ctx.sync()
                dist.all_gather_bytes(d_local.to_numpy())

    steps = args.dag_steps
    t = timed_steps(dist, ctx, step, steps, 2)
    ctx.timer_start()
    for _ in range(steps):
        step()
    dev_ms = ctx.timer_stop() / steps
    total_dirty_nodes = dist.sum(n_dirty_nodes) * steps
    res = {"workload": "1000align DAG S=%d P=%d per GPU, 1%% leaf File IDs toggled per step" % (S, args.dag_pairs),
           "nodes_per_gpu": dag.n_nodes, "jobs_per_gpu": dag.n_jobs,
           "dirty_nodes_per_step": int(n_dirty_nodes), "dirty_jobs_per_step": int(n_dirty_jobs),
           "ms_per_step": t / steps * 1e3, "device_ms_per_step": dev_ms,
           "mnodes_per_s": total_dirty_nodes / t / 1e6,
           "effective_mnodes_per_s": dist.sum(dag.n_nodes) * steps / t / 1e6,
           "full_recompute_ms": full_ms,
           "full_recompute_mnodes_per_s": dag.n_nodes / (full_ms * 1e-3) / 1e6,
           "levels": g.stats().n_levels}
    # full-recompute roofline (VALU): all template blocks hashed
    st = g.stats()
    ach = st.total_blocks * 64 / (full_ms * 1e-3) / 1e9
    res["roofline_full"] = {"bound": "valu", "achieved": round(ach, 2), "peak": round(SHA_VALU_PEAK_GBS, 1),
                            "unit": "GB/s", "frac": round(ach / SHA_VALU_PEAK_GBS, 4)}
    res["canonicalize"] = bench_canon(ctx, g, dag)
    g.close()
    return res, dag


def bench_canon(ctx, g, dag):
    """K5: Canonicalize's flowMap over every node digest of the C3 DAG, as a
    program that builds the shared reference-index chain (Intern -> Exec(bwa
    index) -> Coerce) once per sample would hand it to Flow.Canonicalize: S
    copies of those three nodes, then every other node, in construction order
    (each kind reads only earlier ones)."""
    ref = np.concatenate([dag.kinds[k].out_slot for k in ("R0", "R1", "R2")]).astype(np.uint32)
    rest = [np.asarray(k.out_slot, dtype=np.uint32) for name, k in dag.kinds.items()
            if name not in ("R0", "R1", "R2") and not name.startswith("p")]  # logical digests only
    slots = np.concatenate([np.tile(ref, dag.S)] + rest)
    n = len(slots)
    d_idx = ctx.upload(slots)
    d_dig, d_canon, d_nu = ctx.alloc(32 * n), ctx.alloc(4 * n), ctx.alloc(64)
    g.gather_device(d_idx.ptr, n, d_dig.ptr, ctx.stream)
    ctx.dedup_digests_device(d_dig.ptr, n, d_canon.ptr, d_nu.ptr)  # warm (allocates the table)
    times = []
    for _ in range(5):
        ctx.timer_start()
        ctx.dedup_digests_device(d_dig.ptr, n, d_canon.ptr, d_nu.ptr)
        times.append(ctx.timer_stop())
    nu = int(d_nu.to_numpy()[:4].view(np.uint32)[0])
    canon = d_canon.to_numpy().view(np.uint32)
    ms = float(np.median(times))
    # every ref copy maps to the first; no other duplicates in the 1000align DAG
    ok = nu == dag.n_nodes and n == dag.n_nodes + 3 * (dag.S - 1) and bool((canon[:3 * dag.S].reshape(dag.S, 3) == np.arange(3)).all())
    # random accesses per node: insert = slot read + CAS (+ a 32-B compare read
    # on a hit), resolve = one slot read -> ~3 random 4..32-B touches per node
    res = {"workload": "dedup of %d node digests (C3 DAG + %d duplicated ref-index nodes)" % (n, 3 * (dag.S - 1)),
           "ms": ms, "mnodes_per_s": n / (ms * 1e-3) / 1e6, "unique": nu, "parity_ok": ok,
           "random_accesses_per_node": 3,
           "achieved_g_accesses_per_s": round(3 * n / (ms * 1e-3) / 1e9, 2)}
    for b in (d_idx, d_dig, d_canon, d_nu):
        b.free()
    return res


# --------------------------------------------------------------- C5: probe --
def bench_probe(args, dist, ctx):
    n_ins, n_probe = args.probe_keys, args.probes
    m = int(math.ceil(-1 * float(n_ins) * math.log(0.001) / math.pow(math.log(2), 2)))
    k = int(math.ceil(math.log(2) * float(m) / float(n_ins)))
    keys = ctx.alloc(32 * n_probe)
    # probes: [inserted keys x (n_probe/2n_ins)] ++ [fresh]; generated on device
    half = n_probe // 2
    lens = np.array([32 * n_ins, 32 * (n_probe - half)], dtype=np.uint64)
    offs = np.array([0, 32 * half], dtype=np.uint64)
    d_offs, d_lens = ctx.upload(offs), ctx.upload(lens)
    ctx.gen_fill(keys.ptr, d_offs.ptr, d_lens.ptr, 2, 0x5EED0005 + dist.rank, 32 * n_probe)
    ctx.sync()
    rep = half // n_ins
    for r in range(1, rep):
        capi._check(capi.lib().rf_memcpy_d2d(ctx.handle, keys.ptr + 32 * n_ins * r, keys.ptr, 32 * n_ins))
    b = capi.Bloom.new(ctx, m, k)
    ctx.timer_start()
    b.add_device(keys.ptr, n_ins, ctx.stream)
    add_ms = ctx.timer_stop()
    out = ctx.alloc(n_probe)

    def step():
        b.probe_device(keys.ptr, n_probe, out.ptr, ctx.stream)

    t = timed_steps(dist, ctx, step, args.probe_steps, 1)
    ctx.timer_start()
    step()
    dev_ms = ctx.timer_stop()
    hits = int(out.to_numpy().astype(np.int64).sum())
    fresh = n_probe - rep * n_ins
    fp = (hits - rep * n_ins) / max(fresh, 1)
    bpp = 32 + 8 * k + 1
    ach = n_probe * bpp / (dev_ms * 1e-3) / 1e9
    traffic, tsrc = pmc_traffic("k4_bloom_probe")
    # Words one launch fetches: a present key (or a false positive) all k; an
    # absent key stops at its first clear bit, so with a fraction f of the
    # filter's bits set it fetches sum_{j<k} f^j on average.
    f = float(np.bitwise_count(b.words()).sum()) / m
    absent = n_probe - hits
    reads = hits * k + absent * sum(f ** j for j in range(k))
    gread_s = reads / (dev_ms * 1e-3) / 1e9
    ceil = gather_ceiling(m // 8, n_probe // 4, k)
    # Repository.Collect over the same 1e9 keys as repository objects: probe +
    # ordered compaction of the dead ones (repository/file/repository.go:304-327)
    d_dead, d_cnt = ctx.alloc(8 * n_probe), ctx.alloc(64)
    b.collect_device(keys.ptr, None, n_probe, d_dead.ptr, d_cnt.ptr, ctx.stream)
    ctx.timer_start()
    b.collect_device(keys.ptr, None, n_probe, d_dead.ptr, d_cnt.ptr, ctx.stream)
    coll_ms = ctx.timer_stop()
    n_dead = int(d_cnt.to_numpy()[:8].view(np.uint64)[0])
    d_dead.free()
    d_cnt.free()
    assoc = bench_assoc(ctx, keys, n_ins, n_probe, hits)
    res = {"workload": "bloomlive probe: n=%d keys (m=%d bits, %.1f MiB, k=%d), %d probes (50%% present)"
                       % (n_ins, m, m / 8 / 2**20, k, n_probe),
           "gprobes_per_s": dist.sum(n_probe) * args.probe_steps / t / 1e9,
           "device_ms": dev_ms, "add_ms": add_ms, "false_positive_rate": fp,
           "assoc": assoc,
           "collect": {"objects": n_probe, "dead": n_dead, "dead_matches_probe": n_dead == n_probe - hits,
                       "ms": coll_ms, "g_objects_per_s": n_probe / (coll_ms * 1e-3) / 1e9,
                       "overhead_vs_probe": round(coll_ms / dev_ms, 3)},
           "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 4), "bytes_per_probe": bpp,
                        "traffic": traffic, "traffic_source": tsrc,
                        "note": "algorithmic bytes; each random 8-B word read moves a 64-B line, so the "
                                "real bound is the random-gather rate (roofline_gather)"},
           "roofline_gather": {"bound": "random 8-B gathers", "achieved": round(gread_s, 2),
                               "peak": round(ceil, 2) if ceil else None, "unit": "G words/s",
                               "frac": round(gread_s / ceil, 4) if ceil else None,
                               "words_per_probe": round(reads / n_probe, 3), "filter_fill": round(f, 4),
                               "peak_kind": "measured live: tools/micro.hip k_gather, k independent "
                                            "random 8-B reads per thread over a table of the filter's size"}}
    # bounded sample for the CPU leg (rank 0, N=1): the filter words and the
    # first 2e7 probe keys
    if dist.world == 1 and "cpu" not in args.skip:
        ns = min(n_probe, 20_000_000)
        res["_cpu"] = {"words": b.words(), "length": b.params()[2], "m": m, "k": k,
                       "keys": keys.to_numpy(count=32 * ns), "n": ns}
    for x in (keys, out, d_offs, d_lens):
        x.free()
    b.close()
    # gather-bound kernels beside the probe, against the same live ceiling
    if ceil:
        a = res.get("assoc")
        if a:
            a["roofline_gather"] = {"achieved": round(3 * n_probe / (a["get_ms"] * 1e-3) / 1e9, 2), "peak": round(ceil, 2),
                                    "unit": "G random accesses/s", "frac": round(3 * n_probe / (a["get_ms"] * 1e-3) / 1e9 / ceil, 3),
                                    "accesses_per_get": "3 (tag, 32-B key compare, 32-B value on a hit; absent keys "
                                                        "stop at an empty tag: 1-2)"}
    res["_gather_ceiling"] = ceil
    return res


def bench_assoc(ctx, keys, n_ins, n_probe, hits):
    """HBM assoc behind the probe (assoc.Assoc, assoc/assoc.go:26-38): the
    n_ins inserted cache keys Put with values, then a Get of all n_probe keys
    (the probe's positives resolve to values, the rest are NotExist)."""
    a = capi.Assoc(ctx, capacity=n_ins)
    vals = ctx.alloc(32 * n_ins)
    v_off, v_len = ctx.upload(np.array([0], np.uint64)), ctx.upload(np.array([32 * n_ins], np.uint64))
    ctx.gen_fill(vals.ptr, v_off.ptr, v_len.ptr, 1, 0x5EED0006, 32 * n_ins)
    st = ctx.alloc(4 * n_ins)
    ctx.sync()
    v_off.free()
    v_len.free()
    t0 = time.perf_counter()
    a.put_device(0, keys.ptr, vals.ptr, n_ins, st.ptr)
    put_s = time.perf_counter() - t0
    ok_put = not st.to_numpy(np.int32).any()
    d_v, d_f = ctx.alloc(32 * n_probe), ctx.alloc(n_probe)
    a.get_device(0, keys.ptr, n_probe, d_v.ptr, d_f.ptr)
    ctx.timer_start()
    a.get_device(0, keys.ptr, n_probe, d_v.ptr, d_f.ptr)
    get_ms = ctx.timer_stop()
    found = int(d_f.to_numpy().astype(np.int64).sum())
    occ, cap = a.stats()
    for b in (vals, st, d_v, d_f):
        b.free()
    # Eval.lookup for a batch of nodes (rf_assoc_lookup, host API): CacheKeys
    # [physical (absent), logical (an inserted key)] per node, precise read
    # repair writes the found value under the physical key
    n_nodes = min(2_000_000, n_ins)
    logical = keys.to_numpy(count=32 * n_nodes).reshape(n_nodes, 32)
    physical = np.random.default_rng(0x5EED0007).integers(0, 256, size=(n_nodes, 32), dtype=np.uint8)
    node_keys = np.stack([physical, logical], axis=1).reshape(-1)
    ptr = np.arange(0, 2 * n_nodes + 1, 2, dtype=np.uint64)
    t0 = time.perf_counter()
    which, _ = a.lookup(0, node_keys, ptr, repair=2)
    lk_s = time.perf_counter() - t0
    _, f2 = a.get(0, physical)  # repaired: the physical keys now resolve
    lookup = {"workload": "%d nodes x 2 cache keys (physical absent, logical present), precise read repair"
                          % n_nodes,
              "ms": lk_s * 1e3, "m_nodes_per_s": n_nodes / lk_s / 1e6,
              "hits_on_logical": int((which == 1).sum()), "repaired": int(f2.astype(np.int64).sum()),
              "note": "host API: keys H2D, one Get batch, first-hit select on the device, repair Put batch"}
    a.close()
    # bytes per Get: 32-B key read + a 4-B tag and a 32-B key compare (random)
    # + a 32-B value read (random, hits) + 33-B result write
    return {"workload": "Put %d keys (one batch), Get %d keys (%d present)" % (n_ins, n_probe, found),
            "put_ms": put_s * 1e3, "put_mkeys_per_s": n_ins / put_s / 1e6, "put_ok": ok_put,
            "get_ms": get_ms, "get_g_keys_per_s": n_probe / (get_ms * 1e-3) / 1e9,
            "found_exact": found == (n_probe // 2) // n_ins * n_ins,  # every Put key, no false positive
            "bloom_false_positives_resolved": hits - found,
            "table_slots": cap, "occupied": occ, "lookup": lookup}


def gather_ceiling(table_bytes, n_threads, reads):
    """Random 8-B gather rate (G words/s) of this GPU over a table of
    `table_bytes`, from the diagnostic kernel in tools/_micro.so (built by
    __graft_entry__.build()); None when that library is absent."""
    import ctypes
    so = os.path.join(ROOT, "tools", "_micro.so")
    if not os.path.exists(so):
        return None
    L = ctypes.CDLL(so)
    L.micro_gather.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
    L.micro_gather.restype = ctypes.c_float
    r = 10 if reads >= 10 else 6 if reads >= 6 else 2
    ms = L.micro_gather(int(table_bytes), int(n_threads), r, 1)
    return n_threads * r / (ms * 1e-3) / 1e9 if ms > 0 else None


# ----------------------------------------------------------- CPU baseline --
def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_probe_and_tables(probe, canon_n=2_000_000):
    """CPU legs of the probe / canonicalize / assoc rows: bloom Contains on the
    same filter (oracle/oracle.c, bloom.Test order; 1 thread = bloomlive's
    non-goroutine-safe Contains, and 16 threads), and Go-map-shaped dedup and
    lookups (a Python dict over 32-B keys: the flowMap / in-memory assoc)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import reflow_oracle as O
    L = O.lib()
    c = probe["_cpu"]
    words = np.ascontiguousarray(c["words"])
    keys = np.ascontiguousarray(c["keys"])
    out = np.zeros(c["n"], dtype=np.uint8)
    r = {}
    for th, n in ((1, min(c["n"], 2_000_000)), (16, c["n"])):
        t0 = time.perf_counter()
        L.orc_bloomlive_contains_batch(words.ctypes.data, int(c["length"]), int(c["m"]), int(c["k"]),
                                       keys.ctypes.data, n, out.ctypes.data, th)
        dt = time.perf_counter() - t0
        r["probe_%dt" % th] = {"value": n / dt / 1e9, "unit": "G probes/s", "cores": th, "kind": "port",
                               "sample": "%d probes of the configs[4] set against its filter" % n}
    ks = [keys[32 * i:32 * i + 32].tobytes() for i in range(canon_n)]
    t0 = time.perf_counter()
    first = {}
    for i, kk in enumerate(ks):
        first.setdefault(kk, i)
    dt = time.perf_counter() - t0
    r["canonicalize"] = {"value": canon_n / dt / 1e6, "unit": "M nodes/s", "cores": 1, "kind": "port",
                         "sample": "%d digests into a dict (flowMap.Put shape, flow.go:897-907)" % canon_n}
    t0 = time.perf_counter()
    hit = sum(1 for kk in ks if kk in first)
    dt = time.perf_counter() - t0
    r["assoc_get"] = {"value": canon_n / dt / 1e6, "unit": "M keys/s", "cores": 1, "kind": "port",
                      "sample": "%d dict lookups (test/testutil/assoc.go:49-56 shape)" % canon_n, "hits": hit}
    return r


def cpu_baseline(args, sha, dag):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ctypes

    import reflow_oracle as O  # the oracle: cpu_baseline leg only
    L = O.lib()
    threads = min(16, os.cpu_count() or 1)
    lens = sha["_lens"]
    # bounded sample of the same workload: files in generation order up to the
    # byte budget (the same skewed mix, big files included)
    budget = int(args.cpu_sample_gib * GiB)
    csum = np.cumsum(lens.astype(np.int64))
    n = int(np.searchsorted(csum, budget)) + 1
    n = min(n, len(lens))
    s_lens = lens[:n].copy()
    s_offs, total = arena_layout(s_lens, align=64)
    arena = np.zeros(total, dtype=np.uint8)
    L.orc_fill_batch(sha["_seed"], arena.ctypes.data, s_offs.ctypes.data, s_lens.ctypes.data, n, threads)
    out = np.zeros((n, 32), dtype=np.uint8)
    order = np.argsort(-s_lens.astype(np.int64), kind="stable").astype(np.uint64)  # LPT
    o_offs, o_lens = s_offs[order].copy(), s_lens[order].copy()
    t0 = time.perf_counter()
    L.orc_sha256_batch(arena.ctypes.data, o_offs.ctypes.data, o_lens.ctypes.data, n, out.ctypes.data,
                       threads)
    dt = time.perf_counter() - t0
    back = np.empty_like(out)
    back[order.astype(np.int64)] = out
    match = bool((back == sha["_digests"][:n]).all())
    res = {"value": float(s_lens.sum()) / dt / 1e9, "unit": "GB/s", "cores": threads, "kind": "port",
           "what": "SHA-256 of the C2 files (the headline metric's CPU leg)",
           "sample": "first %d files (%.2f GiB, largest %.2f GiB) of the same C2 set, oracle/oracle.c "
                     "scalar SHA-256, %d pthreads, largest-first" % (n, s_lens.sum() / GiB,
                                                                    s_lens.max() / GiB, threads),
           "seconds": dt, "gpu_digests_match": match, "cpu_model": cpu_model()}
    # The same sample through OpenSSL's SHA-256 (hashlib; SHA-NI where the CPU
    # has it -- what Go >= 1.21's crypto/sha256 uses), same threads, LPT order.
    import hashlib
    from concurrent.futures import ThreadPoolExecutor
    mv = memoryview(arena)

    def one(i):
        o, ln = int(s_offs[i]), int(s_lens[i])
        return hashlib.sha256(mv[o:o + ln]).digest()

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        dig = list(ex.map(one, order.astype(np.int64).tolist()))
    dt2 = time.perf_counter() - t0
    ok2 = all(d == sha["_digests"][int(i)].tobytes() for d, i in zip(dig, order.astype(np.int64)))
    res["openssl"] = {"value": float(s_lens.sum()) / dt2 / 1e9, "unit": "GB/s", "cores": threads,
                      "kind": "library", "sample": "same files, hashlib/OpenSSL SHA-256, %d threads" % threads,
                      "seconds": dt2, "gpu_digests_match": ok2,
                      "sha_ni": "sha_ni" in open("/proc/cpuinfo").read()}
    del mv, arena
    # configs[0] on the CPU port and OpenSSL (the reference's own CPU case)
    c1l = np.full(C1_N, C1_LEN, dtype=np.uint64)
    c1o, c1t = arena_layout(c1l, align=64)
    c1a = np.zeros(c1t, dtype=np.uint8)
    L.orc_fill_batch(C1_SEED, c1a.ctypes.data, c1o.ctypes.data, c1l.ctypes.data, C1_N, threads)
    c1out = np.zeros((C1_N, 32), dtype=np.uint8)
    t0 = time.perf_counter()
    L.orc_sha256_batch(c1a.ctypes.data, c1o.ctypes.data, c1l.ctypes.data, C1_N, c1out.ctypes.data, threads)
    c1_port = time.perf_counter() - t0
    c1mv = memoryview(c1a)
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda i: hashlib.sha256(c1mv[int(c1o[i]):int(c1o[i]) + C1_LEN]).digest(), range(C1_N)))
    c1_ssl = time.perf_counter() - t0
    res["c1"] = {"sample": "configs[0] in full: 4096 x 256 KiB", "port_ms": c1_port * 1e3,
                 "port_gbps": C1_N * C1_LEN / c1_port / 1e9, "openssl_ms": c1_ssl * 1e3,
                 "openssl_gbps": C1_N * C1_LEN / c1_ssl / 1e9, "cores": threads}
    del c1mv, c1a
    # C3 port: full recompute of a bounded sample DAG, 1 thread (Canonicalize is serial)
    if dag is not None:
        small = Dag1000(max(1, args.cpu_dag_samples), dag.P)
        a = small.arrays()
        order = np.zeros(small.n_jobs, dtype=np.uint64)
        # topological order = kinds in construction order (each kind only reads earlier ones)
        order[:] = np.arange(small.n_jobs, dtype=np.uint64)
        slots = np.zeros((small.n_slots, 32), dtype=np.uint8)
        slots[small.file_slots] = small.leaf_ids
        t0 = time.perf_counter()
        L.orc_graph_eval(small.n_jobs, order.ctypes.data, a["out_slot"].ctypes.data,
                         a["tmpl_off"].ctypes.data, a["tmpl_len"].ctypes.data, a["hole_ptr"].ctypes.data,
                         a["hole_pos"].ctypes.data, a["hole_slot"].ctypes.data, a["blob"].ctypes.data,
                         slots.ctypes.data)
        dt = time.perf_counter() - t0
        res["dag"] = {"value": small.n_nodes / dt / 1e6, "unit": "Mnodes/s (full recompute)", "cores": 1,
                      "kind": "port", "sample": "1000align DAG S=%d P=%d (%d nodes, %d jobs), "
                      "oracle/oracle.c orc_graph_eval" % (small.S, small.P, small.n_nodes, small.n_jobs),
                      "seconds": dt}
    _ = ctypes
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--sha-gib", type=float, default=64.0)
    ap.add_argument("--dag-samples", type=int, default=22075)  # ~10M nodes at P=32
    ap.add_argument("--dag-pairs", type=int, default=32)
    ap.add_argument("--dag-steps", type=int, default=20)
    ap.add_argument("--probe-keys", type=int, default=100_000_000)
    ap.add_argument("--probes", type=int, default=1_000_000_000)
    ap.add_argument("--probe-steps", type=int, default=3)
    ap.add_argument("--cpu-sample-gib", type=float, default=20.0)
    ap.add_argument("--cpu-dag-samples", type=int, default=200)
    ap.add_argument("--skip", default="", help="comma list of: c1,install,dag,probe,cpu")
    args = ap.parse_args()
    skip = set(filter(None, args.skip.split(",")))

    dist = Dist(args.gpus)
    device = dist.local
    share = os.environ.get("RF_BENCH_SHARE_GPU") == "1"
    if share:  # rehearsal of the N-rank path on a box with fewer GPUs (never the driver's run)
        device = dist.local % max(capi.device_count(), 1)
    ctx = capi.Context(device)
    comm, exchange = None, "none (1 rank)"
    if dist.world > 1:
        if share:
            exchange = "gloo host all-gather (RF_BENCH_SHARE_GPU: RCCL needs one GPU per rank)"
        else:
            uid = dist.bcast_bytes(capi.Comm.unique_id() if dist.rank == 0 else None)
            comm = capi.Comm(ctx, dist.world, dist.rank, uid)
            exchange = "RCCL all-gather over xGMI"

    sha = bench_sha(args, dist, ctx)
    c1 = None if "c1" in skip else bench_c1(args, dist, ctx)
    dag_res, dag = (None, None)
    if "dag" not in skip:
        dag_res, dag = bench_dag(args, dist, ctx, comm)
    probe = None if "probe" in skip else bench_probe(args, dist, ctx)
    cpu = None
    if dist.rank == 0 and dist.world == 1 and "cpu" not in skip:
        cpu = cpu_baseline(args, sha, dag)
        if probe is not None and "_cpu" in probe:
            cpu.update(cpu_probe_and_tables(probe))
    if probe is not None:
        probe.pop("_cpu", None)
        ceil = probe.pop("_gather_ceiling", None)
        cn = (dag_res or {}).get("canonicalize")
        if cn and ceil:
            cn["roofline_gather"] = {"achieved": cn["achieved_g_accesses_per_s"], "peak": round(ceil, 2),
                                     "unit": "G random accesses/s",
                                     "frac": round(cn["achieved_g_accesses_per_s"] / ceil, 3)}

    if dist.rank == 0:
        line = {
            "metric": "SHA-256 digest GB/s + incremental cache-key recompute Mnodes/s, 1/2/4/8 GPU",
            "value": round(sha["value"], 4), "unit": "GB/s", "n_gpus": dist.world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(sha["ms_per_step"], 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (splitmix64 content generated in HBM)",
            "config": {"workload": "configs[1]: 64 GiB FASTQ/BAM-like Fileset per GPU, %d files 4 KiB-2 GiB "
                                   "(98%% log-uniform 4 KiB-1 MiB, 2%% 64 MiB-2 GiB), SHA-256 of every file"
                                   % sha["files"],
                       "parallelism": "files sharded per GPU (independent); RCCL only for DAG root digests",
                       "exchange": exchange},
            "roofline": sha["roofline"],
            "cpu_baseline": cpu,
            "c1": c1,
            "incremental": dag_res,
            "probe": probe,
        }
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    ctx.close()


if __name__ == "__main__":
    main()
