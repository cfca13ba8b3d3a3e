#!/usr/bin/env python3
"""bench.py -- Reflow memoization hot path on MI355X (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W

Primary line (value): SHA-256 digest GB/s of configs[1], the 64 GiB
FASTQ/BAM-like skewed Fileset (4 KiB-2 GiB files), HBM-resident, per GPU.
A step = one rf_sha_plan_run over the whole set: every File ID, by the K1
planner's legs -- the longest chains on the host leg (SHA-NI threads fed by
chunked D2H; the reference's <=60-goroutine digest pool), the rest on the GPU
kernels (duo / octo / pair / lanes), split by a makespan model.  With N ranks
the global Fileset is N configs[1]-distributed sets (seeds 0x5EED0004+g),
sharded LPT by size over the ranks (weak scaling: 64 GiB per GPU; N = 8 is
configs[3]'s 512 GiB).

Secondary, in the same JSON line:
  "roofline"          the dominant GPU kernel of the hybrid run vs the
                      skew-aware floor; "roofline_gpu_only": k1_sha256_duo on
                      the GPU-only plan (one run); "host_leg": the SHA-NI leg
  "c1"                configs[0] (the reference's CPU case) on the GPU
  "incremental"       configs[2]: 10M-node 1000align DAG, 1% of leaf File
                      IDs changed per step (K3 frontier + K2), dirty blocks
  "probe"             configs[4]: 1e9 probes against the 1e8-key filter
                      (171 MiB, MALL-resident) and a 1.2e9-key one (2 GiB)
  "cpu_baseline"      host-core legs on the GPU box (rank 0, N = 1)
A --budget-s guard skips optional sections (recorded as skipped) so the run
ends in time even on a slow box; the JSON line is printed last.
"""
import argparse
import hashlib
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from reflow_amd import capi  # noqa: E402
from reflow_amd.workloads import Dag1000, GiB, PartitionedDag1000, arena_layout, c2_sizes  # noqa: E402

# ---- hardware constants (MI355X_MICROARCH.md) ------------------------------
CLOCK_HZ = 2.4e9
N_CU = 256
VALU_LANE_OPS = N_CU * 4 * 32 * CLOCK_HZ      # int32 VALU lane-ops/s (= FP32 FMA rate)
SHA_OPS_PER_BLOCK = 1464                        # canonical ops per 64-B block
SHA_VALU_PEAK_GBS = VALU_LANE_OPS / SHA_OPS_PER_BLOCK * 64 / 1e9
# A message's blocks are a serial chain (Merkle-Damgard).  One round's critical
# path is 3 dependent VALU ops (rotate -> xor3 -> add3 into e/a); the
# dependent-issue latency of one wave is 4 cycles (MI355X_MICROARCH.md,
# "Dependent-chain latency"; tools/micro.py lat: 4-5).  So no GPU
# implementation can finish a message of B blocks in less than B*64*3*4 cycles.
CHAIN_CYCLES_PER_BLOCK = 64 * 3 * 4
# The same chain at the wave64 ISSUE floor (reported beside frac, never as
# peak): a wave64 VALU instruction occupies its 16-lane SIMD for 4 cycles, so
# one wave cannot issue faster than one per 4 cycles, dependent or not
# (measured 4.5-5.5, profiles/r01/valu_issue_cost.log); k1_sha256_duo's
# two-lane lagged round is 8 instructions.
DUO_INSTR_PER_ROUND = 8
ISSUE_CYCLES_PER_INSTR = 4
# k2_level_pl's two-lane round (lag_chain.h RF_L2_STEP): 9 instructions
K2_INSTR_PER_ROUND = 9
HBM_PEAK_GBS = 8000.0
T_START = time.perf_counter()


def log(*a):
    print("[bench %6.1fs]" % (time.perf_counter() - T_START), *a, file=sys.stderr, flush=True)


class Budget:
    """Skips optional sections whose estimated cost would overrun --budget-s
    (the driver kills a bench at its own limit, and a killed run prints
    nothing)."""

    def __init__(self, seconds):
        self.seconds = seconds
        self.skipped = []
        self.dist = None  # set once the ranks are up: every rank then takes the same decision

    def allow(self, name, est_s, everyone=False):
        """everyone: every rank calls this and must take the same decision
        (the section holds collectives): the least time left on any rank."""
        left = self.seconds - (time.perf_counter() - T_START)
        if everyone and self.dist is not None and self.dist.world > 1:
            left = -self.dist.max(-left)
        if est_s > left:
            self.skipped.append({"section": name, "estimate_s": est_s, "left_s": round(left, 1)})
            log("SKIP %s: estimated %.0f s, %.0f s left in the budget" % (name, est_s, left))
            return False
        return True


PMC_ROUND = "pmc_r06"  # traffic is read only from this round's pass over the current library (profiles/pmc_r06)


def k2_traffic(graph):
    """HBM traffic of a DAG step from this round's committed rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes (tools/pmc_round6.sh -> tools/pmc_dag.py
    on the same graph and change set; profiles/pmc_r06/k2_traffic_*.json),
    beside the step's algorithmic bytes; None if absent."""
    path = os.path.join(ROOT, "profiles", PMC_ROUND, "k2_traffic_%s.json" % graph)
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    return {"traffic_bytes_per_step": round(d["traffic_bytes_per_step"]),
            "algorithmic_bytes_per_step": d["algorithmic_bytes_per_step"],
            "traffic_over_algorithmic": d["traffic_over_algorithmic"],
            "traffic_bytes_per_dirty_block": d["traffic_bytes_per_dirty_block"],
            "source": os.path.relpath(path, ROOT) + " (separate FETCH_SIZE and WRITE_SIZE passes, raw KiB x 1024)"}


def pmc_traffic(kernel, workload, algo_bytes=None):
    """HBM bytes per launch of `kernel` from this round's committed rocprofv3
    --pmc FETCH_SIZE/WRITE_SIZE pass (profiles/<PMC_ROUND>/pmc_traffic.json,
    tools/pmc_summary.py, corrected as MI355X_MICROARCH.md prescribes) --
    only when that pass ran this same workload (its "workload" key); None
    otherwise (never an earlier round's file: the library changes between
    rounds).  A kernel launched more than once there (the hybrid step's duo
    launch on three files, the GPU-only run's on 35) is matched to this
    launch by its algorithmic bytes: the launch whose traffic is nearest in
    ratio.  PMC counters cannot be read inside this process."""
    for path in [os.path.join(ROOT, "profiles", PMC_ROUND, "pmc_traffic.json")]:
        if not os.path.exists(path):
            continue
        d = json.load(open(path))
        if d.get("workload") != workload:
            continue
        v = d.get("rf::" + kernel)
        if v:
            launches = v.get("launch_traffic_bytes") or []
            if algo_bytes and launches:
                t = min(launches, key=lambda x: abs(np.log(max(x, 1.0) / algo_bytes)))
                return t, os.path.relpath(path, ROOT)
            return v.get("traffic_bytes_largest_launch", v["traffic_bytes_per_launch"]), os.path.relpath(path, ROOT)
    return None, None


class Dist:
    def __init__(self, n_gpus):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # (gloo's "[Gloo] Rank r is connected ..." goes to stderr: main()
            # points the C-level stdout there for the whole run)
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            dist.barrier()
            self.dist = dist
        if n_gpus != self.world and self.world > 1:
            log("warning: --gpus %d but WORLD_SIZE %d" % (n_gpus, self.world))

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def _reduce(self, x, op):
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x):
        return x if self.world == 1 else self._reduce(x, self.dist.ReduceOp.MAX)

    def sum(self, x):
        return x if self.world == 1 else self._reduce(x, self.dist.ReduceOp.SUM)

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
    for _ in range(steps):
        fn()
    ctx.sync()
    dist.barrier()
    t1 = time.perf_counter()
    return dist.max(t1 - t0)


# ---------------------------------------------------------------- C2: SHA --
def shard_lpt(sizes, world):
    """LPT by size: files largest first, each to the least-loaded rank.
    Returns the owner rank of every file."""
    order = np.argsort(-sizes.astype(np.int64), kind="stable")
    load = np.zeros(world, dtype=np.float64)
    owner = np.zeros(len(sizes), dtype=np.int64)
    for i in order:
        r = int(np.argmin(load))
        owner[i] = r
        load[r] += float(sizes[i])
    return owner


def rank_sizes(args, dist):
    """This rank's files.  N = 1: configs[1] itself.  N > 1: the global Fileset
    of N configs[1]-distributed sets (seeds 0x5EED0004 + g), LPT-sharded."""
    total = int(args.sha_gib * GiB)
    if dist.world == 1:
        return c2_sizes(total_bytes=total, seed=0x5EED0002), 0x5EED0002, None
    sets = [c2_sizes(total_bytes=total, seed=0x5EED0004 + g) for g in range(dist.world)]
    allsz = np.concatenate(sets)
    owner = shard_lpt(allsz, dist.world)
    mine = allsz[owner == dist.rank]
    glob_info = {"files": int(len(allsz)), "bytes": int(allsz.sum()),
                 "rank_bytes_max_over_min": float(np.bincount(owner, weights=allsz.astype(np.float64)).max()
                                                  / max(np.bincount(owner, weights=allsz.astype(np.float64)).min(), 1))}
    return mine, 0x5EED0004 + 0x100 * dist.rank, glob_info


def latency_roofline(crit_blocks, ms):
    """The incremental DAG step's latency roofline: its critical path is the
    longest chain of dependent compressions the change set starts
    (workloads critical_path: blocks, constant leading blocks excluded), and
    no implementation hashes a chain faster than 64 rounds x 3 dependent VALU
    x 4 cycles a block (the K1 skew-aware floor); the issue floor is the same
    chain at k2_level_pl's 9-instruction two-lane round."""
    t_chain = crit_blocks * CHAIN_CYCLES_PER_BLOCK / CLOCK_HZ
    t_issue = crit_blocks * 64 * K2_INSTR_PER_ROUND * ISSUE_CYCLES_PER_INSTR / CLOCK_HZ
    return {"bound": "critical path (latency)", "critical_path_blocks": int(crit_blocks),
            "chain_floor_us": round(t_chain * 1e6, 2), "issue_floor_us": round(t_issue * 1e6, 2),
            "achieved_us": round(ms * 1e3, 2), "frac": round(t_chain / (ms * 1e-3), 4),
            "frac_of_issue_floor": round(t_issue / (ms * 1e-3), 4),
            "peak_kind": "critical-path floor: the longest dependent-compression chain of the step x 64 rounds "
                         "x 3 dependent VALU x 4 cycles @2.4GHz (frac = floor / step time); issue floor: the same "
                         "chain x 9 instructions a round (two-lane chain) x 4 cycles"}


def kernel_roofline(name, lens, ids, ms):
    """achieved = the kernel's file bytes / its HIP-event time; peak = the
    skew-aware floor of its message set (the longest chain's critical path,
    or the chip's VALU throughput)."""
    nblk = (lens.astype(np.int64) + 9 + 63) // 64
    b = float(lens[ids].sum())
    t_chain = float(nblk[ids].max()) * CHAIN_CYCLES_PER_BLOCK / CLOCK_HZ
    t_valu = float(nblk[ids].sum()) * SHA_OPS_PER_BLOCK / VALU_LANE_OPS
    t_floor = max(t_chain, t_valu)
    ach = b / (ms * 1e-3) / 1e9
    peak = b / t_floor / 1e9
    extra = {}
    if name == "k1_sha256_duo":  # the chain at the measured single-wave issue rate (not the peak)
        t_issue = float(nblk[ids].max()) * 64 * DUO_INSTR_PER_ROUND * ISSUE_CYCLES_PER_INSTR / CLOCK_HZ
        extra = {"issue_floor_s": round(t_issue, 4), "frac_of_issue_floor": round(t_issue / (ms * 1e-3), 4),
                 "us_per_chain_block": round(ms * 1e3 / float(nblk[ids].max()), 4),
                 "issue_floor_kind": "longest message's blocks x 64 rounds x 8 instructions (the duo round) "
                                     "x 4 cycles (a wave64 VALU op occupies a 16-lane SIMD 4 cycles) @2.4GHz"}
    return {"bound": "valu", "kernel": name, "achieved": round(ach, 3), "peak": round(peak, 3), "unit": "GB/s",
            "frac": round(ach / peak, 4), **extra,
            "peak_kind": "skew-aware floor: max(longest message's blocks x 64 rounds x 3 dependent VALU x 4 cyc "
                         "@2.4GHz, sum blocks x 1464 ops / INT32 VALU peak)",
            "floor_s": round(t_floor, 4), "chain_floor_s": round(t_chain, 4),
            "frac_of_valu_peak": round(ach / SHA_VALU_PEAK_GBS, 6), "launch_ms": round(ms, 3),
            "bytes_per_launch": b, "messages": int(len(ids)), "critical_chain_blocks": int(nblk[ids].max())}


def bench_sha(args, dist, ctx, budget):
    lens, seed, glob_info = rank_sizes(args, dist)
    offs, arena_bytes = arena_layout(lens)
    arena = ctx.alloc(arena_bytes)
    d_offs, d_lens = ctx.upload(offs), ctx.upload(lens)
    out = ctx.alloc(32 * len(lens))
    ctx.gen_fill(arena.ptr, d_offs.ptr, d_lens.ptr, len(lens), seed, arena_bytes)
    ctx.sync()
    # The all-host plan (every file on the SHA-NI leg, fed from HBM): measured
    # beside the hybrid, and the run that calibrates the planner's host-leg
    # feed rate (rf_host_link) before the hybrid plan is made
    all_host = None
    link0 = ctx.host_link()
    if ctx.host_info()[0] and "allhost" not in args.skip:
        pa = ctx.sha_plan(offs, lens, capi.RF_SHA_ALL_HOST)
        runs = []
        for _ in range(3):  # the first one warms the pool and pins the staging
            t0 = time.perf_counter()
            pa.run(arena.ptr, out.ptr)
            sa = pa.stats()
            runs.append(((time.perf_counter() - t0) * 1e3, sa.last_ms_host))
        ms_a = float(np.mean([r[0] for r in runs[1:]]))
        all_host = {"gbps": round(float(lens.sum()) / (ms_a * 1e-3) / 1e9, 3), "ms": round(ms_a, 2),
                    "host_leg_ms": [round(r[1], 2) for r in runs[1:]], "threads": int(sa.host_threads),
                    "what": "RF_SHA_ALL_HOST: every file on the host leg (SHA-NI threads fed D2H from HBM), "
                            "mean of 2 runs after one warm-up"}
        pa.close()
    link1 = ctx.host_link()
    plan = ctx.sha_plan(offs, lens, 0)
    st = plan.stats()
    log("C2: planner's host feed %.1f GB/s (%s; before: %.1f GB/s %s)"
        % (link1[0] / 1e9, "measured" if link1[1] else "assumed", link0[0] / 1e9, "measured" if link0[1] else "assumed"))
    log("C2: %d files, %.1f GiB, largest %.2f GiB: %d on the host leg (%.1f GiB, %d threads), %d duo, %d lane"
        % (len(lens), lens.sum() / GiB, lens.max() / GiB, st.n_host, st.host_bytes / GiB, st.host_threads,
           st.n_solo, len(lens) - st.n_host - st.n_solo))
    rec = {"solo": [], "lanes": [], "host": [], "total": []}

    def step():
        plan.run(arena.ptr, out.ptr)
        s = plan.stats()  # synchronises: per-leg times of this run
        rec["solo"].append(s.last_ms_solo)
        rec["lanes"].append(s.last_ms_lanes)
        rec["host"].append(s.last_ms_host)
        rec["total"].append(s.last_ms_total)

    t = timed_steps(dist, ctx, step, args.steps, args.warmup)
    for k in rec:
        rec[k] = rec[k][args.warmup:]
    log("  hybrid: %.1f ms/step (host leg %.1f ms, duo %.1f ms, lanes %.1f ms)"
        % (t / args.steps * 1e3, np.mean(rec["host"]), np.mean(rec["solo"]), np.mean(rec["lanes"])))
    bytes_all = dist.sum(float(lens.sum())) * args.steps
    nblk = (lens.astype(np.int64) + 9 + 63) // 64
    order = np.argsort(-nblk, kind="stable")
    h, k = int(st.n_host), int(st.n_solo)
    host_ids, solo_ids, lane_ids = order[:h], order[h:h + k], order[h + k:]
    legs = []
    if k:
        legs.append(("k1_sha256_duo", solo_ids, float(np.mean(rec["solo"]))))
    if len(lane_ids):
        n_simd = 4 * N_CU
        lk = "k1_sha256_octo" if len(lane_ids) <= 4 * n_simd else "k1_sha256_pair" if len(lane_ids) <= 16 * n_simd \
            else "k1_sha256_lanes"
        legs.append((lk, lane_ids, float(np.mean(rec["lanes"]))))
    gpu_roofs = [kernel_roofline(name, lens, ids, ms) for name, ids, ms in legs]
    for r, (name, ids, ms) in zip(gpu_roofs, legs):
        r["traffic"] = None
        r["traffic_note"] = ("not measured in the hybrid step: device-wide FETCH/WRITE counters there also see the "
                             "host leg's D2H stream; the GPU-only pass (roofline_gpu_only) measures the duo alone")
    workload = ("configs[1]: %.1f GiB Fileset per GPU, %d files 4 KiB-2 GiB (98%% log-uniform 4 KiB-1 MiB, "
                "2%% 64 MiB-2 GiB), SHA-256 of every file" % (lens.sum() / GiB, len(lens)))
    hb = float(lens[host_ids].sum()) if h else 0.0
    host_ms = float(np.mean(rec["host"])) if h else 0.0
    thr, core_rate, sha_ext = ctx.host_info()
    ways, thread_rate = ctx.host_rate()
    host_leg = None
    step_ms = t / args.steps * 1e3
    if h:
        per_thread = hb / (host_ms * 1e-3) / st.host_threads / 1e9
        host_leg = {"threads": int(st.host_threads), "files": h, "bytes": hb, "ms": round(host_ms, 2),
                    "gbps": round(hb / (host_ms * 1e-3) / 1e9, 3), "per_thread_gbps": round(per_thread, 3),
                    "core_sha_ni_gbps": round(core_rate / 1e9, 3),
                    "thread_rate_gbps": round(thread_rate / 1e9, 3), "chains_per_thread": ways,
                    "frac_of_core_rate": round(per_thread / (core_rate / 1e9), 3) if core_rate else None,
                    "largest_file_gib": round(float(lens[host_ids].max()) / GiB, 3),
                    "feed": "D2H in 8 MiB chunks per thread, double-buffered (PCIe), from the HBM-resident set",
                    "why": "one file is one serial chain: a SHA-NI core runs it ~40x faster than a GPU wave"}
    # the step's roofline is the leg that sets it: on configs[1] the host leg
    # (the chain-bound largest files on SHA-NI threads), priced against its
    # own peak -- threads x one thread's measured rate at the configured
    # chain interleave on this box; the GPU kernels' rooflines sit beside it
    gpu_b = float(lens[np.concatenate([solo_ids, lane_ids])].sum()) if len(lane_ids) + k else 0.0
    # the planner balances the legs' times (the duo leg ends within ~2 % of
    # the host leg), so "dominant" is by bytes: the host leg's 98 %
    if h and thread_rate and hb >= gpu_b:
        ach = hb / (host_ms * 1e-3) / 1e9
        peak = st.host_threads * thread_rate / 1e9
        roof = {"bound": "host SHA-NI issue", "leg": "host_leg", "achieved": round(ach, 3), "peak": round(peak, 3),
                "unit": "GB/s", "frac": round(ach / peak, 4), "traffic": None,
                "traffic_note": "a CPU leg: its input is the files' bytes streamed D2H once (PCIe), no HBM "
                                "re-reads to count; device PMC counters do not describe it",
                "peak_kind": "host-leg threads x one thread's measured SHA-NI rate with %d interleaved chains "
                             "(rf_host_rate, this box)" % ways,
                "leg_ms": round(host_ms, 2), "step_ms": round(step_ms, 2), "bytes": hb,
                "bytes_frac": round(hb / max(hb + gpu_b, 1.0), 4), "threads": int(st.host_threads),
                "gpu_legs_ms": {name: round(ms, 2) for name, _, ms in legs}}
    else:
        dom = max(zip(gpu_roofs, legs), key=lambda x: x[1][2])[0] if legs else None
        roof = dom
    gpu_bytes = gpu_b
    composition = {"host_leg_bytes": hb, "gpu_bytes": gpu_bytes,
                   "host_leg_bytes_frac": round(hb / max(hb + gpu_bytes, 1.0), 4),
                   "gpu_legs_gbps": round(gpu_bytes / (max([ms for _, _, ms in legs] or [1e-9]) * 1e-3) / 1e9, 3)
                   if legs else None,
                   "note": "value is the whole hybrid step (CPU SHA-NI host leg + GPU kernels, split by the K1 "
                           "planner's makespan model); the GPU-only rate of the same set is gpu_only.gbps"}
    rank_gbps = float(lens.sum()) / (step_ms * 1e-3) / 1e9
    if all_host:
        all_host["hybrid_minus_all_host_gbps"] = round(rank_gbps - all_host["gbps"], 3)
        all_host["hybrid_ge_all_host"] = bool(rank_gbps >= all_host["gbps"])
        all_host["planner_feed_gbps"] = round(link1[0] / 1e9, 3)
        all_host["planner_feed_measured"] = bool(link1[1])
        all_host["planner_picked_all_host"] = bool(h == len(lens))
        log("  all-host: %.1f ms (%.2f GB/s); hybrid %.1f ms (%.2f GB/s): the GPU legs add %+.2f GB/s"
            % (all_host["ms"], all_host["gbps"], step_ms, rank_gbps, rank_gbps - all_host["gbps"]))
    res = dict(value=bytes_all / t / 1e9, ms_per_step=step_ms, roofline=roof, roofline_gpu_legs=gpu_roofs,
               host_leg=host_leg, composition=composition, all_host=all_host,
               files=int(len(lens)), bytes_per_gpu=int(lens.sum()), workload=workload, glob=glob_info,
               split={"host": h, "duo": k, "lanes": int(len(lane_ids))},
               step_ms={kk: round(float(np.mean(v)), 3) for kk, v in rec.items()})
    # GPU-only plan (no host leg), one run: the duo chain's roofline on the
    # same set (the chain-bound floor the host leg exists for)
    if args.gpu_only_run and budget.allow("gpu_only_duo", 45):
        p2 = ctx.sha_plan(offs, lens, capi.RF_SHA_NO_HOST)
        out2 = ctx.alloc(32 * len(lens))
        t0 = time.perf_counter()
        p2.run(arena.ptr, out2.ptr)
        s2 = p2.stats()
        wall = time.perf_counter() - t0
        o2 = np.argsort(-nblk, kind="stable")
        duo_ids = o2[:int(s2.n_solo)]
        r2 = kernel_roofline("k1_sha256_duo", lens, duo_ids, s2.last_ms_solo) if s2.n_solo else None
        if r2:
            tr2, ts2 = pmc_traffic("k1_sha256_duo", workload, r2["bytes_per_launch"])
            r2["traffic"], r2["traffic_source"] = tr2, ts2 or ("no %s PMC pass of this workload on the current "
                                                               "library (profiles/%s/pmc_traffic.json)" % (PMC_ROUND, PMC_ROUND))
        same = bool((out2.to_numpy() == out.to_numpy()).all())
        res["roofline_gpu_only"] = r2
        res["gpu_only"] = {"gbps": float(lens.sum()) / wall / 1e9, "ms": wall * 1e3, "duo_files": int(s2.n_solo),
                           "digests_equal_hybrid": same}
        log("  GPU-only plan: %.1f s (duo %.1f s), digests equal: %s" % (wall, s2.last_ms_solo / 1e3, same))
        p2.close()
        out2.free()
    res["_digests"] = out.to_numpy().reshape(-1, 32)
    res["_lens"], res["_seed"], res["_arena"], res["_offs"] = lens, seed, arena, offs
    plan.close()
    for b in (d_offs, d_lens, out):
        b.free()
    return res


# -------------------------------------------------- C1: reference config --
C1_N, C1_LEN, C1_SEED = 4096, 262144, 0x5EED0001


def c1_path(i):
    return ("d%02d/f%04d.fq.gz" % (i // 64, i)).encode()


def bench_c1(args, dist, ctx, budget):
    """configs[0], the reference's own CPU-runnable case, on the GPU: File IDs
    of 1 GiB = 4096 x 256 KiB files (HBM-resident, GPU kernels: octo chains),
    the Fileset digest of the 4096-entry map (executor.go:205-233: one 3137-
    block material, IDs placed from HBM; the planner gives the one long chain
    to the host leg), and CacheKeys of a ~10k-node 1000align DAG (K2 full
    recompute).  Checked against tests/golden/c1_fileset.json."""
    lens = np.full(C1_N, C1_LEN, dtype=np.uint64)
    offs, arena_bytes = arena_layout(lens)
    arena = ctx.alloc(arena_bytes)
    d_offs, d_lens = ctx.upload(offs), ctx.upload(lens)
    out = ctx.alloc(32 * C1_N)
    ctx.gen_fill(arena.ptr, d_offs.ptr, d_lens.ptr, C1_N, C1_SEED, arena_bytes)
    ctx.sync()
    plan = ctx.sha_plan(offs, lens, 0)
    st = plan.stats()
    plan.run(arena.ptr, out.ptr)
    ctx.sync()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        plan.run(arena.ptr, out.ptr)
    ctx.sync()
    ids_ms = (time.perf_counter() - t0) / reps * 1e3
    fp = ctx.fileset_paths([[[c1_path(i) for i in range(C1_N)]]])
    fp.digest_device(out.ptr)
    t0 = time.perf_counter()
    for _ in range(reps):
        fsd = fp.digest_device(out.ptr)[0]
    fs_ms = (time.perf_counter() - t0) / reps * 1e3
    ids = out.to_numpy().reshape(-1, 32)
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "c1_fileset.json")))
    ok = ("sha256:" + fsd.hex() == want["fileset_digest"] and
          hashlib.sha256(ids.tobytes()).hexdigest() == want["ids_sha256"])
    inst = None
    if "install" not in args.skip and dist.rank == 0 and budget.allow("c1_install", 20):
        inst = bench_c1_install(ctx, arena, offs, fsd, cpu_leg=dist.world == 1 and "cpu" not in args.skip)
    plan.close()
    for b in (arena, d_offs, d_lens, out):
        b.free()
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
            "file_ids_split": {"host": int(st.n_host), "duo": int(st.n_solo),
                               "lanes": int(C1_N - st.n_host - st.n_solo)},
            "fileset_digest_ms": fs_ms,
            "fixture_match": ok, "dag_nodes": small.n_nodes, "dag_full_recompute_ms": dag_ms,
            "total_ms": ids_ms + fs_ms + dag_ms, "install": inst}


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
        if cpu_leg:  # the same install on the host: read + OpenSSL SHA-256 on native threads
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import ctypes
            import reflow_oracle as O  # (oracle/baseline_openssl.c: the cpu_baseline leg only)
            paths = [os.path.join(root, c1_path(i).decode()).encode() for i in range(C1_N)]
            arr = (ctypes.c_char_p * C1_N)(*paths)
            threads = ctx.host_info()[0] or 1
            got = np.zeros((C1_N, 32), dtype=np.uint8)
            best = None
            for _ in range(3):  # (best of 3, page cache warm)
                t0 = time.perf_counter()
                rc = O.lib().orc_openssl_sha256_files(ctypes.cast(arr, ctypes.c_void_p), C1_N, got.ctypes.data,
                                                     threads)
                dt = (time.perf_counter() - t0) * 1e3
                best = dt if best is None else min(best, dt)
            ok = rc == 0 and [got[i].tobytes() for i in range(C1_N)] == [e[1] for e in ents]
            res["cpu_openssl"] = {"ms": best, "gbps": C1_N * C1_LEN / (best * 1e-3) / 1e9, "cores": threads,
                                  "ids_match": ok,
                                  "what": "each file read (1 MiB pieces) and hashed with OpenSSL on %d native "
                                          "threads, one queue (oracle/baseline_openssl.c; best of 3)" % threads}
    finally:
        shutil.rmtree(root, ignore_errors=True)
    return res


# ---------------------------------------------------------- lowering leg --
def _lower_run(args, dup):
    import subprocess
    exe = os.path.join(ROOT, "tools", "lower_bench")
    t0 = time.perf_counter()
    cmd = [exe, str(args.dag_samples), str(args.dag_pairs)] + (["dup"] if dup else [])
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    except subprocess.TimeoutExpired:
        return {"error": "timed out after 300 s"}
    wall = time.perf_counter() - t0
    if r.returncode != 0 or not r.stdout.strip():
        return {"error": "rc %d: %s" % (r.returncode, (r.stderr or "")[-300:])}
    res = json.loads(r.stdout.strip().splitlines()[-1])
    res["wall_s"] = round(wall, 2)
    # RF_LOWER_TIMING=1: the lowering's phases (reflow_host.cpp PhaseClock)
    phases = [ln[1:].replace("] ", ": ", 1).rsplit(" ", 2) for ln in (r.stderr or "").splitlines()
              if ln.startswith("[lower] ") or ln.startswith("[load] ")]
    if phases:
        res["phases_s"] = {}
        for ph in phases:  # (a phase seen again -- the second load of a collapse -- gets its ordinal)
            if len(ph) == 3:
                k, n = ph[0], 2
                while k in res["phases_s"]:
                    k, n = "%s (%d)" % (ph[0], n), n + 1
                res["phases_s"][k] = float(ph[1])
        log("lowering phases: " + ", ".join("%s %.2f" % kv for kv in res["phases_s"].items()))
    log("lowering%s: %d nodes: build %.1f s, canonicalize %.1f s (%d collapsed), lower %.1f s, load %.1f s, "
        "incremental %.1f ms" % (" (per-sample reference chains)" if dup else "", res["nodes"], res["build_s"],
                                 res["canonicalize_s"], res.get("collapsed", 0), res["lower_s"], res["load_s"],
                                 res["incremental_s"] * 1e3))
    return res


def bench_lowering(args):
    """The per-Eval host cost a Go shim pays before the device sees a job:
    tools/lower_bench (the product's C++ host mirror, include/reflow_host.hpp)
    builds a configs[2]-sized 1000align Flow graph, Canonicalizes it, lowers
    it to rf_graph jobs, loads it, and takes one 1%-of-files incremental step
    (checked against a full recompute).  Run twice: the shared reference
    chain (nothing collapses), and every sample with its own copy of it
    ("collapsed_graph": Canonicalize collapses the copies and hands over its
    Eval with their jobs dropped -- its root must equal the first run's)."""
    if not os.path.exists(os.path.join(ROOT, "tools", "lower_bench")):
        return {"skipped": "tools/lower_bench not built"}
    res = _lower_run(args, False)
    if "error" in res:
        return res
    res["what"] = ("tools/lower_bench: reflow::Canonicalize + Eval lowering (reflow_host.cpp) of a 1000align "
                   "Flow graph of the configs[2] shape; load = blob + rf_graph_load + full recompute")
    dup = _lower_run(args, True)
    if "error" not in dup:
        dup["root_equals_shared_chain"] = dup.get("root") == res.get("root")
        res["collapsed"] = dup.get("collapsed", 0)
        res["collapsed_canonicalize_s"] = dup.get("canonicalize_s")
        res["collapsed_incremental_equals_full"] = dup.get("incremental_equals_full")
    res["collapsed_graph"] = dup
    return res


# ------------------------------------------------------- C3: incremental --
def bench_dag(args, dist, ctx, budget):
    """configs[2] (N = 1): one 10M-node 1000align DAG, 1% of leaf File IDs
    toggled per step (K3 frontier + K2 levels), plus Canonicalize's flowMap
    over its node digests and the CPU legs' inputs."""
    t0 = time.perf_counter()
    S = args.dag_samples
    dag = Dag1000(S, args.dag_pairs)
    a = dag.arrays()
    t_build = time.perf_counter() - t0
    g = capi.Graph.from_arrays(ctx, a)
    g.set_slots(dag.file_slots, dag.leaf_ids)
    t_load = time.perf_counter() - t0 - t_build
    log("C3: %d nodes, %d jobs built in %.1f s, loaded in %.1f s" % (dag.n_nodes, len(a["out_slot"]), t_build, t_load))
    g.recompute(True)  # first call also captures the hipGraph (host work): untimed
    ctx.timer_start()
    g.recompute(True)
    full_ms = ctx.timer_stop()
    every = np.arange(a["n_slots"], dtype=np.uint32)
    snap_full = g.get_slots(every)  # the full recompute's table (the original File IDs)
    slots, old, new = dag.change_set(0.01)
    d_slots = ctx.upload(slots)
    d_old, d_new = ctx.upload(old), ctx.upload(new)
    # one counted step to learn the dirty-set size
    g.set_slots(slots, new)
    n_dirty_jobs = g.recompute(False)
    g.set_slots(slots, old)
    g.recompute(False)
    pairs = np.unique(slots // 2)
    n_dirty_nodes = n_dirty_jobs - len(pairs)  # minus the pE1 physical keys
    state = {"v": 0}

    def step():
        ver = d_new if state["v"] == 0 else d_old
        state["v"] ^= 1
        g.set_slots_device(d_slots.ptr, ver.ptr, len(slots), ctx.stream)
        g.recompute_async(False, ctx.stream)

    steps = args.dag_steps
    t = timed_steps(dist, ctx, step, steps, 2)
    ctx.timer_start()
    for _ in range(steps):
        step()
    dev_ms = ctx.timer_stop() / steps
    # parity snapshots after the timed steps (untimed): the table one more
    # incremental step leaves with the changed IDs (checked against the
    # oracle in the cpu leg), and the table after stepping back, which must
    # equal the full recompute's slot for slot
    if state["v"] == 1:
        step()
    step()
    ctx.sync()
    snap_new = g.get_slots(every)
    step()
    ctx.sync()
    back_equal_full = bool((g.get_slots(every) == snap_full).all())
    res = {"workload": "configs[2]: 1000align DAG S=%d P=%d, 1%% leaf File IDs toggled per step" % (S, args.dag_pairs),
           "nodes": dag.n_nodes, "jobs": len(a["out_slot"]),
           "dirty_nodes_per_step": int(n_dirty_nodes), "dirty_jobs_per_step": int(n_dirty_jobs),
           "ms_per_step": t / steps * 1e3, "device_ms_per_step": dev_ms,
           "mnodes_per_s": n_dirty_nodes * steps / t / 1e6,
           "effective_mnodes_per_s": dag.n_nodes * steps / t / 1e6,
           "full_recompute_ms": full_ms,
           "full_recompute_mnodes_per_s": dag.n_nodes / (full_ms * 1e-3) / 1e6,
           "levels": g.stats().n_levels, "build_s": round(t_build, 2), "load_s": round(t_load, 2),
           "incremental_equals_full": back_equal_full,
           # filled in by the cpu leg's oracle checks (null if it did not run)
           "digests_equal_oracle": None, "full_digests_equal_oracle": None}
    res["roofline_latency"] = latency_roofline(dag.critical_path(slots), res["device_ms_per_step"])
    st = g.stats()
    ach = st.total_blocks * 64 / (full_ms * 1e-3) / 1e9
    res["roofline_full"] = {"bound": "valu", "achieved": round(ach, 2), "peak": round(SHA_VALU_PEAK_GBS, 1),
                            "unit": "GB/s", "frac": round(ach / SHA_VALU_PEAK_GBS, 4)}
    res["canonicalize"] = bench_canon(ctx, g, dag)
    if "checkpoint" not in args.skip and budget.allow("checkpoint", 25):
        res["checkpoint"] = bench_checkpoint(ctx, g, a, t_build + t_load + full_ms * 1e-3)
    # the configs[2] CPU legs need the host arrays (rank 0, N = 1)
    res["_cpu"] = {"a": a, "dag": dag, "slots": slots, "old": old, "new": new,
                   "gpu_dirty_jobs": int(n_dirty_jobs), "snap_full": snap_full, "snap_new": snap_new}
    for b in (d_slots, d_old, d_new):
        b.free()
    g.close()
    return res


def bench_dag100m(args, dist, ctx, comm, budget):
    """configs[3]'s DAG, strong scaling: ONE global 1000align DAG of
    c4_parts x c4_samples samples (8 x 27,594 x P=32: 100M nodes, 121.6M
    jobs) cut into parts by sample subtree (workloads.PartitionedDag1000,
    SURVEY §8(e)); N ranks hold 8/N parts each -- N = 1 all of it, no
    exchange.  1% of the GLOBAL leaf File IDs toggle per step (every rank
    its own share of the same change set); with N > 1 a step is the local
    recompute, one fixed exchange round of the part roots (RCCL all-gather
    over xGMI) and rank 0's global root -- queued on the stream, no host
    round trip.  Dirty-node and block counts come from the layout
    (PartitionedDag1000.dirty_work, pinned against the oracle in
    tests/test_partition.py) and are checked against the device's count."""
    nparts, S, P = args.c4_parts, args.c4_samples, args.dag_pairs
    if nparts % dist.world:
        raise SystemExit("--c4-parts %d is not a multiple of the %d ranks" % (nparts, dist.world))
    t0 = time.perf_counter()
    pc = PartitionedDag1000(S, P, dist.world, dist.rank, nparts=nparts)
    a = pc.desc
    t_build = time.perf_counter() - t0
    g = capi.Graph.from_arrays(ctx, a)
    g.set_slots(pc.dag.file_slots, pc.dag.leaf_ids)
    t_load = time.perf_counter() - t0 - t_build
    nodes_global = dist.sum(pc.n_nodes - (3 * (dist.world - 1) if dist.rank else 0))  # the ref chain once
    log("C4 DAG: rank %d of %d holds %d of %d parts: %d nodes, %d jobs (%.1f GB of templates) built in %.1f s, "
        "loaded in %.1f s" % (dist.rank, dist.world, pc.k, nparts, pc.n_nodes, len(a["out_slot"]),
                              g.stats().template_bytes / 1e9, t_build, t_load))
    multi = dist.world > 1
    if multi:
        g.set_part(pc.part)
        ag = None
        if comm is None:  # RF_BENCH_SHARE_GPU rehearsal (or no RCCL communicator): gloo host transport
            ag = lambda b: [x.tobytes() for x in np.split(dist.all_gather_bytes(np.frombuffer(b, np.uint8)), dist.world)]  # noqa: E731,E501

        def recompute(full, count=True):
            return g.recompute_part(comm=comm, allgather=ag, nranks=dist.world, full=full, count=count)
    else:
        def recompute(full, count=True):
            return g.recompute(full=full)
    recompute(True)  # first call also captures the hipGraphs (host work): untimed
    dist.barrier()
    ctx.sync()
    t1 = time.perf_counter()
    recompute(True)
    ctx.sync()
    dist.barrier()
    full_ms = dist.max(time.perf_counter() - t1) * 1e3
    every = np.arange(a["n_slots"], dtype=np.uint32)
    snap_full = g.get_slots(every)  # the full recompute's table (the original File IDs)
    n_files_global = 2 * P * S * nparts
    slots, old, new = pc.dag.change_set(0.01, n_global=n_files_global)
    d_slots = ctx.upload(slots if len(slots) else np.zeros(1, np.uint32))
    d_old = ctx.upload(old if len(slots) else np.zeros((1, 32), np.uint8))
    d_new = ctx.upload(new if len(slots) else np.zeros((1, 32), np.uint8))
    jobs_l, nodes_l, blocks_l = pc.dirty_work(slots)
    # one counted step: the device's dirty-job count against the layout's
    g.set_slots(slots, new)
    got_jobs = recompute(False)
    g.set_slots(slots, old)
    recompute(False)
    jobs_ok = dist.max(0.0 if got_jobs == jobs_l + pc.last_twice else 1.0) == 0.0
    state = {"v": 0}

    def step():
        ver = d_new if state["v"] == 0 else d_old
        state["v"] ^= 1
        if len(slots):
            g.set_slots_device(d_slots.ptr, ver.ptr, len(slots), ctx.stream)
        if multi:
            recompute(False, count=False)
        else:
            g.recompute_async(False, ctx.stream)

    steps = args.dag_steps
    t = timed_steps(dist, ctx, step, steps, 2)
    ctx.timer_start()
    for _ in range(steps):
        step()
    dev_ms = ctx.timer_stop() / steps
    # parity after the timed steps (untimed): one more incremental step to the
    # changed IDs -- its table re-derived job by job by the oracle (N = 1) --
    # and one back, which must equal the full recompute's table slot for slot
    if state["v"] == 1:
        step()
    step()
    ctx.sync()
    dist.barrier()
    snap_new = g.get_slots(every)
    step()
    ctx.sync()
    dist.barrier()
    back_equal = bool((g.get_slots(every) == snap_full).all())
    del snap_full
    inc_equal_full = dist.max(0.0 if back_equal else 1.0) == 0.0
    want_in = pc.dag.leaf_ids.copy()
    if len(slots):
        pos = np.searchsorted(pc.dag.file_slots, slots)
        assert (pc.dag.file_slots[pos] == slots).all()
        want_in[pos] = new
    inputs_ok = dist.max(0.0 if (snap_new[pc.dag.file_slots] == want_in).all() else 1.0) == 0.0
    oracle = None
    if not multi and "cpu" not in args.skip and budget.allow("dag100m_oracle", 25):
        oracle = oracle_check_table(a, snap_new)
    del snap_new
    nodes_all, blocks_all = dist.sum(nodes_l), dist.sum(blocks_l)
    per_rank = [dict(rank=i, **{k: int(v) for k, v in zip(("jobs", "dirty_nodes", "dirty_blocks"), row)})
                for i, row in enumerate(np.frombuffer(dist.all_gather_bytes(
                    np.array([len(a["out_slot"]), nodes_l, blocks_l], np.int64)), np.int64).reshape(-1, 3))] \
        if multi else None
    ops = blocks_all * SHA_OPS_PER_BLOCK
    res = {"workload": "configs[3] DAG, strong scaling: one 1000align DAG of %d parts x %d samples x P=%d (%d nodes), "
                       "%d parts per rank over %d ranks; per part a fan-in-32 Merge tree, the global root on rank 0; "
                       "1%% of the global leaf File IDs toggled per step" % (nparts, S, P, nodes_global, pc.k,
                                                                              dist.world),
           "nodes_global": int(nodes_global), "nodes_rank0": int(pc.n_nodes), "jobs_rank0": len(a["out_slot"]),
           "dirty_nodes_per_step": int(nodes_all), "dirty_blocks_per_step": int(blocks_all),
           "dirty_jobs_match_device": bool(jobs_ok),
           "incremental_equals_full": bool(inc_equal_full), "input_slots_ok": bool(inputs_ok),
           "digests_equal_oracle": None if oracle is None else oracle["jobs_mismatching"] == 0 and bool(inputs_ok),
           "oracle_parity": oracle,
           "ms_per_step": t / steps * 1e3, "device_ms_per_step_rank0": dev_ms,
           "mnodes_per_s": nodes_all * steps / t / 1e6,
           "effective_mnodes_per_s": nodes_global * steps / t / 1e6,
           "full_recompute_ms": full_ms,
           "build_s_rank0": round(t_build, 2), "load_s_rank0": round(t_load, 2),
           "exchange": ("none (1 rank)" if not multi else "RCCL all-gather of %d part roots" % nparts if comm
                        else "gloo host all-gather of %d part roots" % nparts),
           "per_rank": per_rank,
           # (N > 1: rank 0's path also runs through the global root, and
           # every part's chain is the same shape)
           "roofline_latency": latency_roofline(dist.max(float(pc.critical_path(slots))), t / steps * 1e3),
           "roofline_incremental": {
               "bound": "valu", "achieved_tops": round(ops / (t / steps) / 1e12, 3),
               "peak_tops": round(dist.world * VALU_LANE_OPS / 1e12, 1),
               "frac": round(ops / (t / steps) / (dist.world * VALU_LANE_OPS), 4),
               "note": "dirty material blocks x 1464 ops per step / wall time per step, against the INT32 "
                       "VALU peak of the ranks' GPUs",
               "traffic": k2_traffic("100m") if not multi else None}}
    for b in (d_slots, d_old, d_new):
        b.free()
    g.close()
    return res


# The strong-scaling bound of a layout: a rank's piece can step no faster than
# its critical path -- the longest chain of dependent compressions a change
# starts -- at the measured per-block rate of a one-message chain: K1's duo
# chain (the fastest measured, us_per_chain_block of the SHA leg's duo launch,
# else its round-4 figure) and K2's two-lane link rounds (1.44 us a block,
# DESIGN.md §5).  The exchange is one all-gather of the part roots' 32-B
# digests a step (RCCL over xGMI); its latency is an ESTIMATE, not measured
# on this one-GPU box, and is not folded into any measured time.
DUO_US_PER_BLOCK_R04 = 1.13
K2_US_PER_BLOCK = 1.44
EXCHANGE_EST_US = 20.0


def piece_bounds(crit_blocks, n1_ms, duo_us=None):
    duo = duo_us or DUO_US_PER_BLOCK_R04
    f_duo, f_k2 = crit_blocks * duo * 1e-3, crit_blocks * K2_US_PER_BLOCK * 1e-3
    return {"critical_path_blocks": int(crit_blocks),
            "floor_ms": round(f_duo, 4), "floor_ms_k2_link_rate": round(f_k2, 4),
            "floor_rate_us_per_block": round(duo, 4),
            "speedup_bound_8": round(n1_ms / f_duo, 3) if f_duo else None,
            "speedup_bound_8_with_exchange_est": round(n1_ms / (f_duo + EXCHANGE_EST_US * 1e-3), 3) if f_duo else None,
            "exchange_est_us": EXCHANGE_EST_US,
            "bound_kind": "N = 1 ms / (critical path blocks x the measured one-chain rate: K1 duo %s us/block); "
                          "the exchange term (one boundary all-gather a step) is an estimate, not measured"
                          % round(duo, 3)}


def bench_piece(args, ctx, ranks, n1_ms, duo_us=None, per_sample=False):
    """N = 1 only: rank 0's piece of the strong-scaling layout at `ranks`
    ranks, stepped on this GPU like bench_dag100m's rank 0 but with no
    exchange -- what one GPU of a `ranks`-GPU run hashes per step, so the
    1 -> N curve's DAG ceiling is visible before the driver's SCALE run.
    Layouts: the bench's (8/ranks parts of configs[3]'s DAG, each with a
    fan-in-32 Merge tree, the global root on rank 0), or per_sample -- SURVEY
    §8(d) C3/C4 as written: per-sample roots only (no Merge tree, no global
    root; /root/reference/doc/1000align/1000align.rf:1-50 is per sample), the
    shared reference-index chain replicated, an empty boundary."""
    S, P, nparts = args.c4_samples, args.dag_pairs, args.c4_parts
    if per_sample:
        dag = Dag1000(S * nparts // ranks, P)
        desc, crit_of = dag.arrays(), dag.critical_path
        slots, old, new = dag.change_set(0.01, n_global=2 * P * S * nparts)
        n_nodes, file_slots, leaf_ids = dag.n_nodes, dag.file_slots, dag.leaf_ids
    else:
        pc = PartitionedDag1000(S, P, ranks, 0, nparts=nparts)
        desc, crit_of = pc.desc, pc.critical_path
        slots, old, new = pc.dag.change_set(0.01, n_global=2 * P * S * nparts)
        n_nodes, file_slots, leaf_ids = pc.n_nodes, pc.dag.file_slots, pc.dag.leaf_ids
    g = capi.Graph.from_arrays(ctx, desc)
    g.set_slots(file_slots, leaf_ids)
    g.recompute(True)
    d_slots, d_old, d_new = ctx.upload(slots), ctx.upload(old), ctx.upload(new)
    every = np.arange(desc["n_slots"], dtype=np.uint32)
    full = g.get_slots(every)
    state = {"v": 0}

    def step():
        ver = d_new if state["v"] == 0 else d_old
        state["v"] ^= 1
        g.set_slots_device(d_slots.ptr, ver.ptr, len(slots), ctx.stream)
        g.recompute_async(False, ctx.stream)

    for _ in range(2):
        step()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.dag_steps):
        step()
    ctx.sync()
    ms = (time.perf_counter() - t0) / args.dag_steps * 1e3
    if state["v"] == 1:
        step()
    ctx.sync()
    same = bool((g.get_slots(every) == full).all())
    for b in (d_slots, d_old, d_new):
        b.free()
    g.close()
    log("  rank 0's piece at %d ranks%s: %d nodes, %.4f ms/step (N = 1: %.4f ms, ratio %.2f)"
        % (ranks, " (per-sample roots)" if per_sample else "", n_nodes, ms, n1_ms, n1_ms / ms))
    return {"ranks": ranks, "nodes": int(n_nodes), "changed_slots": int(len(slots)), "ms_per_step": round(ms, 4),
            "projected_speedup": round(n1_ms / ms, 3), "incremental_equals_full": same,
            **piece_bounds(crit_of(slots), n1_ms, duo_us),
            "what": "rank 0's piece of the %s layout at %d ranks, local step only (no exchange), on this GPU; "
                    "projected_speedup = the layout's N = 1 ms/step / this"
                    % ("per-sample-root (SURVEY C3/C4)" if per_sample else "strong Merge-tree", ranks)}


def bench_persample(args, dist, ctx, duo_us=None):
    """SURVEY §8(d) C3/C4's DAG as written: 8 x c4_samples samples of the
    1000align DAG (100M nodes) with per-sample roots and no Merge tree --
    /root/reference/doc/1000align/1000align.rf:37-47 runs one module per
    sample, so the samples are independent.  Strong scaling like
    bench_dag100m: N ranks hold S x 8 / N consecutive samples each (the
    shared reference-index chain replicated), the global change set (1 % of
    the global leaf File IDs) restricted to each rank's slice, and NO
    exchange -- the boundary is empty.  At N = 1 also rank 0's piece at 8
    ranks (bench_piece), the 8-GPU projection; at N > 1 the measured step is
    the max over ranks.  Reported beside the Merge-tree layout at every N."""
    S, P, nparts = args.c4_samples, args.dag_pairs, args.c4_parts
    world, rank = dist.world, dist.rank
    if (S * nparts) % world:
        raise SystemExit("the per-sample layout's %d samples do not split over %d ranks" % (S * nparts, world))
    s_rank = S * nparts // world
    t0 = time.perf_counter()
    dag = Dag1000(s_rank, P, sample0=rank * s_rank)
    a = dag.arrays()
    g = capi.Graph.from_arrays(ctx, a)
    g.set_slots(dag.file_slots, dag.leaf_ids)
    g.recompute(True)
    slots, old, new = dag.change_set(0.01, n_global=2 * P * S * nparts)
    if not len(slots):
        raise SystemExit("rank %d: empty change set" % rank)
    d_slots, d_old, d_new = ctx.upload(slots), ctx.upload(old), ctx.upload(new)
    every = np.arange(a["n_slots"], dtype=np.uint32)
    full = g.get_slots(every)
    state = {"v": 0}

    def step():
        ver = d_new if state["v"] == 0 else d_old
        state["v"] ^= 1
        g.set_slots_device(d_slots.ptr, ver.ptr, len(slots), ctx.stream)
        g.recompute_async(False, ctx.stream)

    t = timed_steps(dist, ctx, step, args.dag_steps, 2)
    ms = t / args.dag_steps * 1e3
    if state["v"] == 1:
        step()
    ctx.sync()
    same = dist.max(0.0 if (g.get_slots(every) == full).all() else 1.0) == 0.0
    for b in (d_slots, d_old, d_new):
        b.free()
    g.close()
    del full
    f = np.asarray(slots, dtype=np.int64)
    pairs, samples = np.unique(f // 2), np.unique(f // 2 // P)
    n_dirty_l = int(2 * len(f) + 10 * len(pairs) + 5 * len(samples))  # Val + Coerce a file, the pair chain, the tail
    n_dirty = int(dist.sum(n_dirty_l))
    nodes = int(dist.sum(dag.n_nodes - (3 if rank else 0)))  # (the replicated ref chain counted once)
    crit = int(dist.max(float(dag.critical_path(slots))))
    log("  per-sample-root layout (SURVEY C3/C4): %d nodes over %d rank(s), %.4f ms/step, built+loaded in %.1f s"
        % (nodes, world, ms, time.perf_counter() - t0))
    res = {"workload": "SURVEY §8(d) C3/C4 as written: 1000align DAG of %d samples x P=%d (%d nodes), per-sample "
                       "roots, no Merge tree or global root, %d samples per rank over %d rank(s), no exchange; 1%% of "
                       "the global leaf File IDs toggled per step" % (S * nparts, P, nodes, s_rank, world),
           "nodes": nodes, "ranks": world, "ms_per_step": round(ms, 4), "incremental_equals_full": same,
           "dirty_nodes_per_step": n_dirty,
           "mnodes_per_s": round(n_dirty / (ms * 1e-3) / 1e6, 1),
           "critical_path_blocks": crit}
    del dag, a
    if world == 1:
        pc8 = bench_piece(args, ctx, 8, ms, duo_us, per_sample=True)
        res["piece_8"] = pc8
        res["piece_ms_8"], res["projected_speedup_8"] = pc8["ms_per_step"], pc8["projected_speedup"]
    return res


def oracle_check_table(a, table):
    """Checker leg (untimed, rank 0 at N = 1): the oracle re-derives every
    job of a GPU slot table from that table's own hole digests
    (orc_graph_check, flow.go:675-750 per node on cpu_threads() threads);
    with the input slots at their assigned values (checked by the caller)
    this is the table's parity with the full evaluation."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import reflow_oracle as O  # the oracle: as the checker only
    th = cpu_threads()
    t0 = time.perf_counter()
    bad, first = O.check_slots(a, table, th)
    dt = time.perf_counter() - t0
    log("  oracle check: %d jobs re-derived on %d threads in %.1f s: %d mismatching"
        % (len(a["out_slot"]), th, dt, bad))
    return {"what": "every job of the GPU's table after an incremental step re-hashed by the oracle from the "
                    "table's own hole digests (orc_graph_check); inputs checked against the change set",
            "jobs_checked": int(len(a["out_slot"])), "jobs_mismatching": bad, "first_bad_job": first,
            "seconds": round(dt, 2), "threads": th}


def bench_checkpoint(ctx, g, a, cold_s):
    """Checkpoint / resume of the loaded configs[2] graph (rf_graph_save /
    rf_graph_restore): the file holds the lowered device form and
    every slot digest, so a restarted process resumes incremental steps
    without lowering, level analysis or a full recompute.  cold_s: what the
    same process paid to get there (build + load + full recompute)."""
    import shutil
    import tempfile
    d = tempfile.mkdtemp(prefix="rf_ckpt_")
    try:
        path = os.path.join(d, "c3.ckpt")
        t0 = time.perf_counter()
        g.save(path)
        save_s = time.perf_counter() - t0
        size = os.path.getsize(path)
        t0 = time.perf_counter()
        r = capi.Graph.restore(ctx, path)
        restore_s = time.perf_counter() - t0
        every = np.arange(a["n_slots"], dtype=np.uint32)
        same = bool((r.get_slots(every) == g.get_slots(every)).all())
        r.close()
    finally:
        shutil.rmtree(d, ignore_errors=True)
    log("  checkpoint: %.2f GB saved in %.1f s, restored in %.1f s (cold start %.1f s), slots equal: %s"
        % (size / 1e9, save_s, restore_s, cold_s, same))
    return {"file_bytes": size, "save_s": round(save_s, 2), "restore_s": round(restore_s, 2),
            "cold_start_s": round(cold_s, 2), "slots_equal": same,
            "what": "rf_graph_save after the timed steps, rf_graph_restore into a new graph, every slot compared"}


def first_index_of_equal(dig):
    """For rows of 32-B digests: the first row index holding an equal digest
    (flowMap.Put keeps the first flow of each digest, flow.go:897-907) --
    a stable sort by the first 64-bit word, then each run's minimum; if two
    different digests share that word (~n^2/2^65) the full lexicographic
    sort decides."""
    n = len(dig)
    w = np.ascontiguousarray(dig).view(np.uint64).reshape(n, 4)
    order = np.argsort(w[:, 0], kind="stable")
    sw = w[order, 0]
    start = np.ones(n, dtype=bool)
    start[1:] = sw[1:] != sw[:-1]
    run = np.cumsum(start) - 1
    out = np.empty(n, dtype=np.int64)
    out[order] = order[start][run]
    if (w[out] == w).all():
        return out
    order = np.lexsort((np.arange(n), w[:, 3], w[:, 2], w[:, 1], w[:, 0]))
    sw = w[order]
    start = np.ones(n, dtype=bool)
    start[1:] = (sw[1:] != sw[:-1]).any(axis=1)
    run = np.cumsum(start) - 1
    first_of_run = order[start]  # the lowest index of each run (the sort is stable by index)
    out = np.empty(n, dtype=np.int64)
    out[order] = first_of_run[run]
    return out


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
    ok = nu == dag.n_nodes and n == dag.n_nodes + 3 * (dag.S - 1) and bool(
        (canon[:3 * dag.S].reshape(dag.S, 3) == np.arange(3)).all())
    # every canon[i] against flowMap's answer computed on the host: the first
    # index in Put order holding an equal digest (flow.go:897-907)
    dig = d_dig.to_numpy().reshape(n, 32)
    want = first_index_of_equal(dig)
    canon_equal = bool((canon.astype(np.int64) == want).all())
    res = {"workload": "dedup of %d node digests (C3 DAG + %d duplicated ref-index nodes)" % (n, 3 * (dag.S - 1)),
           "ms": ms, "mnodes_per_s": n / (ms * 1e-3) / 1e6, "unique": nu, "parity_ok": ok,
           "canon_equal_host": canon_equal,
           "canon_check": "every canon[i] == the first index with an equal 32-B digest (host, numpy sort)",
           "random_accesses_per_node": 3,
           "achieved_g_accesses_per_s": round(3 * n / (ms * 1e-3) / 1e9, 2)}
    for b in (d_idx, d_dig, d_canon, d_nu):
        b.free()
    return res


# --------------------------------------------------------------- C5: probe --
def probe_case(ctx, dist, n_ins, n_probe, steps, seed):
    """Filter of n_ins keys (bloom.NewWithEstimates(n, 0.001), eval.go:838-843)
    and n_probe probes: the inserted keys repeated to half the batch, then
    fresh keys.  Keys generated on the device."""
    m = int(math.ceil(-1 * float(n_ins) * math.log(0.001) / math.pow(math.log(2), 2)))
    k = int(math.ceil(math.log(2) * float(m) / float(n_ins)))
    half = n_probe // 2
    # rows [0, n_ins): the inserted keys.  n_ins <= half: probes = the inserted
    # keys repeated to half the batch, then fresh keys; else probes = the last
    # `half` inserted keys, then fresh keys after them.
    lens = np.array([32 * n_ins, 32 * (n_probe - half)], dtype=np.uint64)
    if n_ins <= half:
        rows, offs = n_probe, np.array([0, 32 * half], dtype=np.uint64)
    else:
        rows, offs = n_ins + n_probe - half, np.array([0, 32 * n_ins], dtype=np.uint64)
    keys = ctx.alloc(32 * rows)
    d_offs, d_lens = ctx.upload(offs), ctx.upload(lens)
    ctx.gen_fill(keys.ptr, d_offs.ptr, d_lens.ptr, 2, seed, 32 * rows)
    ctx.sync()
    if n_ins <= half:
        rep = half // n_ins
        for r in range(1, rep):
            capi._check(capi.lib().rf_memcpy_d2d(ctx.handle, keys.ptr + 32 * n_ins * r, keys.ptr, 32 * n_ins))
        present = rep * n_ins
        probe_ptr = keys.ptr
    else:
        present = half
        probe_ptr = keys.ptr + 32 * (n_ins - half)
    b = capi.Bloom.new(ctx, m, k)
    ctx.timer_start()
    b.add_device(keys.ptr, n_ins, ctx.stream)
    add_ms = ctx.timer_stop()
    out = ctx.alloc(n_probe)

    def step():
        b.probe_device(probe_ptr, n_probe, out.ptr, ctx.stream)

    t = timed_steps(dist, ctx, step, steps, 1)
    ctx.timer_start()
    step()
    dev_ms = ctx.timer_stop()
    o_np = out.to_numpy()
    hits = int(o_np.astype(np.int64).sum())
    no_false_negative = bool(o_np[:present].all())  # every inserted key's probe says "contains"
    del o_np
    fresh = n_probe - present
    fp = (hits - present) / max(fresh, 1)
    bpp = 32 + 8 * k + 1
    ach = n_probe * bpp / (dev_ms * 1e-3) / 1e9
    f = float(np.bitwise_count(b.words()).sum()) / m
    absent = n_probe - hits
    reads = hits * k + absent * sum(f ** j for j in range(k))
    gread_s = reads / (dev_ms * 1e-3) / 1e9
    ceil = gather_ceiling(m // 8, n_probe // 4, k)
    res = {"workload": "bloomlive probe: n=%d keys (m=%d bits, %.1f MiB, k=%d), %d probes (%.0f%% present)"
                       % (n_ins, m, m / 8 / 2**20, k, n_probe, 100.0 * present / n_probe),
           "gprobes_per_s": dist.sum(n_probe) * steps / t / 1e9,
           "device_ms": dev_ms, "add_ms": add_ms, "false_positive_rate": fp,
           "no_false_negatives": no_false_negative, "present": present,
           "false_positives": hits - present,
           "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 4), "bytes_per_probe": bpp,
                        "note": "algorithmic bytes; each random 8-B word read moves a 64-B line, so the "
                                "real bound is the random-gather rate (roofline_gather)"},
           "roofline_gather": {"bound": "random 8-B gathers", "achieved": round(gread_s, 2),
                               "peak": round(ceil, 2) if ceil else None, "unit": "G words/s",
                               "frac": round(gread_s / ceil, 4) if ceil else None,
                               "words_per_probe": round(reads / n_probe, 3), "filter_fill": round(f, 4),
                               "peak_kind": "measured live: tools/micro.hip k_gather, k independent "
                                            "random 8-B reads per thread over a table of the filter's size"}}
    return res, {"keys": keys, "probe_ptr": probe_ptr, "out": out, "bloom": b, "hits": hits, "m": m, "k": k,
                 "extra": (d_offs, d_lens), "ceil": ceil, "present": present}


def bench_probe(args, dist, ctx, budget):
    n_ins, n_probe = args.probe_keys, args.probes
    res, h = probe_case(ctx, dist, n_ins, n_probe, args.probe_steps, 0x5EED0005 + dist.rank)
    keys, out, b, hits = h["keys"], h["out"], h["bloom"], h["hits"]
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
    res["collect"] = {"objects": n_probe, "dead": n_dead, "dead_matches_probe": n_dead == n_probe - hits,
                      "ms": coll_ms, "g_objects_per_s": n_probe / (coll_ms * 1e-3) / 1e9,
                      "overhead_vs_probe": round(coll_ms / res["device_ms"], 3)}
    res["assoc"] = bench_assoc(ctx, keys, n_ins, n_probe, hits)
    ceil = h["ceil"]
    if ceil and res["assoc"]:
        a = res["assoc"]
        ga = 3 * n_probe / (a["get_ms"] * 1e-3) / 1e9
        a["roofline_gather"] = {"achieved": round(ga, 2), "peak": round(ceil, 2), "unit": "G random accesses/s",
                                "frac": round(ga / ceil, 3),
                                "accesses_per_get": "3 (tag, 32-B key compare, 32-B value on a hit; absent keys "
                                                    "stop at an empty tag: 1-2)"}
    # bounded sample for the CPU leg (rank 0, N = 1): the filter words and
    # the first 2e7 probe keys
    if dist.world == 1 and "cpu" not in args.skip:
        ns = min(n_probe, 20_000_000)
        res["_cpu"] = {"words": b.words(), "length": b.params()[2], "m": h["m"], "k": h["k"],
                       "keys": keys.to_numpy(count=32 * ns), "n": ns, "gpu_bits": out.to_numpy(count=ns)}
    for x in (keys, out) + h["extra"]:
        x.free()
    b.close()
    res["_gather_ceiling"] = ceil
    # SURVEY §8(d) C5 second case: n = 1.2e9 keys -> m = 17.25 G bits (2.0 GiB):
    # larger than the 256 MB MALL, so the gathers go to HBM
    if args.probe_big_keys and budget.allow("probe_2gib_filter", 25, everyone=True):
        rb, hb = probe_case(ctx, dist, args.probe_big_keys, n_probe, args.probe_steps, 0x5EED0015 + dist.rank)
        for x in (hb["keys"], hb["out"]) + hb["extra"]:
            x.free()
        hb["bloom"].close()
        res["filter_2gib"] = rb
        log("  probe 2 GiB filter: %.2f G probes/s (171 MiB: %.2f)" % (rb["gprobes_per_s"], res["gprobes_per_s"]))
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
    # sampled parity with the Go map the reference's test assoc is
    # (test/testutil/assoc.go:34-56): a dict of the first 2M Puts, asked for
    # the first 1M probes (inserted keys) and the last 1M (fresh keys)
    ns = min(1_000_000, n_ins, n_probe // 2)
    d = dict(zip(map(bytes, keys.to_numpy(count=32 * 2 * ns).reshape(-1, 32)),
                 map(bytes, vals.to_numpy(count=32 * 2 * ns).reshape(-1, 32))))
    assoc_ok = True
    for lo in ((0, n_probe - ns) if n_ins <= n_probe // 2 else (0,)):  # (rows past n_ins: fresh keys)
        pk = keys.to_numpy(count=32 * ns, offset=32 * lo).reshape(ns, 32)
        gv = d_v.to_numpy(count=32 * ns, offset=32 * lo).reshape(ns, 32)
        gf = d_f.to_numpy(count=ns, offset=lo)
        for i in range(ns):
            w = d.get(bytes(pk[i]))
            if (w is None) != (gf[i] == 0) or (w is not None and w != bytes(gv[i])):
                assoc_ok = False
                break
    del d
    for b in (vals, st, d_v, d_f):
        b.free()
    n_nodes = min(2_000_000, n_ins)
    logical = keys.to_numpy(count=32 * n_nodes).reshape(n_nodes, 32)
    physical = np.random.default_rng(0x5EED0007).integers(0, 256, size=(n_nodes, 32), dtype=np.uint8)
    node_keys = np.stack([physical, logical], axis=1).reshape(-1)
    ptr = np.arange(0, 2 * n_nodes + 1, 2, dtype=np.uint64)
    t0 = time.perf_counter()
    which, fsids, kf, _ = a.lookup(0, node_keys, ptr)
    a.repair(0, node_keys, ptr, which, fsids, kf)  # precise; every fsid taken as verified
    lk_s = time.perf_counter() - t0
    _, f2 = a.get(0, physical)
    lookup = {"workload": "%d nodes x 2 cache keys (physical absent, logical present), precise read repair"
                          % n_nodes,
              "ms": lk_s * 1e3, "m_nodes_per_s": n_nodes / lk_s / 1e6,
              "hits_on_logical": int((which == 1).sum()), "repaired": int(f2.astype(np.int64).sum()),
              "note": "host API: keys H2D, one Get batch, first-hit select on the device (rf_assoc_lookup), "
                      "then the precise repair Put batch (rf_assoc_repair)"}
    a.close()
    return {"workload": "Put %d keys (one batch), Get %d keys (%d present)" % (n_ins, n_probe, found),
            "put_ms": put_s * 1e3, "put_mkeys_per_s": n_ins / put_s / 1e6, "put_ok": ok_put,
            "get_ms": get_ms, "get_g_keys_per_s": n_probe / (get_ms * 1e-3) / 1e9,
            "found_exact": found == (n_probe // 2) // n_ins * n_ins,
            "get_equal_dict": assoc_ok,
            "get_check": "%d inserted + %d fresh probe keys: found flag and value vs a dict of the Puts" % (ns, ns),
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


def valu_ceiling():
    """SHA-256's measured VALU ceiling on this GPU, T int32 ops/s: every lane
    of 8 waves per SIMD compresses register data (tools/micro.hip k_compute,
    the same sha256_compress as the K1/K2 lane paths; 1464 canonical ops a
    block).  Beside the 78.6 T spec peak every VALU roofline is also given
    against this (the op mix's 8-byte VOP3 forms issue slower
    than the spec's one op per lane per clock).  None without tools/_micro.so."""
    import ctypes
    so = os.path.join(ROOT, "tools", "_micro.so")
    if not os.path.exists(so):
        return None
    L = ctypes.CDLL(so)
    L.micro_compute.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    L.micro_compute.restype = ctypes.c_float
    grid, nblk = N_CU * 8, 1000
    L.micro_compute(grid, 20)  # (code and clocks warm)
    ms = L.micro_compute(grid, nblk)
    return grid * 256 * nblk * SHA_OPS_PER_BLOCK / (ms * 1e-3) / 1e12 if ms > 0 else None


def with_measured_valu(line, tops):
    """Every VALU frac of the line, again against the measured ceiling."""
    if not tops:
        return
    gbps = tops * 1e12 / SHA_OPS_PER_BLOCK * 64 / 1e9
    for r in [line.get("roofline")] + list(line.get("roofline_gpu_legs") or []) + [line.get("roofline_gpu_only")]:
        if r and r.get("frac_of_valu_peak") is not None:
            r["frac_of_measured_valu"] = round(r["frac_of_valu_peak"] * SHA_VALU_PEAK_GBS / gbps, 6)
    inc = line.get("incremental") or {}
    if inc.get("roofline_full"):
        rf = inc["roofline_full"]
        rf["frac_of_measured_valu"] = round(rf["achieved"] / gbps, 4)
    for d in (line.get("incremental_100m") or {}, (line.get("incremental_100m") or {}).get("per_sample_layout") or {}):
        ri = d.get("roofline_incremental")
        if ri:
            ri["frac_of_measured_valu"] = round(ri["achieved_tops"] / tops, 4)
            ri["measured_valu_tops"] = round(tops, 2)


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
    non-goroutine-safe Contains, and the host leg's thread count), and
    Go-map-shaped dedup and lookups (a Python dict over 32-B keys)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import reflow_oracle as O
    L = O.lib()
    c = probe["_cpu"]
    words = np.ascontiguousarray(c["words"])
    keys = np.ascontiguousarray(c["keys"])
    out = np.zeros(c["n"], dtype=np.uint8)
    r = {}
    th_n = cpu_threads()
    for th, n in ((1, min(c["n"], 2_000_000)), (th_n, c["n"])):
        t0 = time.perf_counter()
        L.orc_bloomlive_contains_batch(words.ctypes.data, int(c["length"]), int(c["m"]), int(c["k"]),
                                       keys.ctypes.data, n, out.ctypes.data, th)
        dt = time.perf_counter() - t0
        r["probe_%dt" % th] = {"value": n / dt / 1e9, "unit": "G probes/s", "cores": th, "kind": "port",
                               "sample": "%d probes of the configs[4] set against its filter" % n}
    # the last run covered every sampled key: the GPU's answers bit for bit
    r["probe_bits_equal_gpu"] = bool(((out != 0) == (c["gpu_bits"] != 0)).all())
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


def cpu_threads():
    """min(60, the CPU share): DigestLimiter (local/executor.go:41) on the
    cores this process may use -- the same width as the host leg."""
    ctx_threads = int(os.environ.get("RF_BENCH_CPU_THREADS", "0"))
    if ctx_threads:
        return ctx_threads
    share = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            share = min(share, -(-int(q) // int(p)))
    except (OSError, ValueError):
        pass
    return max(1, min(60, share))


def cpu_baseline(args, sha, dag_res, budget):
    """The headline's CPU leg: the oracle's scalar C port (~Go 1.9/1.10 speed
    class, kind "port") on a bounded sample of configs[1] -- the value; beside
    it OpenSSL SHA-256 (libcrypto from C on native threads, oracle/
    baseline_openssl.c; SHA-NI, what Go >= 1.21 crypto/sha256 uses) over the
    WHOLE set on min(60, CPU share) threads, LPT order; configs[0];
    configs[2] on its own DAG and change set (1 thread: Canonicalize is
    serial)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import reflow_oracle as O  # the oracle: cpu_baseline leg only
    L = O.lib()
    threads = cpu_threads()
    lens, offs = sha["_lens"], sha["_offs"]
    res = {"cores": threads, "cpu_model": cpu_model(), "sha_ni": "sha_ni" in open("/proc/cpuinfo").read()}
    # the set itself, copied out of HBM (not timed)
    t0 = time.perf_counter()
    host = sha["_arena"].to_numpy()
    log("cpu: copied the %.1f GiB set to host memory in %.1f s" % (host.nbytes / GiB, time.perf_counter() - t0))
    order = np.ascontiguousarray(np.argsort(-lens.astype(np.int64), kind="stable").astype(np.uint64))
    a_offs, a_lens = np.ascontiguousarray(offs, dtype=np.uint64), np.ascontiguousarray(lens, dtype=np.uint64)
    dig = np.zeros((len(lens), 32), dtype=np.uint8)
    t0 = time.perf_counter()
    rc = L.orc_openssl_sha256_batch(host.ctypes.data, a_offs.ctypes.data, a_lens.ctypes.data, order.ctypes.data,
                                    len(lens), dig.ctypes.data, threads)
    dt = time.perf_counter() - t0
    ok = rc == 0 and bool((dig == sha["_digests"]).all())
    res["openssl"] = {"value": float(lens.sum()) / dt / 1e9, "unit": "GB/s", "kind": "library", "cores": threads,
                      "what": "SHA-256 of every configs[1] file, OpenSSL libcrypto (SHA-NI) on %d native threads "
                              "taking files largest first from one queue (oracle/baseline_openssl.c)" % threads,
                      "sample": "the whole configs[1] set (%d files, %.1f GiB)" % (len(lens), lens.sum() / GiB),
                      "seconds": dt, "gpu_digests_match": ok}
    # scalar port on a bounded sample (files in generation order up to the budget)
    budget_b = int(args.cpu_sample_gib * GiB)
    n = min(int(np.searchsorted(np.cumsum(lens.astype(np.int64)), budget_b)) + 1, len(lens))
    s_lens = np.ascontiguousarray(lens[:n])
    s_offs = np.ascontiguousarray(offs[:n])
    s_order = np.argsort(-s_lens.astype(np.int64), kind="stable").astype(np.uint64)
    o_offs, o_lens = np.ascontiguousarray(s_offs[s_order]), np.ascontiguousarray(s_lens[s_order])
    out = np.zeros((n, 32), dtype=np.uint8)
    t0 = time.perf_counter()
    L.orc_sha256_batch(host.ctypes.data, o_offs.ctypes.data, o_lens.ctypes.data, n, out.ctypes.data, threads)
    dt = time.perf_counter() - t0
    back = np.empty_like(out)
    back[s_order.astype(np.int64)] = out
    # the cpu_baseline proper: the oracle's port (the reference is Go and
    # cannot be built here) on a bounded sample of the same workload
    res.update({"value": float(s_lens.sum()) / dt / 1e9, "unit": "GB/s", "kind": "port",
                "what": "oracle/oracle.c scalar SHA-256 (the Go 1.9/1.10 speed class: no SHA-NI) on %d threads "
                        "(min(60, CPU share): DigestLimiter), largest-first" % threads,
                "sample": "first %d files (%.2f GiB, largest %.2f GiB) of configs[1]"
                          % (n, s_lens.sum() / GiB, s_lens.max() / GiB),
                "seconds": dt, "gpu_digests_match": bool((back == sha["_digests"][:n]).all()),
                # the same cores with SHA-NI (what Go >= 1.21 crypto/sha256 runs): the
                # CPU figure the GPU step should be read against
                "value_openssl": res["openssl"]["value"],
                "note": "value = the scalar port (Go 1.9/1.10 speed class); value_openssl = OpenSSL SHA-NI on the "
                        "same %d threads over the whole set" % threads})
    del host
    # configs[0]: port and OpenSSL
    c1l = np.full(C1_N, C1_LEN, dtype=np.uint64)
    c1o, c1t = arena_layout(c1l, align=64)
    c1a = np.zeros(c1t, dtype=np.uint8)
    L.orc_fill_batch(C1_SEED, c1a.ctypes.data, c1o.ctypes.data, c1l.ctypes.data, C1_N, threads)
    c1out = np.zeros((C1_N, 32), dtype=np.uint8)
    t0 = time.perf_counter()
    L.orc_sha256_batch(c1a.ctypes.data, c1o.ctypes.data, c1l.ctypes.data, C1_N, c1out.ctypes.data, threads)
    c1_port = time.perf_counter() - t0
    c1ssl = np.zeros((C1_N, 32), dtype=np.uint8)
    c1o64 = np.ascontiguousarray(c1o, dtype=np.uint64)
    best = None
    for _ in range(3):  # (1 GiB takes ~30 ms on 16 threads: the best of three)
        t0 = time.perf_counter()
        rc = L.orc_openssl_sha256_batch(c1a.ctypes.data, c1o64.ctypes.data, c1l.ctypes.data, None, C1_N,
                                        c1ssl.ctypes.data, threads)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    c1_ssl = best
    res["c1"] = {"sample": "configs[0] in full: 4096 x 256 KiB", "port_ms": c1_port * 1e3,
                 "port_gbps": C1_N * C1_LEN / c1_port / 1e9, "openssl_ms": c1_ssl * 1e3,
                 "openssl_gbps": C1_N * C1_LEN / c1_ssl / 1e9, "cores": threads,
                 "openssl_equals_port": rc == 0 and bool((c1ssl == c1out).all()),
                 "openssl_what": "OpenSSL libcrypto on %d native threads, one shared queue (oracle/baseline_openssl.c; "
                                 "best of 3)" % threads}
    del c1a
    # configs[2] on the CPU: the same 10M-node DAG and change set, 1 thread
    c = (dag_res or {}).get("_cpu")
    if c is not None and budget.allow("cpu_dag", 40):
        og = O.OGraph(c["a"])
        og.set_inputs(c["dag"].file_slots, c["dag"].leaf_ids)
        t0 = time.perf_counter()
        og.full()
        full_s = time.perf_counter() - t0
        full_eq = int((og.slots != c["snap_full"]).any(axis=1).sum())  # slots differing (0 = parity)
        t0 = time.perf_counter()
        hashed = og.update(c["slots"], c["new"])
        inc_s = time.perf_counter() - t0
        blocks = og.last_blocks()
        inc_eq = int((og.slots != c["snap_new"]).any(axis=1).sum())
        # and every job of the GPU's post-step table re-derived from its own
        # holes (orc_graph_check: job-local, threaded)
        bad, first = O.check_slots(c["a"], c["snap_new"], threads)
        if dag_res is not None:
            dag_res["digests_equal_oracle"] = inc_eq == 0 and bad == 0
            dag_res["full_digests_equal_oracle"] = full_eq == 0
            dag_res["oracle_parity"] = {
                "what": "every slot of the GPU's tables vs the oracle's serial evaluation (orc_graph_full; "
                        "orc_graph_update on the bench's change set), plus every job of the post-step table "
                        "re-hashed from its own holes (orc_graph_check)",
                "slots": int(len(og.slots)), "full_slots_differing": full_eq, "incremental_slots_differing": inc_eq,
                "jobs_checked": int(len(c["a"]["out_slot"])), "jobs_mismatching": bad, "first_bad_job": first}
        n_nodes = c["dag"].n_nodes
        res["dag_full"] = {"value": n_nodes / full_s / 1e6, "unit": "M graph nodes/s", "cores": 1, "kind": "port",
                           "what": "every digest recomputed, the reference's behaviour per Eval (flow.go:653-664 "
                                   "memoises per *Flow node only)",
                           "sample": "configs[2] in full: %d nodes / %d jobs, oracle/oracle.c orc_graph_full"
                                     % (n_nodes, c["dag"].n_jobs), "seconds": full_s}
        res["dag_incremental"] = {"value": (c["gpu_dirty_jobs"] - len(np.unique(c["slots"] // 2))) / inc_s / 1e6,
                                  "unit": "M dirty nodes/s", "cores": 1, "kind": "port",
                                  "sample": "configs[2] in full, the bench's own change set (1%% of leaf File IDs): "
                                            "%d jobs / %d blocks re-hashed (oracle/oracle.c orc_graph_update)"
                                            % (hashed, blocks),
                                  "seconds": inc_s, "jobs_equal_gpu": hashed == c["gpu_dirty_jobs"]}
        if dag_res is not None:
            dag_res["dirty_blocks_per_step"] = int(blocks)
            ops = blocks * SHA_OPS_PER_BLOCK
            dag_res["roofline_incremental"] = {
                "bound": "valu", "achieved_tops": round(ops / (dag_res["device_ms_per_step"] * 1e-3) / 1e12, 3),
                "peak_tops": round(VALU_LANE_OPS / 1e12, 1),
                "frac": round(ops / (dag_res["device_ms_per_step"] * 1e-3) / VALU_LANE_OPS, 4),
                "note": "dirty blocks x 1464 ops per step / device time; the step is latency-bound (fused "
                        "chains of dependent jobs), not throughput-bound",
                "traffic": k2_traffic("configs2")}
        og.close()
    return res


def parity_summary(sha, c1, dag, dag100, probe, cpu):
    """Every digest / answer check this run made, one boolean each (None =
    not run here: a section skipped, or a check that needs the N = 1 cpu
    leg).  `all` is true iff every check that ran passed."""
    def get(d, *path):
        for p in path:
            if not isinstance(d, dict) or d.get(p) is None:
                return None
            d = d[p]
        return bool(d)
    checks = {
        "configs1_ids_vs_openssl": get(cpu, "openssl", "gpu_digests_match"),
        "configs1_ids_vs_oracle_sample": get(cpu, "gpu_digests_match"),
        "configs1_gpu_only_equals_hybrid": get(sha, "gpu_only", "digests_equal_hybrid"),
        "configs0_fileset_vs_fixture": get(c1, "fixture_match"),
        "configs0_install_vs_fixture": get(c1, "install", "fileset_digest_match"),
        "configs2_incremental_vs_oracle": get(dag, "digests_equal_oracle"),
        "configs2_full_vs_oracle": get(dag, "full_digests_equal_oracle"),
        "configs2_incremental_equals_full": get(dag, "incremental_equals_full"),
        "configs2_dedup_vs_host": get(dag, "canonicalize", "canon_equal_host"),
        "configs2_checkpoint_slots": get(dag, "checkpoint", "slots_equal"),
        "configs3_incremental_vs_oracle": get(dag100, "digests_equal_oracle"),
        "configs3_incremental_equals_full": get(dag100, "incremental_equals_full"),
        "configs3_piece8_incremental_equals_full": get(dag100, "piece_8", "incremental_equals_full"),
        "configs3_dirty_jobs_vs_layout": get(dag100, "dirty_jobs_match_device"),
        "configs4_probe_vs_oracle": get(cpu, "probe_bits_equal_gpu"),
        "configs4_no_false_negatives": get(probe, "no_false_negatives"),
        "configs4_collect_vs_probe": get(probe, "collect", "dead_matches_probe"),
        "assoc_get_vs_dict": get(probe, "assoc", "get_equal_dict"),
    }
    ran = [v for v in checks.values() if v is not None]
    return {"all": bool(ran) and all(ran), "checks_run": len(ran), **checks}


def main():
    # stdout carries exactly ONE line, the JSON result: everything else any
    # library prints on the C-level stdout (gloo's "[Gloo] Rank r is
    # connected", RCCL's "RCCL version : ..." banner and NCCL WARN lines at
    # communicator init) goes to stderr; the result is written to the saved fd
    sys.stdout.flush()
    result_fd = os.dup(1)
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sha-gib", type=float, default=64.0)
    ap.add_argument("--dag-samples", type=int, default=22075)  # ~10M nodes at P=32
    ap.add_argument("--dag-pairs", type=int, default=32)
    ap.add_argument("--c4-samples", type=int, default=27594,
                    help="samples per part of configs[3]'s DAG (12.5M nodes per part)")
    ap.add_argument("--c4-parts", type=int, default=8,
                    help="parts of configs[3]'s DAG (8 x 12.5M = 100M nodes, fixed for every N: strong scaling)")
    ap.add_argument("--dag-steps", type=int, default=20)
    ap.add_argument("--probe-keys", type=int, default=100_000_000)
    ap.add_argument("--probe-big-keys", type=int, default=1_200_000_000)
    ap.add_argument("--probes", type=int, default=1_000_000_000)
    ap.add_argument("--probe-steps", type=int, default=3)
    ap.add_argument("--cpu-sample-gib", type=float, default=16.0)
    ap.add_argument("--gpu-only-run", type=int, default=1, help="one GPU-only run (duo roofline)")
    ap.add_argument("--budget-s", type=float, default=420.0)
    ap.add_argument("--skip", default="",
                    help="comma list of: lower,c1,install,dag,dag100m,piece,persample,checkpoint,probe,cpu")
    args = ap.parse_args()
    args.skip = set(filter(None, args.skip.split(",")))
    budget = Budget(args.budget_s)

    dist = Dist(args.gpus)
    budget.dist = dist
    # the product lowering leg runs first, in a child process of its own,
    # before this process touches the GPU (N = 1 only)
    lowering = None
    if dist.world == 1 and "lower" not in args.skip:
        lowering = bench_lowering(args)
    device = dist.local
    share = os.environ.get("RF_BENCH_SHARE_GPU") == "1"
    if share:  # rehearsal of the N-rank path on a box with fewer GPUs (never the driver's run)
        device = dist.local % max(capi.device_count(), 1)
    ctx = capi.Context(device)
    comm, exchange, rccl = None, "none (1 rank)", None
    if dist.world > 1:
        # RF_BENCH_TRY_RCCL=1 with RF_BENCH_SHARE_GPU: attempt the communicator anyway (RCCL refuses two
        # ranks on one GPU), which rehearses the fallback below
        if share and os.environ.get("RF_BENCH_TRY_RCCL") != "1":
            exchange = "gloo host all-gather (RF_BENCH_SHARE_GPU: RCCL needs one GPU per rank)"
        else:
            uid = dist.bcast_bytes(capi.Comm.unique_id() if dist.rank == 0 else None)
            err = None
            try:
                comm = capi.Comm(ctx, dist.world, dist.rank, uid)
            except Exception as e:  # noqa: BLE001 - keep the run: the DAG exchange then goes over gloo
                err, comm = str(e), None
            # every rank must take the same transport
            if dist.max(1.0 if comm is None else 0.0) > 0:
                if comm is not None:
                    comm.close()
                    comm = None
                exchange = "gloo host all-gather (RCCL communicator failed: %s)" % (err or "on another rank")
                log("warning: " + exchange)
                rccl = False
                # a real multi-GPU run must not report a host exchange as the
                # xGMI result: RF_BENCH_REQUIRE_RCCL=1 makes this fatal, and
                # the line always carries "rccl": false for the driver
                if os.environ.get("RF_BENCH_REQUIRE_RCCL") == "1":
                    raise SystemExit("RCCL communicator could not be created (RF_BENCH_REQUIRE_RCCL=1): %s" % err)
            else:
                exchange = "RCCL all-gather over xGMI"
                rccl = True

    sha = bench_sha(args, dist, ctx, budget)
    sha_ranks = None
    if dist.world > 1:  # per rank: host-leg threads and bytes, GPU-leg bytes, step ms (is the curve host-bound?)
        hl, comp = sha["host_leg"] or {}, sha["composition"]
        gpu_ms = max([v for k, v in sha["step_ms"].items() if k in ("solo", "lanes")] or [0.0])
        row = np.array([hl.get("threads", 0), comp["host_leg_bytes"], comp["gpu_bytes"], sha["ms_per_step"],
                        hl.get("ms", 0.0), gpu_ms], np.float64)
        # per rank: the host leg's and the GPU legs' own rates, so a 1 -> N SHA
        # curve shows which leg it measures (the host legs share the node's CPUs)
        sha_ranks = [dict(rank=i, host_threads=int(r[0]), host_leg_bytes=float(r[1]), gpu_bytes=float(r[2]),
                          ms_per_step=round(float(r[3]), 2),
                          host_leg_gbps=round(r[1] / (r[4] * 1e-3) / 1e9, 3) if r[4] else None,
                          gpu_legs_ms=round(float(r[5]), 2),
                          gpu_legs_gbps=round(r[2] / (r[5] * 1e-3) / 1e9, 3) if r[5] else None)
                     for i, r in enumerate(np.frombuffer(dist.all_gather_bytes(row), np.float64).reshape(-1, 6))]
    c1 = bench_c1(args, dist, ctx, budget) if "c1" not in args.skip and budget.allow("c1", 15, everyone=True) else None
    dag_res = dag100 = None
    if dist.world == 1 and "dag" not in args.skip and budget.allow("dag", 30):
        dag_res = bench_dag(args, dist, ctx, budget)
    if "dag100m" not in args.skip and budget.allow("dag100m", 150, everyone=True):
        dag100 = bench_dag100m(args, dist, ctx, comm, budget)
        duo_us = next((r.get("us_per_chain_block") for r in sha["roofline_gpu_legs"]
                       if r.get("kernel") == "k1_sha256_duo"), None)
        if dist.world == 1 and "piece" not in args.skip and budget.allow("piece_8", 20):
            pc8 = bench_piece(args, ctx, 8, dag100["ms_per_step"], duo_us)
            dag100["piece_8"] = pc8
            dag100["piece_ms_8"], dag100["projected_speedup_8"] = pc8["ms_per_step"], pc8["projected_speedup"]
        # SURVEY C3/C4 as written (per-sample roots) at every N; at N = 1 its 8-rank piece too
        if "persample" not in args.skip and budget.allow("persample", 60, everyone=True):
            dag100["per_sample_layout"] = bench_persample(args, dist, ctx, duo_us)
    probe = bench_probe(args, dist, ctx, budget) if "probe" not in args.skip and budget.allow("probe", 30, everyone=True) \
        else None
    cpu = None
    if dist.rank == 0 and dist.world == 1 and "cpu" not in args.skip and budget.allow("cpu", 60):
        cpu = cpu_baseline(args, sha, dag_res, budget)
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
    if dag_res is not None:
        dag_res.pop("_cpu", None)
    sha["_arena"].free()
    parity = parity_summary(sha, c1, dag_res, dag100, probe, cpu)
    valu_tops = valu_ceiling() if dist.rank == 0 else None

    if dist.rank == 0:
        workload = sha["workload"]
        if dist.world > 1:
            workload = ("configs[3] weak-scaled: the global Fileset = %d configs[1]-distributed sets (%d files, "
                        "%.0f GiB), LPT-sharded by size: %.1f GiB / %d files on rank 0"
                        % (dist.world, sha["glob"]["files"], sha["glob"]["bytes"] / GiB,
                           sha["bytes_per_gpu"] / GiB, sha["files"]))
        line = {
            "metric": "SHA-256 digest GB/s + incremental cache-key recompute Mnodes/s, 1/2/4/8 GPU",
            "value": round(sha["value"], 4), "unit": "GB/s", "n_gpus": dist.world,
            # the metric's other halves beside value: the
            # GPU-only SHA rate of the same set, and the DAG legs' dirty nodes/s
            "gpu_only_gbps": round(sha["gpu_only"]["gbps"], 4) if sha.get("gpu_only") else None,
            # the same set with every file on the host leg (measured), and
            # what the GPU legs add to one rank's rate over it
            "all_host_gbps": (sha["all_host"] or {}).get("gbps"),
            "gpu_marginal_gbps": (sha["all_host"] or {}).get("hybrid_minus_all_host_gbps"),
            "incremental_mnodes_per_s": round(dag_res["mnodes_per_s"], 1) if dag_res else None,
            "incremental_100m_mnodes_per_s": round(dag100["mnodes_per_s"], 1) if dag100 else None,
            "valu_measured_tops": round(valu_tops, 2) if valu_tops else None,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(sha["ms_per_step"], 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (splitmix64 content generated in HBM)",
            "config": {"workload": workload,
                       "parallelism": "files sharded per GPU (LPT by size); per GPU: host leg (SHA-NI threads) + "
                                      "GPU kernels split by the K1 planner; DAG partitioned by sample subtree, "
                                      "RCCL only for its boundary exchange",
                       "exchange": exchange, "split_rank0": sha["split"], "step_ms_rank0": sha["step_ms"]},
            "rccl": rccl,
            "parity": parity,
            "roofline": sha["roofline"],
            "roofline_gpu_legs": sha["roofline_gpu_legs"],
            "composition": sha["composition"],
            "host_leg": sha["host_leg"],
            "sha_per_rank": sha_ranks,
            "roofline_gpu_only": sha.get("roofline_gpu_only"),
            "gpu_only": sha.get("gpu_only"),
            "cpu_baseline": cpu,
            "c1": c1,
            "incremental": dag_res,
            "incremental_100m": dag100,
            "lowering": lowering,
            "probe": probe,
            "budget": {"seconds": args.budget_s, "skipped": budget.skipped,
                       "elapsed_s": round(time.perf_counter() - T_START, 1)},
        }
        with_measured_valu(line, valu_tops)
        line["summary"] = run_summary(line)  # last: the driver's record keeps the line's tail
        sys.stdout.flush()
        os.write(result_fd, (json.dumps(line) + "\n").encode())
    if comm is not None:
        comm.close()
    ctx.close()


def run_summary(line):
    """The DAG and probe results in a few numbers, written at the END of the
    line: the driver's record keeps only the line's tail."""
    def g(d, *ks):
        for k in ks:
            if not isinstance(d, dict):
                return None
            d = d.get(k)
        return d
    inc, big = line.get("incremental"), line.get("incremental_100m")
    ps = g(big, "per_sample_layout")
    out = {
        "sha_gbps": line.get("value"), "sha_all_host_gbps": line.get("all_host_gbps"),
        "sha_gpu_only_gbps": line.get("gpu_only_gbps"), "sha_gpu_marginal_gbps": line.get("gpu_marginal_gbps"),
        "configs2_ms_per_step": g(inc, "ms_per_step"), "configs2_device_ms_per_step": g(inc, "device_ms_per_step"),
        "configs2_mnodes_per_s": g(inc, "mnodes_per_s"),
        "configs2_latency_frac_of_issue_floor": g(inc, "roofline_latency", "frac_of_issue_floor"),
        "dag100m_ms_per_step": g(big, "ms_per_step"), "dag100m_mnodes_per_s": g(big, "mnodes_per_s"),
        "dag100m_frac_of_measured_valu": g(big, "roofline_incremental", "frac_of_measured_valu"),
        "dag100m_dirty_blocks_per_step": g(big, "dirty_blocks_per_step"),
        "merge_tree_piece8_ms": g(big, "piece_8", "ms_per_step"),
        "merge_tree_projected_speedup_8": g(big, "piece_8", "projected_speedup"),
        "per_sample_ms_per_step": g(ps, "ms_per_step"), "per_sample_mnodes_per_s": g(ps, "mnodes_per_s"),
        "per_sample_piece8_ms": g(ps, "piece_8", "ms_per_step"),
        "per_sample_projected_speedup_8": g(ps, "piece_8", "projected_speedup"),
        "probe_gprobes_per_s": g(line.get("probe"), "gprobes_per_s"),
        "n_gpus": line.get("n_gpus"), "parity_all": g(line.get("parity"), "all"),
    }
    return {k: v for k, v in out.items() if v is not None}


if __name__ == "__main__":
    main()
