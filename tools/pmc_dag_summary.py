"""K2/K3 HBM traffic per incremental step from two rocprofv3 passes of
tools/pmc_dag.py (FETCH_SIZE, WRITE_SIZE), against its algorithmic bytes.

    python tools/pmc_dag_summary.py FETCH.csv WRITE.csv PMC_DAG_STDOUT OUT.json

The incremental steps are the dispatches after the full recompute's
k3_step_end (the initial set_slots and the full recompute come before it);
k_gather_slots (slot read-backs) is left out.  FETCH_SIZE / WRITE_SIZE are in
KiB; K2's reads are scattered 16-64 B records and digests plus template
blocks, not wide streams, so the raw figure is reported (MI355X_MICROARCH.md
"HBM": the 2x correction applies to wide coalesced streams only) -- it counts
Infinity-Cache hits too, so it bounds the HBM bytes from above."""
import collections
import csv
import json
import sys

STEP_KERNELS = ("k3_mark_slots", "k3_mark_slots_lf", "k2_level_pl", "k2_level_lf", "k2_level_oct", "k2_level_pc")


def dispatches(path):
    """[(dispatch id, kernel, KiB)] in dispatch order"""
    per = collections.OrderedDict()
    for i, r in enumerate(csv.DictReader(open(path))):
        k = r["Kernel_Name"].split("(")[0]
        k = k[5:] if k.startswith("void ") else k
        k = k.split("<")[0].replace("rf::", "")
        key = int(r.get("Dispatch_Id", i))
        kk, v = per.get(key, (k, 0.0))
        per[key] = (k, v + float(r["Counter_Value"]))
    return [(d, k, v) for d, (k, v) in sorted(per.items())]


def step_part(ds):
    last_end = max((i for i, (_, k, _) in enumerate(ds) if k == "k3_step_end"), default=-1)
    return [(d, k, v) for d, k, v in ds[last_end + 1:] if k in STEP_KERNELS]


def main():
    f, w, info, out = sys.argv[1:5]
    meta = next(json.loads(ln) for ln in open(info) if ln.startswith("{"))
    F, W = step_part(dispatches(f)), step_part(dispatches(w))
    steps = meta["steps"]
    per_kernel = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for _, k, v in F:
        per_kernel[k][0] += 1
        per_kernel[k][1] += v * 1024
    for _, k, v in W:
        per_kernel[k][2] += v * 1024
    fetch = sum(v for _, _, v in F) * 1024 / steps
    write = sum(v for _, _, v in W) * 1024 / steps
    alg = meta["algorithmic_bytes_per_step"]
    res = {"graph": meta["graph"], "steps": steps,
           "fetch_bytes_per_step": fetch, "write_bytes_per_step": write,
           "traffic_bytes_per_step": fetch + write,
           "algorithmic_bytes_per_step": alg, "dirty_blocks_per_step": meta["dirty_blocks_per_step"],
           "jobs_per_step": meta["jobs_per_step"],
           "traffic_over_algorithmic": round((fetch + write) / alg, 3) if alg else None,
           "traffic_bytes_per_dirty_block": round((fetch + write) / max(meta["dirty_blocks_per_step"], 1), 1),
           "algorithmic_bytes_per_dirty_block": round(alg / max(meta["dirty_blocks_per_step"], 1), 1),
           "per_kernel": {k: {"dispatches_per_step": v[0] / steps, "fetch_bytes_per_step": v[1] / steps,
                              "write_bytes_per_step": v[2] / steps} for k, v in sorted(per_kernel.items())},
           "note": "raw FETCH_SIZE (KiB x 1024): K2's accesses are scattered records/digests and template blocks, "
                   "not the wide streams the guide's 2x correction is for; Infinity-Cache hits are included"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
