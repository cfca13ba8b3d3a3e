"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel.

    python tools/pmc_summary.py FETCH_DIR/x_counter_collection.csv WRITE_DIR/x_counter_collection.csv OUT.json [BENCH.json]

BENCH.json (the profiled bench's stdout line) supplies the "workload" key
bench.py matches before it uses these figures as its roofline `traffic`.

FETCH_SIZE and WRITE_SIZE are reported by rocprofv3 in KiB.  Per
MI355X_MICROARCH.md (HBM / rocprofv3): on gfx950 FETCH_SIZE reads exactly
half of the bytes of a wide coalesced streaming read (128-B requests tallied
at 64 B), so `fetch_bytes_corrected` = 2 x FETCH_SIZE x 1024 for kernels whose
reads are wide coalesced streams (K1: 64 B per lane, 4 KiB per wave); for
random 8-B gathers (K4) the raw figure is reported (uncalibrated access width:
the guide gives no correction), and Infinity-Cache hits are counted too."""
import collections
import csv
import json
import sys

WIDE_STREAM = {"rf::k1_sha256_duo", "rf::k1_sha256_octo", "rf::k1_sha256_solo", "rf::k1_sha256_lanes",
               "rf::k1_sha256_pair", "rf::k_gen_fill"}


def load(path):
    """kernel -> [dispatches, total KiB, largest dispatch's KiB, [KiB per dispatch in order]]"""
    per = collections.OrderedDict()
    for i, r in enumerate(csv.DictReader(open(path))):
        k = r["Kernel_Name"].split("(")[0]
        k = k[5:] if k.startswith("void ") else k
        k = k.split("<")[0]  # one entry per kernel template
        key = (k, int(r.get("Dispatch_Id", i)))
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, []])
    for (k, _), v in sorted(per.items(), key=lambda kv: kv[0][1]):
        agg[k][0] += 1
        agg[k][1] += v
        agg[k][2] = max(agg[k][2], v)
        agg[k][3].append(v)
    return agg


def main():
    f, w, out = sys.argv[1:4]
    F, W = load(f), load(w)
    res = {}
    if len(sys.argv) > 4:
        for line in open(sys.argv[4]):
            if line.startswith("{"):
                res["workload"] = json.loads(line)["config"]["workload"]
    for k in sorted(set(F) | set(W)):
        nf, vf, mf, lf = F.get(k, [0, 0.0, 0.0, []])
        nw, vw, mw, lw = W.get(k, [0, 0.0, 0.0, []])
        fb = vf / max(nf, 1) * 1024
        wb = vw / max(nw, 1) * 1024
        corr = 2.0 if k in WIDE_STREAM else 1.0
        # the mean mixes a kernel's big launches with its small ones (e.g. the
        # duo chain runs the 64 GiB set and configs[0]'s Fileset material):
        # the largest dispatch is the one a bench roofline prices
        res[k] = {"calls": nf, "fetch_bytes_raw": fb, "fetch_bytes_corrected": fb * corr,
                  "fetch_correction": corr, "write_bytes": wb,
                  "traffic_bytes_per_launch": fb * corr + wb,
                  "traffic_bytes_largest_launch": (mf * corr + mw) * 1024,
                  # every launch in dispatch order (the fetch and write passes
                  # run the same command, so their launches pair up in order)
                  "launch_traffic_bytes": [(a * corr + b) * 1024 for a, b in zip(lf, lw)] if len(lf) == len(lw) else []}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        if k == "workload":
            print("workload:", v)
            continue
        print("%-36s traffic/launch %.4e B, largest launch %.4e B (fetch raw %.4e x%.0f, write %.4e)"
              % (k, v["traffic_bytes_per_launch"], v["traffic_bytes_largest_launch"], v["fetch_bytes_raw"],
                 v["fetch_correction"], v["write_bytes"]))


if __name__ == "__main__":
    main()
