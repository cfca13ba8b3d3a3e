"""Per-dispatch L2 hit rate and fabric fetch of the bloomlive probe kernels
from rocprofv3 --pmc passes (tools/profile_r02.sh): TCC_HIT_sum /
(TCC_HIT_sum + TCC_MISS_sum) per dispatch, FETCH_SIZE (KiB, raw: random 8-B
gathers are an uncalibrated access width per MI355X_MICROARCH.md) per
dispatch, grouped by grid size in launch order -- bench.py probes the 171 MiB
filter first, then the 2 GiB one.

    python tools/pmc_probe.py TCC.csv FETCH.csv"""
import collections
import csv
import sys


def per_dispatch(path, counters):
    rows = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
        if "bloom" not in k and "k4" not in k:
            continue
        key = (r.get("Dispatch_Id"), k)
        d = rows.setdefault(key, {"kernel": k, "grid": r.get("Grid_Size", r.get("Grid_Size_X", "?"))})
        if r["Counter_Name"] in counters:
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(rows.values())


def main(tcc, fetch):
    print("L2 (TCC) hit rate per probe-kernel dispatch (launch order):")
    for d in per_dispatch(tcc, ("TCC_HIT_sum", "TCC_MISS_sum")):
        h, m = d.get("TCC_HIT_sum", 0.0), d.get("TCC_MISS_sum", 0.0)
        print("  %-34s grid %-10s hit %.3e miss %.3e  hit rate %.3f" % (d["kernel"], d["grid"], h, m,
                                                                          h / max(h + m, 1.0)))
    print("FETCH_SIZE per probe-kernel dispatch (raw KiB -> bytes):")
    for d in per_dispatch(fetch, ("FETCH_SIZE",)):
        print("  %-34s grid %-10s %.4e B" % (d["kernel"], d["grid"], d.get("FETCH_SIZE", 0.0) * 1024))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
