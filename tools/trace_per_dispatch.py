"""Per-dispatch kernel durations (µs) from rocprofv3 --kernel-trace CSVs, one
row per kernel name in launch order -- side by side for A/B traces.

    python tools/trace_per_dispatch.py DIR_A/t_kernel_trace.csv [DIR_B/t_kernel_trace.csv ...]
"""
import collections
import csv
import statistics
import sys

SKIP = ("rocclr", "midstates", "k_gather")


def per_kernel(path):
    d = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if any(s in n for s in SKIP):
            continue
        d.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    return d


def main():
    for path in sys.argv[1:]:
        print(path)
        for n, v in per_kernel(path).items():
            tail = v[1:] if len(v) > 2 else v  # (the first dispatch: cold, or the load's full pass)
            print("  %-36s n %3d  median %8.1f  min %8.1f   %s" % (
                n[:36], len(v), statistics.median(tail), min(tail), " ".join("%.1f" % x for x in v[:14])))


if __name__ == "__main__":
    main()
