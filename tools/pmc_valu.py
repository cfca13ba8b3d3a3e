"""Per-kernel summary of a rocprofv3 --pmc counter_collection.csv with the
VALU / wait counters SURVEY §8(d) names (SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU,
SQ_WAIT_INST_ANY, SQ_WAIT_ANY, SQ_ACTIVE_INST_ANY, SQ_WAVE_CYCLES,
GRBM_GUI_ACTIVE): mean per dispatch, and the shares of wave cycles that
issue VALU, are issue-stalled, or wait (s_waitcnt / barrier).  SQ cycle
counters count quad-cycles (MI355X_MICROARCH.md, "s_memtime tick vs SQ PMC
units"); the shares are ratios of the same unit.

    python tools/pmc_valu.py counter_collection.csv [kernel-substring ...]
"""
import collections
import csv
import sys


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for row in csv.DictReader(open(path)):
        name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
        if pats and not any(p in name for p in pats):
            continue
        cnt = row.get("Counter_Name") or row.get("Counter-Name")
        val = float(row.get("Counter_Value") or row.get("Counter-Value") or 0)
        disp = row.get("Dispatch_Id") or row.get("Dispatch-Id") or row.get("Correlation_Id")
        per[name.split("(")[0][:80]][cnt].append((disp, val))
    for name, cs in sorted(per.items()):
        mean = {c: sum(v for _, v in xs) / max(len(xs), 1) for c, xs in cs.items()}
        n = max(len(xs) for xs in cs.values())
        print("%s  (%d dispatches)" % (name, n))
        for c in sorted(mean):
            print("    %-22s %16.1f" % (c, mean[c]))
        wc = mean.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
                if c in mean:
                    print("    %-22s %16.3f of wave cycles" % (c, mean[c] / wc))
        if mean.get("SQ_INSTS_VALU") and mean.get("SQ_ACTIVE_INST_VALU"):
            print("    %-22s %16.2f quad-cycles per VALU instruction" % (
                "active/insts", mean["SQ_ACTIVE_INST_VALU"] / mean["SQ_INSTS_VALU"]))


if __name__ == "__main__":
    main()
