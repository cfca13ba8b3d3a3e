"""K4 probe traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE)
over bench.py's probe leg (tools/gpu_r5b.sh k4): per probe-kernel dispatch
group (grid size: the 171 MiB filter first, then the 2 GiB one), the mean
FETCH and WRITE bytes per dispatch and per probe, against the algorithmic
32 + 8k + 1 B a probe (the key, k filter words, the answer byte).  FETCH_SIZE
is raw KiB (the probe is random 8-B gathers plus one 32-B key stream per
lane; the guide's 2x correction is for wide streams only, so raw is an upper
bound on the gathers' share).

    python tools/pmc_k4_summary.py FETCH.csv WRITE.csv N_PROBE K [out.json]
"""
import collections
import csv
import json
import sys


def groups(path, counter):
    per = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name", "")
        if "k4_bloom_probe" not in name or r.get("Counter_Name") != counter:
            continue
        key = (r.get("Dispatch_Id"), r.get("Grid_Size", r.get("Grid_Size_X", "?")))
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    g = collections.OrderedDict()
    for (disp, grid), v in per.items():
        g.setdefault(grid, []).append(v * 1024.0)  # KiB -> B
    return g


def main():
    fetch, write, n_probe, k = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    bpp = 32 + 8 * k + 1
    fg, wg = groups(fetch, "FETCH_SIZE"), groups(write, "WRITE_SIZE")
    out = []
    for grid, fs in fg.items():
        ws = wg.get(grid, [0.0])
        f, w = sum(fs) / len(fs), sum(ws) / len(ws)
        row = {"grid": grid, "dispatches": len(fs), "fetch_bytes": f, "write_bytes": w,
               "fetch_per_probe": f / n_probe, "write_per_probe": w / n_probe,
               "algorithmic_per_probe": bpp, "traffic_over_algorithmic": (f + w) / n_probe / bpp}
        out.append(row)
        print("k4_bloom_probe grid %s: %d dispatches, FETCH %.3e B (%.1f B/probe), WRITE %.3e B (%.2f B/probe); "
              "algorithmic %d B/probe -> traffic %.2fx" % (grid, len(fs), f, f / n_probe, w, w / n_probe, bpp,
                                                          (f + w) / n_probe / bpp))
    if len(sys.argv) > 5:
        json.dump(out, open(sys.argv[5], "w"), indent=1)


if __name__ == "__main__":
    main()
