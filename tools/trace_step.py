"""Prints the kernels of incremental DAG steps from a rocprofv3
--kernel-trace CSV (tools/dag_probe.py or tools/dag_forms.py under rocprofv3):
name, grid, duration and the gap to the previous kernel.  A step starts at a
k3_mark_slots dispatch.

  python tools/trace_step.py trace.csv [K ...]

K: steps counted back from the last complete one (default 1: the last)."""
import csv
import sys


def main(path, back):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "k3_mark_slots" in r["Kernel_Name"]]
    for k in back:
        i0, i1 = marks[-1 - k], marks[-k]
        prev = None
        print("-- step %d back" % k)
        for r in rows[i0:i1]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            name = r["Kernel_Name"].split("(")[0].replace("rf::", "")
            print("%-32s grid=%8s dur=%8.2f us gap=%6.2f us" % (name, r["Grid_Size_X"], (e - s) / 1e3,
                                                                (s - prev) / 1e3 if prev else 0.0))
            prev = e
        print("step span %.1f us" % ((int(rows[i1]["Start_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) / 1e3))


if __name__ == "__main__":
    main(sys.argv[1], [int(x) for x in sys.argv[2:]] or [1])
