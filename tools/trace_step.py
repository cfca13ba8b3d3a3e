"""Prints the kernels of the last incremental DAG step from a rocprofv3
--kernel-trace CSV (tools/dag_probe.py under rocprofv3): name, grid,
duration and the gap to the previous kernel."""
import csv
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "k3_mark_slots" in r["Kernel_Name"]]
    i0, i1 = marks[-2], marks[-1]
    prev = None
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("rf::", "")
        print("%-32s grid=%8s dur=%8.2f us gap=%6.2f us" % (name, r["Grid_Size_X"], (e - s) / 1e3,
                                                            (s - prev) / 1e3 if prev else 0.0))
        prev = e
    print("step span %.1f us" % ((int(rows[i1]["Start_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) / 1e3))


if __name__ == "__main__":
    main(sys.argv[1])
