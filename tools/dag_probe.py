"""Runs bench.py's configs[2] incremental-DAG leg alone (for profiling:
rocprofv3 --kernel-trace -- python tools/dag_probe.py) and prints its line."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from reflow_amd import capi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dag-samples", type=int, default=22075)
    ap.add_argument("--dag-pairs", type=int, default=32)
    ap.add_argument("--dag-steps", type=int, default=20)
    a = ap.parse_args()
    import faulthandler
    faulthandler.dump_traceback_later(80, exit=True)  # a stuck run names its line
    dist = bench.Dist(1)
    ctx = capi.Context(0, host_threads=0)
    a.skip = {"checkpoint"}
    r = bench.bench_dag(a, dist, ctx, bench.Budget(600))
    r.pop("_cpu", None)
    print(json.dumps(r), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
