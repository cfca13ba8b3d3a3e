"""Runs bench.py's configs[4] probe leg alone and prints its result line
(used to choose K4's fetch schedule, k4_bloom.hip launch_bloom_probe)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from reflow_amd import capi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--probe-keys", type=int, default=100_000_000)
    ap.add_argument("--probes", type=int, default=1_000_000_000)
    ap.add_argument("--probe-steps", type=int, default=3)
    a = ap.parse_args()
    dist = bench.Dist(1)
    ctx = capi.Context(0)
    r = bench.bench_probe(a, dist, ctx)
    print(json.dumps(r), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
