#!/bin/bash
# The GPU suite, smoke() and (optionally) the driver's bench command, every
# GPU step under its own time limit, chained with && (a failure ends it).
#   bash tools/gpu_suite.sh <tag> [bench]
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
step tests && timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 && tail -2 $out/gpu_tests.log &&
step smoke && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 && tail -1 $out/smoke.log &&
if [ "$2" = bench ]; then
    step bench && RF_LOWER_TIMING=1 timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.log && tail -8 $out/bench.log
fi
rc=$?
echo "rc=$rc"
exit $rc
