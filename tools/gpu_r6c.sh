#!/bin/bash
# Round 6: the memo parity test first, then the whole GPU suite, then the
# driver's bench command -- every GPU step under its own limit, chained.
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
step memo && timeout -k 10 300 python -u -m pytest tests/test_gpu_dag_memo.py -x -v --timeout 200 --timeout-method thread > $out/memo.log 2>&1 && tail -3 $out/memo.log &&
step tests && timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 && tail -2 $out/gpu_tests.log &&
if [ "$2" = bench ]; then
    step bench && timeout -k 10 800 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.log && tail -6 $out/bench.log
fi
rc=$?
echo "rc=$rc"
exit $rc
