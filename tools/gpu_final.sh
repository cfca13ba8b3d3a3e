#!/bin/bash
# Round-end GPU sessions on one box, every GPU step under its own time limit
# and chained with && (a failure ends the session):
#   bash tools/gpu_final.sh <tag> A    the GPU suite, smoke(), the driver's bench command
#   bash tools/gpu_final.sh <tag> C    the same bench command under rocprofv3 --kernel-trace --stats,
#                                      then the 100M DAG's forms (default / octo off / round-3 sinks)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
if [ "$2" = A ]; then
    step tests && timeout -k 10 800 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 && tail -2 $out/gpu_tests.log &&
    step smoke && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 && tail -1 $out/smoke.log &&
    step bench && RF_LOWER_TIMING=1 timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.log &&
    tail -6 $out/bench.log
else
    step trace && timeout -k 10 800 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/trace_bench.json 2> $out/trace_bench.log &&
    step forms100m && timeout -k 10 300 python -u tools/dag_forms.py --c4-ranks 1 --steps 10 > $out/f100m_new.json 2> $out/f100m_new.log &&
    RF_K2_OCT=0 timeout -k 10 300 python -u tools/dag_forms.py --c4-ranks 1 --steps 10 > $out/f100m_nooct.json 2> $out/f100m_nooct.log &&
    grep auto $out/f100m_*.log
fi
rc=$?
echo "rc=$rc"
exit $rc
