#!/bin/bash
# One GPU-box session: the GPU test suite, smoke(), then the driver's bench
# command; every GPU step under its own time limit, chained so a failure
# ends the session.   usage: tools/gpu_session.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
echo "== focus: ${FOCUS:-none}" && \
{ [ -z "$FOCUS" ] || timeout -k 10 300 python -u -m pytest $FOCUS -x -v --timeout 120 --timeout-method thread > $out/focus.log 2>&1; } && \
echo "== tests" && \
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 && \
tail -3 $out/gpu_tests.log && \
echo "== smoke" && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 && \
tail -2 $out/smoke.log && \
echo "== bench" && \
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 "$@" > $out/bench.json 2> $out/bench.log
rc=$?
tail -3 $out/focus.log 2>/dev/null
tail -3 $out/gpu_tests.log 2>/dev/null
tail -25 $out/bench.log 2>/dev/null
exit $rc
