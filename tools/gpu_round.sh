#!/bin/bash
# One GPU-box session: the given pytest selection, then a short bench.
# usage: tools/gpu_round.sh <tag> <pytest args...>
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/$tag/tests.log 2>&1
rc=$?
tail -5 gpurun_out/$tag/tests.log
exit $rc
