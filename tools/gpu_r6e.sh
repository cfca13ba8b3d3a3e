#!/bin/bash
# Round 6: kernel trace of the latency-bound DAG steps (configs[2] and the
# per-sample layout's 8-rank piece), per-dispatch summary.
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
step trace && timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o t -- python3 tools/dag_forms.py --c2 --persample 8 --steps 10 > $out/forms.json 2> $out/forms.log &&
grep "ms/step" $out/forms.log | head -20
rc=$?
echo "rc=$rc"
exit $rc
