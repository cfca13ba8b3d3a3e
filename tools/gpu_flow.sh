#!/bin/bash
# Round 5: the flow step on the GPU -- its tests, the DAG tests around it,
# then the forms A/B (flow on / off) on configs[2], the 8-rank piece and 100M.
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
step flow_tests && timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_checkpoint.py -x -v --timeout 200 --timeout-method thread > $out/flow_tests.log 2>&1 && tail -3 $out/flow_tests.log &&
step dag_tests && timeout -k 10 600 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_dag_default_forms.py tests/test_gpu_dag_modes.py tests/test_gpu_dag_fusion.py -x -q --timeout 200 --timeout-method thread > $out/dag_tests.log 2>&1 && tail -3 $out/dag_tests.log &&
step forms && timeout -k 10 600 python -u tools/dag_forms.py --c2 --c4-ranks 8,1 --steps 20 > $out/forms.json 2> $out/forms.log && grep -E "auto|flow" $out/forms.log
rc=$?
echo "rc=$rc"
exit $rc
