#!/bin/bash
# one chain block-step call site + pass-0 instruction-cache warm-up: DAG tests, stamps, A/B vs no warm-up
set -o pipefail
O=gpurun_out/h31
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_dag_fusion.py tests/test_gpu_dag_midstate.py tests/test_gpu_dag_update.py tests/test_gpu_partition.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
RF_K2_STAMPS=1 timeout -k 10 150 python tools/dag_probe.py --dag-steps 3 > $O/probe.json 2> $O/stamps.log || { tail -5 $O/stamps.log; exit 1; }
grep stamps $O/stamps.log | head -4
bash tools/gpu_ab.sh $O "-" "RF_K2_DBG_NOEXP=5"
