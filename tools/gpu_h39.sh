#!/bin/bash
# kW=3 frontier atomics on the producer: DAG tests, A/B vs on the chain (RF_K2_DBG_NOEXP=6)
set -o pipefail
O=gpurun_out/h39
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_dag_fusion.py tests/test_gpu_dag_midstate.py tests/test_gpu_dag_update.py tests/test_gpu_partition.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
RF_K2_WIDE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_dag_fusion.py tests/test_gpu_dag_midstate.py tests/test_gpu_partition.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_wide.log 2>&1 || { tail -30 $O/tests_wide.log; exit 1; }
tail -1 $O/tests_wide.log
bash tools/gpu_ab.sh $O "-" "RF_K2_DBG_NOEXP=6"
