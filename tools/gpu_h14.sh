#!/bin/bash
# chain-built block 0 (cb0): DAG GPU tests, then A/B against RF_K2_CB0=0
set -o pipefail
O=gpurun_out/h14
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_dag_fusion.py tests/test_gpu_dag_midstate.py \
    tests/test_gpu_dag_update.py tests/test_gpu_partition.py tests/test_golden_fixtures.py tests/test_gpu_scale.py \
    tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab.sh $O/ab - RF_K2_CB0=0
