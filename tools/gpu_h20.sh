#!/bin/bash
# parity cursors (no step-end kernel): DAG / partition / update tests, step A/B, full-recompute graph A/B
set -o pipefail
O=gpurun_out/h20
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_dag_fusion.py tests/test_gpu_dag_midstate.py \
    tests/test_gpu_dag_update.py tests/test_gpu_partition.py tests/test_golden_fixtures.py tests/test_gpu_scale.py \
    tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab.sh $O/ab - RF_K2_GRAPH=1 || exit 1
bash tools/gpu_h19.sh
