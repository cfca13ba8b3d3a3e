#!/bin/bash
set -o pipefail
O=gpurun_out/h25
mkdir -p $O
export TMPDIR=/tmp
T="tests/test_gpu_dag.py tests/test_gpu_dag_fusion.py tests/test_gpu_dag_midstate.py tests/test_gpu_dag_update.py tests/test_gpu_partition.py tests/test_gpu_scale.py tests/test_golden_fixtures.py"
timeout -k 10 400 python -u -m pytest $T -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh $O/ab - RF_K2_SF=0 && bash tools/gpu_h24.sh
