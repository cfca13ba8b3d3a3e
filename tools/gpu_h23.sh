#!/bin/bash
# streamed hand-over with the chain-built chunk 0: DAG tests in both hand-over modes, then A/B
set -o pipefail
O=gpurun_out/h23
mkdir -p $O
export TMPDIR=/tmp
T="tests/test_gpu_dag.py tests/test_gpu_dag_fusion.py tests/test_gpu_dag_midstate.py tests/test_gpu_dag_update.py tests/test_gpu_partition.py tests/test_gpu_scale.py"
RF_K2_STREAM=1 timeout -k 10 400 python -u -m pytest $T -x -v --timeout 200 --timeout-method thread > $O/tests_stream.log 2>&1 || { tail -40 $O/tests_stream.log; exit 1; }
tail -1 $O/tests_stream.log
bash tools/gpu_ab.sh $O/ab - RF_K2_STREAM=1
