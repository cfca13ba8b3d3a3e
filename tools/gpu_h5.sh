#!/bin/bash
# session: DAG GPU tests on the in-tree library, then dag_ab.sh over builds
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_dag_fusion.py tests/test_gpu_dag_midstate.py \
    tests/test_gpu_dag_update.py tests/test_gpu_partition.py tests/test_golden_fixtures.py tests/test_gpu_scale.py \
    -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 bash tools/dag_ab.sh "$@" 2>&1 | tee $O/ab.txt
