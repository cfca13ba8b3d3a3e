#!/bin/bash
# mark: the slot's other consumer's record loads + dirty atomic issued before the chain (X) vs HEAD (H)
set -o pipefail
O=gpurun_out/h40
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_dag_fusion.py tests/test_gpu_dag_midstate.py tests/test_gpu_dag_update.py tests/test_gpu_partition.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/dag_ab.sh tools/_var/X.so tools/_var/H.so tools/_var/X.so tools/_var/H.so tools/_var/X.so tools/_var/H.so
