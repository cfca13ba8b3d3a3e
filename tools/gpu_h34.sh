#!/bin/bash
# mark kernel: next job's operands pinned before the digest store (M) vs the committed build (A)
set -o pipefail
O=gpurun_out/h34
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_dag_fusion.py tests/test_gpu_dag_midstate.py tests/test_gpu_dag_update.py tests/test_gpu_partition.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/dag_ab.sh tools/_var/M.so tools/_var/A.so tools/_var/M.so tools/_var/A.so tools/_var/M.so tools/_var/A.so
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/tr -o t -- python tools/dag_probe.py --dag-steps 20 > $O/probe.json 2> $O/probe.log || { tail -5 $O/probe.log; exit 1; }
python tools/dag_step_trace.py $O/tr 2>/dev/null | tail -6 || true
