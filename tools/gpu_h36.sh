#!/bin/bash
# mark chain: first job's operands pinned before the loop (P) vs M; then the step's kernel trace on P
set -o pipefail
O=gpurun_out/h36
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_dag_fusion.py tests/test_gpu_dag_midstate.py tests/test_gpu_dag_update.py tests/test_gpu_partition.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/dag_ab.sh tools/_var/P.so tools/_var/M.so tools/_var/P.so tools/_var/M.so tools/_var/P.so tools/_var/M.so
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $O/dtr -o d -- python tools/dag_probe.py --dag-steps 20 > $O/probe.json 2> $O/probe.log || { tail -5 $O/probe.log; exit 1; }
python3 tools/trace_step.py $(find $O/dtr -name 'd_kernel_trace.csv' | head -1) > $O/dag_step.txt 2>&1; cat $O/dag_step.txt
