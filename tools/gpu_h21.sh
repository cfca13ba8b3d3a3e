#!/bin/bash
set -o pipefail
O=gpurun_out/h21
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/dtr -o d -- python3 tools/dag_probe.py --dag-steps 20 > $O/dag_probe.json 2> $O/dag_probe.log || { echo trace failed; tail -5 $O/dag_probe.log; exit 1; }
python3 tools/trace_step.py $(find $O/dtr -name 'd_kernel_trace.csv' | head -1) > $O/dag_step.txt 2>&1; cat $O/dag_step.txt
