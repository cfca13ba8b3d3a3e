#!/bin/bash
# session h2: DAG / partition GPU tests, then an A/B of slot fusion on the
# configs[2] step (RF_K2_SLOT_FUSE=0 vs default) and the step's kernel trace
set -o pipefail
O=gpurun_out/h2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_dag_fusion.py tests/test_gpu_dag_midstate.py \
    tests/test_gpu_dag_update.py tests/test_gpu_partition.py tests/test_gpu_parity.py tests/test_golden_fixtures.py \
    tests/test_gpu_scale.py tests/test_gpu_assoc.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for v in 0 1; do
    RF_K2_SLOT_FUSE=$v timeout -k 10 150 python tools/dag_probe.py --dag-steps 50 > $O/ab_$v_$r.json 2>$O/ab.log || { echo probe failed; tail -5 $O/ab.log; exit 1; }
    echo "slot_fuse=$v run $r: $(python -c "import json; d=json.load(open('$O/ab_$v_$r.json')); print(round(d['ms_per_step'],4), round(d['device_ms_per_step'],4), d['dirty_jobs_per_step'])")"
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/dtr -o d -- python3 tools/dag_probe.py --dag-steps 20 > $O/dag_probe.json 2> $O/dag_probe.log || { echo trace failed; tail -5 $O/dag_probe.log; exit 1; }
python3 tools/trace_step.py $(find $O/dtr -name 'd_kernel_trace.csv' | head -1) > $O/dag_step.txt 2>&1; cat $O/dag_step.txt
