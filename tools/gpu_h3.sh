#!/bin/bash
# session h3: DAG / partition / assoc GPU tests, slot-fusion A/B on configs[2]
# (RF_K2_SLOT_FUSE=0 vs default), the step's trace, the assoc Put timing
set -o pipefail
O=gpurun_out/h3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_dag_fusion.py tests/test_gpu_dag_midstate.py \
    tests/test_gpu_dag_update.py tests/test_gpu_partition.py tests/test_gpu_parity.py tests/test_golden_fixtures.py \
    tests/test_gpu_scale.py tests/test_gpu_assoc.py tests/test_gpu_coalesce.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for v in 0 1; do
    RF_K2_SLOT_FUSE=$v timeout -k 10 150 python tools/dag_probe.py --dag-steps 50 > $O/ab_${v}_${r}.json 2>$O/ab.log || { echo probe failed; tail -5 $O/ab.log; exit 1; }
    echo "slot_fuse=$v run $r: $(python -c "import json; d=json.load(open('$O/ab_${v}_${r}.json')); print(round(d['ms_per_step'],4), round(d['device_ms_per_step'],4), d['dirty_jobs_per_step'])")"
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/dtr -o d -- python3 tools/dag_probe.py --dag-steps 20 > $O/dag_probe.json 2> $O/dag_probe.log || { echo trace failed; tail -5 $O/dag_probe.log; exit 1; }
python3 tools/trace_step.py $(find $O/dtr -name 'd_kernel_trace.csv' | head -1) > $O/dag_step.txt 2>&1; cat $O/dag_step.txt
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --sha-gib 0.25 --gpu-only-run 0 --probe-steps 1 --skip cpu,c1,install,dag > $O/probe.json 2> $O/probe.log || { echo probe bench failed; tail -5 $O/probe.log; exit 1; }
python -c "import json; d=json.load(open('$O/probe.json'))['probe']['assoc']; print('assoc put_ms', d['put_ms'], 'get_ms', d['get_ms'], d['put_ok'], d['found_exact'])"
