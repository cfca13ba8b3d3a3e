#!/bin/bash
# session h1: assoc tests, the driver's bench command (timed), the configs[2]
# step's kernel trace, and the 2-rank-on-one-GPU RCCL probe
set -o pipefail
O=gpurun_out/h1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_assoc.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
s=$(date +%s.%N)
timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || { echo bench failed; tail -5 $O/bench.log; exit 1; }
echo "bench wall $(python -c "print(round($(date +%s.%N) - $s, 1))") s"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/dtr -o d -- python3 tools/dag_probe.py --dag-steps 20 > $O/dag_probe.json 2> $O/dag_probe.log || { echo trace failed; tail -5 $O/dag_probe.log; exit 1; }
python3 tools/trace_step.py $(ls $O/dtr/*/d_kernel_trace.csv $O/dtr/d_kernel_trace.csv 2>/dev/null | head -1) > $O/dag_step.txt 2>&1; cat $O/dag_step.txt
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tools/rccl_pair_probe.py > $O/rccl_pair.json 2> $O/rccl_pair.log
echo "rccl probe rc=$?"; cat $O/rccl_pair.json; tail -3 $O/rccl_pair.log
