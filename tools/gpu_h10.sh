#!/bin/bash
# partition GPU tests (both exchange protocols) + a 2-rank shared-GPU rehearsal of bench's N-rank path
set -o pipefail
O=gpurun_out/h10
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_partition.py tests/test_gpu_dag.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
RF_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 \
    bench.py --gpus 2 --steps 5 --warmup 2 --sha-gib 4 --c4-samples 4000 --skip cpu,c1,install,probe > $O/bench2.json 2> $O/bench2.log || { echo bench2 failed; tail -20 $O/bench2.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench2.json')); i=d['incremental']; print(d['value'], d['config']['exchange']); print(i['workload']); print(i['ms_per_step'], i['device_ms_per_step'], i['mnodes_per_s'])"
