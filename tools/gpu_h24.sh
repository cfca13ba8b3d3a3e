#!/bin/bash
# 2-rank rehearsal on one GPU with the RCCL communicator attempted (refused: two ranks on one GPU) -> gloo fallback
set -o pipefail
O=gpurun_out/h24
mkdir -p $O
export TMPDIR=/tmp
RF_BENCH_SHARE_GPU=1 RF_BENCH_TRY_RCCL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 2 --steps 5 --warmup 2 --sha-gib 2 --c4-samples 2000 \
    --skip cpu,c1,install,probe > $O/bench2.json 2> $O/bench2.log || { echo bench2 failed; tail -20 $O/bench2.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench2.json')); i=d['incremental']; print(d['value'], d['config']['exchange']); print(i['ms_per_step'], i['mnodes_per_s'])"
