#!/bin/bash
set -o pipefail
O=gpurun_out/h26
mkdir -p $O
export TMPDIR=/tmp
RF_BENCH_SHARE_GPU=1 RF_BENCH_TRY_RCCL=1 NCCL_DEBUG=WARN timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29515 bench.py --gpus 2 --steps 3 --warmup 1 --sha-gib 1 --c4-samples 1000 \
    --gpu-only-run 0 --skip cpu,c1,install,probe > $O/bench2.json 2> $O/bench2.log
echo "torchrun rc=$?"; ls -la $O; grep -v "amdgpu.ids\|^\[W" $O/bench2.log | tail -30
