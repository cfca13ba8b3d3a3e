#!/bin/bash
# stdout hygiene: N=1 short bench and the 2-rank rehearsal with the RCCL attempt; stdout must be ONE JSON line
set -o pipefail
O=gpurun_out/h38
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --sha-gib 4 --gpu-only-run 0 --skip cpu,install,probe > $O/b1.json 2> $O/b1.log || { echo b1 failed; tail -5 $O/b1.log; exit 1; }
echo "N=1 stdout lines: $(grep -c '' $O/b1.json)"; python -c "import json; d=json.load(open('$O/b1.json')); print(d['value'], d['incremental']['ms_per_step'])"
RF_BENCH_SHARE_GPU=1 RF_BENCH_TRY_RCCL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29516 bench.py --gpus 2 --steps 3 --warmup 1 --sha-gib 1 --c4-samples 1000 \
    --gpu-only-run 0 --skip cpu,c1,install,probe > $O/b2.json 2> $O/b2.log || { echo b2 failed; tail -5 $O/b2.log; exit 1; }
echo "N=2 stdout lines: $(grep -c '' $O/b2.json)"; python -c "import json; d=json.load(open('$O/b2.json')); print(d['value'], d['config']['exchange'][:60], d['incremental']['ms_per_step'])"
