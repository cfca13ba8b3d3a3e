#!/bin/bash
# Round 6: the driver's bench command on the current tree, then a 2-rank
# shared-GPU rehearsal of the N-rank path (both DAG layouts), every GPU step
# under its own time limit, chained with && (a failure ends it).
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
step bench && timeout -k 10 800 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.log &&
tail -4 $out/bench.log &&
step n2 && RF_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 3 --skip probe,cpu,c1 \
    > $out/n2.json 2> $out/n2.log && tail -3 $out/n2.log
rc=$?
echo "rc=$rc"
exit $rc
