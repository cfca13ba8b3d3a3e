#!/bin/bash
# Round 6 GPU sessions, every GPU step under its own limit, chained with &&:
#   bash tools/gpu_final6.sh <tag> A   the GPU suite, smoke(), the driver's bench command
#   bash tools/gpu_final6.sh <tag> B   the same bench command under rocprofv3 --kernel-trace --stats
#   bash tools/gpu_final6.sh <tag> N2  a 2-rank shared-GPU rehearsal of the N-rank bench path
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
if [ "$2" = A ]; then
    step tests && timeout -k 10 800 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 && tail -2 $out/gpu_tests.log &&
    step smoke && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 && tail -1 $out/smoke.log &&
    step bench && timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.log &&
    tail -6 $out/bench.log
elif [ "$2" = B ]; then
    step trace && timeout -k 10 800 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/trace_bench.json 2> $out/trace_bench.log &&
    python3 tools/trace_per_dispatch.py $(find $out/trace -name "*kernel_trace.csv" | head -1) > $out/per_dispatch.txt && head -40 $out/per_dispatch.txt
else
    step n2 && RF_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --skip probe,cpu,c1 \
        > $out/n2.json 2> $out/n2.log && tail -3 $out/n2.log
fi
rc=$?
echo "rc=$rc"
exit $rc
