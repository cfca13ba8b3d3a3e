#!/bin/bash
# Round 5 evidence passes, each GPU step under its own limit, chained:
#   trace  the driver's bench command under rocprofv3 --kernel-trace --stats
#   sqw    SQ VALU / wait counters over configs[2]'s and the 100M DAG's steps (tools/gpu_r5b.sh sqw)
#   k4     FETCH_SIZE / WRITE_SIZE passes over the probe leg (tools/gpu_r5b.sh k4)
#   bash tools/gpu_r5c.sh <tag> [trace,sqw,k4]
set -o pipefail
tag=$1
what=${2:-trace,sqw,k4}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
has() { [[ ",$what," == *",$1,"* ]]; }
rocm-smi --showclocks > $out/clocks.txt 2>&1 || true
if has trace; then
  echo "== trace ($(date +%T))"
  timeout -s KILL 900 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o bench \
      -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_under_rocprof.json 2> $out/bench_under_rocprof.log || exit $?
fi
if has sqw || has k4; then
  w=""; has sqw && w="sqw"; has k4 && w="$w,k4"
  bash tools/gpu_r5b.sh $tag ${w#,} || exit $?
fi
echo rc=0
