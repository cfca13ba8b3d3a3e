#!/bin/bash
# Session-3 close-out on the final library: the K2 traffic passes (their JSON
# into profiles/pmc_r06, which bench.py reads), then the GPU suite, smoke()
# and the driver's bench command (tools/gpu_final6.sh A).
#   bash tools/gpu_final6b.sh <tag>
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
bash tools/pmc_round6.sh $out/pmc dag 1 || exit $?
cp $out/pmc/c2/traffic.json profiles/pmc_r06/k2_traffic_configs2.json &&
cp $out/pmc/r1/traffic.json profiles/pmc_r06/k2_traffic_100m.json &&
cp profiles/pmc_r06/k2_traffic_*.json $out/ &&
bash tools/gpu_final6.sh $tag A
