#!/bin/bash
# Round-2 profile on the GPU box (run from the repo root):
#   1. the driver's bench command under rocprofv3 --kernel-trace --stats;
#   2. FETCH_SIZE and WRITE_SIZE passes (one counter group per run, as
#      MI355X_MICROARCH.md prescribes) over the same configs[1] SHA workload,
#      one step, summarised into pmc_traffic.json with its "workload" key;
#   3. probe-only passes: TCC_HIT/TCC_MISS and FETCH_SIZE for the 171 MiB
#      (MALL-resident) and 2 GiB (HBM) bloomlive filters (tools/pmc_probe.py).
# usage: bash tools/profile_r02.sh OUTDIR
set -euo pipefail
OUT=${1:-gpurun_out/prof2}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[prof] kernel trace of the driver command" >&2
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.log"
SHA="--steps 1 --warmup 0 --skip cpu,c1,install,dag,probe"
echo "[prof] FETCH_SIZE pass" >&2
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o f \
    -- python3 bench.py $SHA > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.log"
echo "[prof] WRITE_SIZE pass" >&2
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o w \
    -- python3 bench.py $SHA > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.log"
python3 tools/pmc_summary.py "$OUT/fetch/f_counter_collection.csv" "$OUT/write/w_counter_collection.csv" \
    "$OUT/pmc_traffic.json" "$OUT/pmc_fetch.json" > "$OUT/pmc_summary.txt"
PROBE="--steps 1 --warmup 0 --sha-gib 0.25 --gpu-only-run 0 --probe-steps 1 --skip cpu,c1,install,dag"
echo "[prof] probe TCC_HIT/TCC_MISS pass" >&2
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/tcc" -o t \
    -- python3 bench.py $PROBE > "$OUT/pmc_tcc.json" 2> "$OUT/pmc_tcc.log"
echo "[prof] probe FETCH_SIZE pass" >&2
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pfetch" -o pf \
    -- python3 bench.py $PROBE > "$OUT/pmc_pfetch.json" 2> "$OUT/pmc_pfetch.log"
python3 tools/pmc_probe.py "$OUT/tcc/t_counter_collection.csv" "$OUT/pfetch/pf_counter_collection.csv" \
    > "$OUT/pmc_probe.txt"
echo "[prof] done" >&2
