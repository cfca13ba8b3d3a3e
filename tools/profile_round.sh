#!/bin/bash
# Round profile on the GPU box: bench.py under rocprofv3 --kernel-trace --stats,
# then one PMC pass each for FETCH_SIZE and WRITE_SIZE (separate runs, as
# MI355X_MICROARCH.md prescribes), summarised by tools/pmc_summary.py.
# Usage (from the repo root, on the box): bash tools/profile_round.sh OUTDIR
set -euo pipefail
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench \
    -- python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.log"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o f \
    -- python3 bench.py --steps 1 --warmup 0 --skip cpu > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o w \
    -- python3 bench.py --steps 1 --warmup 0 --skip cpu > "$OUT/pmc_write.log" 2>&1
python3 tools/pmc_summary.py "$OUT/fetch/f_counter_collection.csv" "$OUT/write/w_counter_collection.csv" \
    "$OUT/pmc_traffic.json" > "$OUT/pmc_summary.txt"
