#!/bin/bash
# Round-6 traffic passes (the round-4 recipe) on the GPU box (MI355X_MICROARCH.md "HBM": one
# counter per run, FETCH_SIZE and WRITE_SIZE in separate passes, kernel
# trace only).  K2/K3: tools/pmc_dag.py on configs[2] and on rank 0's piece
# at R ranks; K1: the bench's GPU-only duo run (bench.py --steps 1, cpu and
# lowering legs skipped) -> profiles-ready pmc_traffic.json.
#   bash tools/pmc_round4.sh OUTDIR [dag|bench|all] [R...]
set -o pipefail
OUT=${1:-gpurun_out/pmc}; WHAT=${2:-all}; if [ $# -ge 2 ]; then shift 2; else shift $#; fi; RANKS=${@:-8}
mkdir -p "$OUT"
export TMPDIR=/tmp
rc=0
if [ "$WHAT" = dag ] || [ "$WHAT" = all ]; then
  for g in c2 $(for r in $RANKS; do echo r$r; done); do
    if [ $g = c2 ]; then a="--c2"; else a="--c4-ranks ${g#r}"; fi
    mkdir -p "$OUT/$g"
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/$g/$c" -o p \
          -- python3 tools/pmc_dag.py $a > "$OUT/$g/$c.json" 2> "$OUT/$g/$c.log" || { rc=$?; echo "pmc $g $c failed rc=$rc"; exit $rc; }
    done
    python3 tools/pmc_dag_summary.py "$OUT/$g/FETCH_SIZE/p_counter_collection.csv" \
        "$OUT/$g/WRITE_SIZE/p_counter_collection.csv" "$OUT/$g/FETCH_SIZE.json" "$OUT/$g/traffic.json" | tail -1
  done
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  mkdir -p "$OUT/bench"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 500 rocprofv3 --pmc $c --output-format csv -d "$OUT/bench/$c" -o p \
        -- python3 bench.py --steps 1 --warmup 0 --skip cpu,lower,dag,dag100m,piece,probe,c1 \
        > "$OUT/bench/$c.json" 2> "$OUT/bench/$c.log" || { rc=$?; echo "pmc bench $c failed rc=$rc"; exit $rc; }
  done
  python3 tools/pmc_summary.py "$OUT/bench/FETCH_SIZE/p_counter_collection.csv" \
      "$OUT/bench/WRITE_SIZE/p_counter_collection.csv" "$OUT/bench/pmc_traffic.json" "$OUT/bench/FETCH_SIZE.json" | tail -3
fi
exit $rc
