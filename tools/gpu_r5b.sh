#!/bin/bash
# Round 5 probes on the GPU box, every GPU step under its own limit, chained:
#   atomic   same-address atomic contention (tools/micro.py atomic)
#   forms    the level forms and the flow step on configs[2] and the 8-rank piece
#   sqw      SQ VALU / wait counters (one pass) over configs[2] and the 100M DAG's steps
#   k4       FETCH_SIZE and WRITE_SIZE passes over the bench's probe leg
#   trace    kernel trace + stats of configs[2]'s and the 100M DAG's steps
#   lower    tools/lower_bench with per-sample reference chains, phase times
#   bash tools/gpu_r5b.sh <tag> [atomic,forms,sqw,k4,trace,lower]
set -o pipefail
tag=$1
what=${2:-atomic,forms,sqw,k4,trace,lower}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
step() { echo "== $1 ($(date +%T))"; }
has() { [[ ",$what," == *",$1,"* ]]; }
rc=0
if has atomic; then
  step atomic && timeout -k 10 120 python3 -u tools/micro.py atomic > $out/atomic.log 2>&1 && cat $out/atomic.log || exit $?
fi
if has lower; then
  step lower && RF_LOWER_TIMING=1 timeout -k 10 300 tools/lower_bench 22075 32 dup > $out/lower.json 2> $out/lower.log && cat $out/lower.json || exit $?
fi
if has trace; then
  for g in c2 r1; do
    if [ $g = c2 ]; then a="--c2"; else a="--c4-ranks 1"; fi
    step "trace $g" && timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_$g -o t \
        -- python3 tools/pmc_dag.py $a > $out/trace_$g.json 2> $out/trace_$g.log || exit $?
  done
fi
if has forms; then
  step forms && timeout -k 10 600 python3 -u tools/dag_forms.py --c2 --c4-ranks 8 --steps 20 > $out/forms.json 2> $out/forms.log && grep -E "ms/step" $out/forms.log || exit $?
fi
if has sqw; then
  for g in c2 r1; do
    if [ $g = c2 ]; then a="--c2"; else a="--c4-ranks 1"; fi
    step "sqw $g" && timeout -s KILL 400 rocprofv3 --pmc $SQ --output-format csv -d $out/sqw_$g -o p \
        -- python3 tools/pmc_dag.py $a > $out/sqw_$g.json 2> $out/sqw_$g.log || exit $?
    python3 tools/pmc_valu.py $out/sqw_$g/p_counter_collection.csv k3_mark k2_level > $out/sqw_$g.txt && head -40 $out/sqw_$g.txt
  done
fi
if has k4; then
  mkdir -p $out/k4
  for c in FETCH_SIZE WRITE_SIZE; do
    step "k4 $c" && timeout -s KILL 500 rocprofv3 --pmc $c --output-format csv -d $out/k4/$c -o p \
        -- python3 bench.py --steps 1 --warmup 0 --skip cpu,lower,dag,dag100m,piece,persample,c1,install,checkpoint \
        > $out/k4/$c.json 2> $out/k4/$c.log || exit $?
  done
  python3 tools/pmc_k4_summary.py $out/k4/FETCH_SIZE/p_counter_collection.csv $out/k4/WRITE_SIZE/p_counter_collection.csv \
      1000000000 10 $out/k4/k4_traffic.json
fi
echo "rc=$rc"
exit $rc
