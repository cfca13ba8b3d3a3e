#!/bin/bash
# Round-6 (session 3) K2 counters on the 100M layout at N = 1: a kernel trace
# and one SQ pass (VALU / wait shares, tools/pmc_valu.py), each its own run.
#   bash tools/gpu_sq6.sh <tag>
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
export TMPDIR=/tmp
echo "== trace ($(date +%T))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o p \
    -- python3 tools/pmc_dag.py --c4-ranks 1 > $out/trace.json 2> $out/trace.log || exit $?
python3 tools/trace_per_dispatch.py $(find $out/trace -name "*kernel_trace.csv" | head -1) > $out/per_dispatch.txt && grep -E "k2_level|k3_mark" $out/per_dispatch.txt
echo "== sq ($(date +%T))"
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $out/sq -o p -- python3 tools/pmc_dag.py --c4-ranks 1 > $out/sq.json 2> $out/sq.log || exit $?
python3 tools/pmc_valu.py $(find $out/sq -name "*counter_collection.csv" | head -1) k2_level k3_mark > $out/sq_valu_wait_100m.txt && cat $out/sq_valu_wait_100m.txt
