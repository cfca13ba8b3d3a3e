#!/bin/bash
# Round 6: memo A/B on the 100M layouts, and a kernel trace of the Merge-tree A/B.
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
step ab_mt && timeout -k 10 300 python -u tools/memo_ab.py --layout mt > $out/ab_mt.json 2> $out/ab_mt.log && cat $out/ab_mt.json &&
step ab_ps && timeout -k 10 300 python -u tools/memo_ab.py --layout ps > $out/ab_ps.json 2> $out/ab_ps.log && cat $out/ab_ps.json &&
step trace && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o t -- python3 tools/memo_ab.py --layout mt --reps 1 --steps 10 > $out/trace_ab.json 2> $out/trace_ab.log &&
python3 tools/trace_per_dispatch.py $(find $out/trace -name "*kernel_trace.csv" | head -1) > $out/per_dispatch.txt && cat $out/per_dispatch.txt
rc=$?
echo "rc=$rc"
exit $rc
