#!/bin/bash
# A/B of configs[2] step variants selected by environment strings:
#   bash tools/gpu_ab.sh OUT "ENV=.. ENV2=.." "ENV=.." ...   ("-" = defaults)
# each variant twice, alternating; prints ms_per_step / device ms / dirty jobs
set -o pipefail
O=$1; shift
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  k=0
  for v in "$@"; do
    k=$((k+1))
    e=""; [ "$v" != "-" ] && e="$v"
    env $e timeout -k 10 150 python tools/dag_probe.py --dag-steps 50 > $O/ab_${k}_${r}.json 2>$O/ab_${k}_${r}.log || { echo "probe failed ($v)"; tail -5 $O/ab_${k}_${r}.log; exit 1; }
    echo "[$v] run $r: $(python -c "import json; d=json.load(open('$O/ab_${k}_${r}.json')); print(round(d['ms_per_step'],4), round(d['device_ms_per_step'],4), d['dirty_jobs_per_step'])")"
  done
done
