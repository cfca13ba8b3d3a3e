#!/bin/bash
set -o pipefail
O=gpurun_out/h19
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do for v in "-" "RF_K2_FULL_GRAPH=0"; do
  e=""; [ "$v" != "-" ] && e="$v"
  env $e timeout -k 10 150 python tools/dag_probe.py --dag-steps 20 > $O/f.json 2> $O/f.log || { tail -5 $O/f.log; exit 1; }
  echo "[$v] $(python -c "import json; d=json.load(open('$O/f.json')); print(round(d['full_recompute_ms'],4), round(d['ms_per_step'],4))")"
done; done
