#!/bin/bash
# A/B of environment settings on the 100M layouts (N = 1), one process each,
# alternating; "base" = no extra setting:
#   bash tools/gpu_abenv.sh <tag> "VAR=value [VAR2=value]" ["..."]
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
  k=0
  for v in base "$@"; do
    k=$((k+1))
    if [ "$v" = base ]; then envs=""; else envs="$v"; fi
    echo "== $rep [$v] ($(date +%T))"
    env $envs timeout -k 10 300 python3 -u tools/dag_forms.py --c4-ranks 1 --persample 1 --steps 20 \
        > $out/forms_$k.$rep.json 2> $out/forms_$k.$rep.log || exit $?
    grep -h " auto " $out/forms_$k.$rep.log
  done
done
