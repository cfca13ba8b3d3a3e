#!/bin/bash
# A/B of two library builds on the 100M layouts (Merge-tree and per-sample,
# N = 1) and configs[2], alternating builds, one process each:
#   bash tools/gpu_ab100m.sh <tag> <other.so>
set -o pipefail
tag=$1; other=$2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for v in other main other main; do
  if [ $v = other ]; then lib="--lib $other"; else lib=""; fi
  echo "== $v ($(date +%T))"
  timeout -k 10 400 python3 -u tools/dag_forms.py --c2 --c4-ranks 1 --persample 1,8 --steps 20 $lib > $out/forms_$v.json 2>> $out/forms_$v.log || exit $?
done
grep -h "auto" $out/forms_other.log | sed 's/^/other: /'
grep -h "auto" $out/forms_main.log | sed 's/^/main:  /'
