#!/bin/bash
# A/B of several library builds on the 100M layouts (N = 1), alternating
# builds, one process each; "main" = the in-tree library:
#   bash tools/gpu_abn.sh <tag> <lib1.so> [lib2.so ...]
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in main "$@"; do
    if [ $v = main ]; then lib=""; name=main; else lib="--lib $v"; name=$(basename $v .so); fi
    echo "== $rep $name ($(date +%T))"
    timeout -k 10 300 python3 -u tools/dag_forms.py --c4-ranks 1 --persample 1 --steps 20 $lib > $out/forms_$name.$rep.json 2> $out/forms_$name.$rep.log || exit $?
    grep -h " auto " $out/forms_$name.$rep.log
  done
done
