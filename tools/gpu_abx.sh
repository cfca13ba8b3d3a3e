#!/bin/bash
# A/B of several library builds on every DAG layout the bench times:
# configs[2], the 100M Merge-tree layout at N = 1 and its 8-rank piece, the
# per-sample-root layout at N = 1 and its 8-rank piece -- alternating builds,
# one process each; "main" = the in-tree library:
#   bash tools/gpu_abx.sh <tag> <lib1.so> [lib2.so ...]
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in main "$@"; do
    if [ $v = main ]; then lib=""; name=main; else lib="--lib $v"; name=$(basename $v .so); fi
    echo "== $rep $name ($(date +%T))"
    timeout -k 10 400 python3 -u tools/dag_forms.py --c2 --c4-ranks 1,8 --persample 1,8 --steps 20 $lib \
        > $out/forms_$name.$rep.json 2> $out/forms_$name.$rep.log || exit $?
    grep -h " auto " $out/forms_$name.$rep.log
  done
done
