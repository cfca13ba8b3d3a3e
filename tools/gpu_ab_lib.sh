#!/bin/bash
# A/B of two library builds on one box: tools/dag_forms.py (configs[2] and
# the 8-rank piece, every form) and a kernel trace of configs[2]'s steps, for
# the in-tree library and for another build (tools/_ab/*.so).
#   bash tools/gpu_ab_lib.sh <tag> <other.so>
set -o pipefail
tag=$1; other=$2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for v in other main other main; do
  if [ $v = other ]; then lib="--lib $other"; else lib=""; fi
  timeout -k 10 400 python3 -u tools/dag_forms.py --c2 --c4-ranks 8 --steps 20 $lib > $out/forms_$v.json 2>> $out/forms_$v.log || exit $?
done
for v in other main; do
  if [ $v = other ]; then lib="--lib $other"; else lib=""; fi
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_$v -o t \
      -- python3 tools/pmc_dag.py --c2 $lib > $out/trace_$v.json 2> $out/trace_$v.log || exit $?
done
grep -h "auto" $out/forms_other.log $out/forms_main.log
