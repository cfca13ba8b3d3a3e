#!/bin/bash
# A/B of two library builds on the mark kernels, in phases (each GPU step
# under its own limit, a failure ends the call):
#   tests  -- the GPU suite on the in-tree library
#   forms  -- tools/dag_forms.py over configs[2], the 8-rank piece and the
#             100M layout at N = 1, other build then in-tree build
#   traces -- kernel traces of configs[2] and the 100M step, both builds
#   [FORMS='--c2 --c4-ranks 8'] [TRACES='c2 r8'] bash tools/gpu_ab_mark.sh <tag> <other.so> <phase>...
set -o pipefail
tag=$1; other=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for ph in "$@"; do
  case $ph in
  tests)
    echo "== tests ($(date +%T))"
    timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || exit $?
    tail -2 $out/gpu_tests.log ;;
  forms)
    for v in other main; do
      if [ $v = other ]; then lib="--lib $other"; else lib=""; fi
      echo "== forms $v ($(date +%T))"
      timeout -k 10 500 python3 -u tools/dag_forms.py ${FORMS:---c2 --c4-ranks 8,1} --steps 20 $lib >> $out/forms_$v.json 2>> $out/forms_$v.log || exit $?
    done ;;
  traces)
    for v in other main; do
      if [ $v = other ]; then lib="--lib $other"; else lib=""; fi
      for n in ${TRACES:-c2 r1}; do  # c2 = configs[2], rN = rank 0's piece at N ranks
        if [ $n = c2 ]; then g="--c2"; else g="--c4-ranks ${n#r}"; fi
        echo "== trace $v $n ($(date +%T))"
        timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_${v}_$n -o t \
            -- python3 tools/pmc_dag.py $g $lib > $out/trace_${v}_$n.json 2> $out/trace_${v}_$n.log || exit $?
      done
    done ;;
  esac
done
grep -h "auto" $out/forms_other.log $out/forms_main.log
exit 0
