#!/bin/bash
# A full GPU-box session: the focus tests, the GPU suite, smoke(), the
# driver's bench command, then the K2 form A/B on one box (default; round 3's
# forms: RF_K2_OCT=0 RF_K2_SINK_LAST=0 RF_K2_SPLIT=0; split block 0 off;
# default again), per-level workgroup stamps of the 8-rank piece, and the PMC
# traffic passes.  Every GPU
# step has its own time limit; the steps are chained so a failure ends it.
#   FOCUS="tests/..." bash tools/gpu_s2.sh <tag> A    focus tests, GPU suite, smoke, bench
#   bash tools/gpu_s2.sh <tag> B                        forms A/B, stamps, PMC passes
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
if [ "$2" = A ]; then
    step focus && { [ -z "$FOCUS" ] || timeout -k 10 400 python -u -m pytest $FOCUS -x -v --timeout 200 --timeout-method thread > $out/focus.log 2>&1; } && tail -2 $out/focus.log &&
    step tests && timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 && tail -2 $out/gpu_tests.log &&
    step smoke && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 && tail -1 $out/smoke.log &&
    step bench && RF_LOWER_TIMING=1 timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.log &&
    tail -4 $out/bench.log
else
step forms && timeout -k 10 400 python -u tools/dag_forms.py --c2 --c4-ranks 8 > $out/forms_new.json 2> $out/forms_new.log &&
RF_K2_OCT=0 RF_K2_SINK_LAST=0 RF_K2_SPLIT=0 timeout -k 10 400 python -u tools/dag_forms.py --c2 --c4-ranks 8 > $out/forms_old.json 2> $out/forms_old.log &&
RF_K2_SPLIT=0 timeout -k 10 400 python -u tools/dag_forms.py --c2 --c4-ranks 8 > $out/forms_nosplit.json 2> $out/forms_nosplit.log &&
timeout -k 10 400 python -u tools/dag_forms.py --c2 --c4-ranks 8 > $out/forms_new2.json 2> $out/forms_new2.log &&
grep "ms/step" $out/forms_new.log $out/forms_old.log $out/forms_nosplit.log $out/forms_new2.log &&
step stamps && RF_K2_WGSTAMPS=1 timeout -k 10 300 python -u tools/stamp_probe.py c4 8 > $out/wg_c4r8.log 2>&1 &&
step pmc && timeout -k 10 900 bash tools/pmc_round4.sh $out/pmc all 8 > $out/pmc.log 2>&1
fi
rc=$?
echo "rc=$rc"
tail -3 $out/focus.log $out/gpu_tests.log 2>/dev/null
tail -3 $out/pmc.log 2>/dev/null
exit $rc
