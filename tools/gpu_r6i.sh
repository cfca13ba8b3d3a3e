#!/bin/bash
set -o pipefail
out=gpurun_out/$1; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/dag_forms.py --c4-ranks 1 --persample 1 --steps 20 --extra > $out/forms.json 2> $out/forms.log; rc=$?; grep "ms/step" $out/forms.log; exit $rc
