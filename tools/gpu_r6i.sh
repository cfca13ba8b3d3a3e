#!/bin/bash
set -o pipefail
out=gpurun_out/$1; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 env RF_K2_WGSTAMPS=1 RF_K2_STAMPS=0 STAMP_LIB=tools/_ab/libreflow_diag.so python3 -u tools/stamp_probe.py c4 1 > $out/wg_c4.log 2>&1 && grep wgstamps $out/wg_c4.log | tail -24 &&
timeout -k 10 300 env RF_K2_WGSTAMPS=1 RF_K2_STAMPS=0 STAMP_LIB=tools/_ab/libreflow_diag.so python3 -u tools/stamp_probe.py ps 1 > $out/wg_ps.log 2>&1 && grep wgstamps $out/wg_ps.log | tail -12 &&
timeout -k 10 500 python3 -u tools/dag_forms.py --c4-ranks 1 --persample 1 --steps 20 --extra > $out/forms.json 2> $out/forms.log && grep "ms/step" $out/forms.log
