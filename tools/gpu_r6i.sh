#!/bin/bash
set -o pipefail
out=gpurun_out/$1; mkdir -p $out; export TMPDIR=/tmp
echo "== small"; timeout -k 10 120 env RF_K2_WGSTAMPS=1 RF_K2_STAMPS=0 STAMP_LIB=tools/_ab/libreflow_diag.so python3 -u tools/stamp_probe.py 2000 > $out/wg_small.log 2>&1; rc=$?; tail -5 $out/wg_small.log; [ $rc = 0 ] &&
echo "== c4" && timeout -k 10 240 env RF_K2_WGSTAMPS=1 RF_K2_STAMPS=0 STAMP_LIB=tools/_ab/libreflow_diag.so python3 -u tools/stamp_probe.py c4 1 > $out/wg_c4.log 2>&1 && grep wgstamps $out/wg_c4.log | tail -30
