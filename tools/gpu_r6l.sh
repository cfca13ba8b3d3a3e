#!/bin/bash
set -o pipefail
out=gpurun_out/$1; mkdir -p $out; export TMPDIR=/tmp
echo "== diag"; timeout -k 10 90 python3 -u tools/diag_check.py tools/_ab/libreflow_diag.so > $out/diag.log 2>&1; rc=$?; tail -3 $out/diag.log; [ $rc = 0 ] || exit $rc
echo "== wg c4"; timeout -k 10 240 env RF_K2_WGSTAMPS=1 RF_K2_STAMPS=0 STAMP_LIB=tools/_ab/libreflow_diag.so python3 -u tools/stamp_probe.py c4 1 > $out/wg_c4.log 2>&1; rc=$?; grep -E "wgstamps|recomputed" $out/wg_c4.log | tail -40; [ $rc = 0 ] || exit $rc
echo "== wg ps8"; timeout -k 10 120 env RF_K2_WGSTAMPS=1 RF_K2_STAMPS=0 STAMP_LIB=tools/_ab/libreflow_diag.so python3 -u tools/stamp_probe.py ps 8 > $out/wg_ps8.log 2>&1; rc=$?; grep -E "wgstamps|recomputed" $out/wg_ps8.log | tail -12; exit $rc
