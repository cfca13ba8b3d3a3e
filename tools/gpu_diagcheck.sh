#!/bin/bash
set -o pipefail
out=gpurun_out/$1; mkdir -p $out; export TMPDIR=/tmp
echo "== release"; timeout -k 10 90 python3 -u tools/diag_check.py reflow_amd/libreflow_hip.so > $out/release.log 2>&1; rc=$?; cat $out/release.log | tail -8; [ $rc = 0 ] || exit $rc
echo "== diag"; timeout -k 10 90 python3 -u tools/diag_check.py tools/_ab/libreflow_diag.so > $out/diag.log 2>&1; rc=$?; cat $out/diag.log | tail -8; exit $rc
