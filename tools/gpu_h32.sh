#!/bin/bash
# finer K2 stamps (RF_K2_STAMPS=2: chain stamps around the first iteration's expansion and block step)
set -o pipefail
O=gpurun_out/h32
mkdir -p $O
export TMPDIR=/tmp
RF_K2_STAMPS=2 timeout -k 10 150 python tools/dag_probe.py --dag-steps 3 > $O/probe.json 2> $O/stamps.log || { tail -5 $O/stamps.log; exit 1; }
grep stamps $O/stamps.log | head -4
