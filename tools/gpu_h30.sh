#!/bin/bash
# current K2 per-phase stamps (workgroup 0 of each launched level), configs[2]
set -o pipefail
O=gpurun_out/h30
mkdir -p $O
export TMPDIR=/tmp
RF_K2_STAMPS=1 timeout -k 10 150 python tools/dag_probe.py --dag-steps 3 > $O/probe.json 2> $O/stamps.log || { tail -5 $O/stamps.log; exit 1; }
RF_K2_STAMPS=2 timeout -k 10 150 python tools/dag_probe.py --dag-steps 3 > $O/probe2.json 2> $O/stamps2.log || { tail -5 $O/stamps2.log; exit 1; }
grep -c stamps $O/stamps.log $O/stamps2.log
