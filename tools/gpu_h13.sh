#!/bin/bash
# K2 per-phase stamps of workgroup 0 (chain wave 0, producer) on configs[2]: barrier mode and streamed mode
set -o pipefail
O=gpurun_out/h13
mkdir -p $O
export TMPDIR=/tmp
RF_K2_STAMPS=1 timeout -k 10 150 python tools/dag_probe.py --dag-steps 5 > $O/barrier.json 2> $O/barrier.log || { tail -5 $O/barrier.log; exit 1; }
RF_K2_STAMPS=1 RF_K2_STREAM=1 timeout -k 10 150 python tools/dag_probe.py --dag-steps 5 > $O/stream.json 2> $O/stream.log || { tail -5 $O/stream.log; exit 1; }
RF_K2_STAMPS=2 RF_K2_STREAM=1 timeout -k 10 150 python tools/dag_probe.py --dag-steps 5 > $O/stream2.json 2> $O/stream2.log || { tail -5 $O/stream2.log; exit 1; }
grep -c stamps $O/*.log
