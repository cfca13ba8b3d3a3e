#!/bin/bash
# full GPU suite + smoke, then the incremental graph A/B
set -o pipefail
O=gpurun_out/h18
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
bash tools/gpu_ab.sh $O/ab - RF_K2_GRAPH=1
