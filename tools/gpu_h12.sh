#!/bin/bash
# host leg diagnostics: wait vs hash time per thread (RF_HOST_LEG_TIMING), chunk size
set -o pipefail
O=gpurun_out/h12
mkdir -p $O
export TMPDIR=/tmp
for v in "RF_HOST_CHUNK_MB=8" "RF_HOST_CHUNK_MB=32" "RF_HOST_CHUNK_MB=2"; do
  env RF_HOST_LEG_TIMING=1 $v timeout -k 10 200 python bench.py --steps 3 --warmup 1 --gpu-only-run 0 --skip c1,install,dag,probe,cpu > $O/w.json 2> $O/w.log || { echo "failed $v"; tail -5 $O/w.log; exit 1; }
  python -c "import json; d=json.load(open('$O/w.json')); h=d['host_leg']; print('$v', d['value'], d['ms_per_step'], h['threads'], h['gbps'], d['config']['split_rank0'])"
  grep "host leg\]" $O/w.log | tail -2
done
