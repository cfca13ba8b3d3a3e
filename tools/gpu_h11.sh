#!/bin/bash
# host-leg width: SHA-NI chains interleaved per thread (RF_HOST_WAYS) and thread count, configs[1] SHA only
set -o pipefail
O=gpurun_out/h11
mkdir -p $O
export TMPDIR=/tmp
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; lscpu | grep -E "Model name|Thread|Core|Socket" | head -5
for v in "RF_HOST_WAYS=2" "RF_HOST_WAYS=3" "RF_HOST_WAYS=4" "RF_HOST_WAYS=1" "RF_HOST_THREADS=24" "RF_HOST_THREADS=12"; do
  env $v timeout -k 10 200 python bench.py --steps 5 --warmup 1 --gpu-only-run 0 --skip c1,install,dag,probe,cpu > $O/w.json 2> $O/w.log || { echo "failed $v"; tail -5 $O/w.log; exit 1; }
  python -c "import json; d=json.load(open('$O/w.json')); h=d['host_leg']; print('$v', d['value'], d['ms_per_step'], h['threads'], h['gbps'], d['config']['split_rank0'])"
done
