#!/bin/bash
# round-close evidence on the final library (session 3, after the OpK producer-side frontier atomics): GPU suite + smoke, the driver's bench command (timed),
# then the same command under rocprofv3 --kernel-trace --stats (K1 unchanged since profiles/r02/final's PMC passes)
set -o pipefail
O=gpurun_out/final3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
s=$(date +%s.%N)
timeout -k 10 450 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || { echo bench failed; tail -5 $O/bench.log; exit 1; }
echo "bench wall $(python -c "print(round($(date +%s.%N) - $s, 1))") s; stdout lines $(grep -c '' $O/bench.json)"
python -c "import json; d=json.load(open('$O/bench.json')); i=d['incremental']; print(d['value'], d['ms_per_step'], d['roofline']['frac'], i['ms_per_step'], i['mnodes_per_s'], i.get('roofline_incremental'))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.log || { echo prof failed; tail -5 $O/bench_under_rocprof.log; exit 1; }
echo prof ok
