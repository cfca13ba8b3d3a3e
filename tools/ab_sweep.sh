# Same-process A/Bs of load-time options against the defaults (tools/ab_load.py),
# one after another on one box; every run under its own time limit
set -o pipefail
out=gpurun_out/${1:-sweep}; mkdir -p $out
shift
for spec in "$@"; do
    graph=${spec%%:*}; env=${spec#*:}
    timeout -k 10 240 python -u tools/ab_load.py --env "$env" $graph --reps 5 --steps 20 > "$out/${graph//[- ]/}_${env}.json" 2> "$out/${graph//[- ]/}_${env}.log" || exit $?
    tail -1 "$out/${graph//[- ]/}_${env}.log" | cut -c1-300
done
