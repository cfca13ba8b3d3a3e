set -e
for r in 0 40 82; do
  export RF_K2_RESERVE=$r
  echo "reserve $r KiB"
  timeout -k 10 120 python tools/dag_probe.py --dag-steps 50 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['mnodes_per_s'])"
done
