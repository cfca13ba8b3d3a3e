set -e
for v in 0 1; do
  echo "hash2 $v"; if [ $v = 1 ]; then export RF_DBG_HASH2=1; fi
  timeout -k 10 120 python tools/dag_probe.py --dag-steps 50 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['device_ms_per_step'], d['mnodes_per_s'], d['full_recompute_ms'])"
done
