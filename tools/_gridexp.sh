set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_parity.py tests/test_golden_fixtures.py tests/test_host_cpp.py -x -q --timeout 120 --timeout-method thread
for v in pc lanes; do
  echo "k2 $v"; if [ $v = lanes ]; then export RF_K2_LANES=1; fi
  timeout -k 10 120 python tools/dag_probe.py --dag-steps 50 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['device_ms_per_step'], d['mnodes_per_s'], d['full_recompute_ms'])"
done
