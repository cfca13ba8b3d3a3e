set -e
timeout -k 10 300 python -u bench.py --sha-gib 0.25 --dag-samples 200 --skip cpu,dag,probe 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['c1']['file_ids_ms'], d['c1']['fixture_match'])"
