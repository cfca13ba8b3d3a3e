set -o pipefail
out=gpurun_out/fp; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 && tail -1 $out/gpu_tests.log &&
timeout -k 10 400 python -u tools/dag_forms.py --c2 --c4-ranks 8,1 --steps 20 > $out/forms.json 2> $out/forms.log && grep auto $out/forms.log
