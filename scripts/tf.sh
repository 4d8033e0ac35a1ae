set -o pipefail
O=gpurun_out/tf; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_fuzz.py -k "tall" > $O/tests.log 2>&1; tail -8 $O/tests.log
