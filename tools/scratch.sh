set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3
