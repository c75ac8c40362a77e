set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "edge or deep or identity" -x -q --timeout 200 --timeout-method thread > gpurun_out/parity.log 2>&1 || { tail -30 gpurun_out/parity.log; exit 1; }
tail -1 gpurun_out/parity.log
