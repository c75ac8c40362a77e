set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_witness.py -x -q --timeout 200 --timeout-method thread > gpurun_out/parity.log 2>&1 || { tail -30 gpurun_out/parity.log; exit 1; }
tail -2 gpurun_out/parity.log
timeout -k 10 200 python -u bench.py --steps 96 --warmup 16 --no-cpu-baseline > gpurun_out/bench_new.log 2>&1 || { tail -5 gpurun_out/bench_new.log; exit 1; }
tail -1 gpurun_out/bench_new.log
