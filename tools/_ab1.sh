set -o pipefail
mkdir -p gpurun_out/ab1
for r in 1 2; do for v in old t3 t4; do
  ZKFL_LIB=build_ab/$v/libzkfl.so timeout -k 10 120 python -u tools/ko_probe.py --steps 64 --warmup 8 >> gpurun_out/ab1/ko.log 2>&1 || exit 1
  tail -n 1 gpurun_out/ab1/ko.log
done; done
ZKFL_LIB=build_ab/t4/libzkfl.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_metric.py > gpurun_out/ab1/tests_t4.log 2>&1; tail -n 2 gpurun_out/ab1/tests_t4.log
