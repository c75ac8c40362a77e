set -o pipefail
mkdir -p gpurun_out/ab2
ZKFL_LIB=build_ab/g2s4/libzkfl.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_metric.py > gpurun_out/ab2/tests_g2s4.log 2>&1; rc=$?; tail -n 2 gpurun_out/ab2/tests_g2s4.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do for v in old t4 g2s g2s4; do
  ZKFL_LIB=build_ab/$v/libzkfl.so timeout -k 10 120 python -u tools/ko_probe.py --steps 64 --warmup 8 >> gpurun_out/ab2/ko.log 2>&1 || exit 1
  tail -n 1 gpurun_out/ab2/ko.log
done; done
for v in ko2 ko4 ko8 ko16 ko32 ko64 g2s; do
  ZKFL_LIB=build_ab/$v/libzkfl.so timeout -k 10 120 python -u tools/ko_probe.py --steps 64 --warmup 8 >> gpurun_out/ab2/ko.log 2>&1 || exit 1
  tail -n 1 gpurun_out/ab2/ko.log
done
