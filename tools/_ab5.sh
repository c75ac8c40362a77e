set -o pipefail
mkdir -p gpurun_out/ab5
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_metric.py > gpurun_out/ab5/tests.log 2>&1; rc=$?
tail -n 5 gpurun_out/ab5/tests.log
[ $rc -eq 0 ] || exit $rc
for v in cur in-tree aw2 cur in-tree aw2; do
  if [ $v = in-tree ]; then unset ZKFL_LIB; else export ZKFL_LIB=build_ab/$v/libzkfl.so; fi
  timeout -k 10 150 python -u tools/ko_probe.py --steps 64 --warmup 8 >> gpurun_out/ab5/ko.log 2>&1 || exit 1
  tail -n 1 gpurun_out/ab5/ko.log
done
