set -o pipefail
ZKFL_LIB=$PWD/build_ab/libzkfl_trim.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/parity.log 2>&1 || { tail -30 gpurun_out/parity.log; exit 1; }
tail -1 gpurun_out/parity.log
bash tools/sweep_env.sh ZKFL_LIB "$PWD/build_ab/libzkfl_prev.so $PWD/build_ab/libzkfl_trim.so $PWD/build_ab/libzkfl_prev.so $PWD/build_ab/libzkfl_trim.so"
