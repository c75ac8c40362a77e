set -o pipefail
ZKFL_LIB=$PWD/build_ab/libzkfl_L24.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "msm or proof" -x -q --timeout 200 --timeout-method thread > gpurun_out/parity.log 2>&1 || { tail -30 gpurun_out/parity.log; exit 1; }
tail -1 gpurun_out/parity.log
bash tools/sweep_env.sh ZKFL_LIB "$PWD/build_ab/libzkfl_prev.so $PWD/build_ab/libzkfl_L24.so $PWD/build_ab/libzkfl_L32.so $PWD/build_ab/libzkfl_prev.so $PWD/build_ab/libzkfl_L24.so $PWD/build_ab/libzkfl_L32.so"
