set -o pipefail
bash tools/sweep_env.sh ZKFL_LIB "$PWD/build_ab/libzkfl_L16.so $PWD/build_ab/libzkfl_L32.so"
