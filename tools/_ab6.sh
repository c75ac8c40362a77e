set -o pipefail
mkdir -p gpurun_out/ab6
run() { echo "$*" >> gpurun_out/ab6/ko.log; timeout -k 10 150 "$@" >> gpurun_out/ab6/ko.log 2>&1 || exit 1; tail -n 1 gpurun_out/ab6/ko.log; }
for r in 1 2; do
  ZKFL_LIB=build_ab/cur/libzkfl.so run python -u tools/ko_probe.py --steps 64 --warmup 8
  ZKFL_LIB=build_ab/l32/libzkfl.so run python -u tools/ko_probe.py --steps 64 --warmup 8
  ZKFL_LIB=build_ab/l24/libzkfl.so run python -u tools/ko_probe.py --steps 64 --warmup 8
  ZKFL_LIB=build_ab/g2l24/libzkfl.so run python -u tools/ko_probe.py --steps 64 --warmup 8
done
ZKFL_LIB=build_ab/cur/libzkfl.so ZKFL_HW_QUEUES=32 run python -u tools/ko_probe.py --steps 64 --warmup 8 --slots 24
ZKFL_LIB=build_ab/cur/libzkfl.so ZKFL_HW_QUEUES=24 run python -u tools/ko_probe.py --steps 64 --warmup 8 --slots 16
ZKFL_LIB=build_ab/cur/libzkfl.so ZKFL_HW_QUEUES=32 run python -u tools/ko_probe.py --steps 64 --warmup 8 --slots 28
