set -o pipefail
mkdir -p gpurun_out/ab7
run() { echo "$*" >> gpurun_out/ab7/ko.log; timeout -k 10 150 "$@" >> gpurun_out/ab7/ko.log 2>&1 || exit 1; tail -n 1 gpurun_out/ab7/ko.log; }
for r in 1 2; do for v in cur v4 ns3 ns4 ns4g3; do
  ZKFL_LIB=build_ab/$v/libzkfl.so run python -u tools/ko_probe.py --steps 64 --warmup 8
done; done
