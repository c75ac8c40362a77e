set -o pipefail
mkdir -p gpurun_out/ab4
for v in cur kos kon kosn cur kos kon kosn; do
  ZKFL_LIB=build_ab/$v/libzkfl.so timeout -k 10 120 python -u tools/ko_probe.py --steps 64 --warmup 8 >> gpurun_out/ab4/ko.log 2>&1 || exit 1
  tail -n 1 gpurun_out/ab4/ko.log
done
