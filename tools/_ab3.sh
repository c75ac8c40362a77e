set -o pipefail
mkdir -p gpurun_out/ab3
for v in g2s nr4 nl9 nl11 sb256 s7b256 nosf g2s nr4 nl11 sb256 nosf; do
  ZKFL_LIB=build_ab/$v/libzkfl.so timeout -k 10 120 python -u tools/ko_probe.py --steps 64 --warmup 8 >> gpurun_out/ab3/ko.log 2>&1 || exit 1
  tail -n 1 gpurun_out/ab3/ko.log
done
