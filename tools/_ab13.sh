# tail knobs on the round-3 kernels: stitching group 4 / 16 (default 8), bucket-reduction fold Q = 8 (default 16)
set -o pipefail
mkdir -p gpurun_out/ab13
run() { echo "$*" >> gpurun_out/ab13/ab.log; timeout -k 10 150 "$@" >> gpurun_out/ab13/ab.log 2>&1 || exit 1; tail -n 1 gpurun_out/ab13/ab.log; }
for r in 1 2; do for v in cur sg4 sg16 g1q8 g2q8; do
  if [ $v = cur ]; then run python -u tools/ko_probe.py --steps 40 --warmup 6
  else ZKFL_LIB=build_ab/$v/libzkfl.so run python -u tools/ko_probe.py --steps 40 --warmup 6; fi
done; done
