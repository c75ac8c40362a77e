# chunk-length A/B (G1 L = 16 / 24 / 32, G2 L = 24) on the round-3 tree
set -o pipefail
mkdir -p gpurun_out/ab9
run() { echo "$*" >> gpurun_out/ab9/ab.log; timeout -k 10 150 "$@" >> gpurun_out/ab9/ab.log 2>&1 || exit 1; tail -n 1 gpurun_out/ab9/ab.log; }
for r in 1 2; do for v in cur g1l24 g1l32 g2l24; do
  if [ $v = cur ]; then run python -u tools/ko_probe.py --steps 48 --warmup 8
  else ZKFL_LIB=build_ab/$v/libzkfl.so run python -u tools/ko_probe.py --steps 48 --warmup 8; fi
done; done
