# same-box A/B: packed 29-bit G1 base records (in-tree) vs the previous build
set -o pipefail
mkdir -p gpurun_out/ab12
run() { echo "$*" >> gpurun_out/ab12/ab.log; timeout -k 10 150 "$@" >> gpurun_out/ab12/ab.log 2>&1 || exit 1; tail -n 1 gpurun_out/ab12/ab.log; }
for r in 1 2 3; do for v in cur prev; do
  if [ $v = cur ]; then run python -u tools/ko_probe.py --steps 48 --warmup 8
  else ZKFL_LIB=build_ab/$v/libzkfl.so run python -u tools/ko_probe.py --steps 48 --warmup 8; fi
done; done
