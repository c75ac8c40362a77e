# knock-out marginal costs on the round-3 tree (cur = the in-tree library)
set -o pipefail
mkdir -p gpurun_out/ab8
run() { echo "$*" >> gpurun_out/ab8/ko.log; timeout -k 10 150 "$@" >> gpurun_out/ab8/ko.log 2>&1 || exit 1; tail -n 1 gpurun_out/ab8/ko.log; }
for r in 1 2; do for v in cur ko8 ko16 ko64 ko32; do
  if [ $v = cur ]; then run python -u tools/ko_probe.py --steps 48 --warmup 8
  else ZKFL_LIB=build_ab/$v/libzkfl.so run python -u tools/ko_probe.py --steps 48 --warmup 8; fi
done; done
