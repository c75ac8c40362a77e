# slots x hardware-queue re-sweep on the round-3 kernels (tools/ko_probe.py, main path, 20-slot default)
set -o pipefail
mkdir -p gpurun_out/sweep3
for r in 1 2; do for c in "20 28" "24 32" "22 28" "18 24" "20 32" "16 20"; do set -- $c
  echo "slots $1 queues $2" >> gpurun_out/sweep3/sweep.log
  ZKFL_HW_QUEUES=$2 timeout -k 10 150 python -u tools/ko_probe.py --steps 40 --warmup 6 --slots $1 >> gpurun_out/sweep3/sweep.log 2>&1 || exit 1
  tail -n 1 gpurun_out/sweep3/sweep.log
done; done
