set -o pipefail
mkdir -p gpurun_out/sweep
for cfg in "3 24 8" "1 24 24" "1 32 32" "1 16 16" "3 32 10"; do
  set -- $cfg
  ZKFL_SLOT_STREAMS=$1 ZKFL_HW_QUEUES=$2 timeout -k 10 120 python -u bench.py --steps 96 --warmup 16 --slots $3 --no-cpu-baseline > gpurun_out/sweep/s$1_q$2_n$3.log 2>&1 || exit 1
  echo "streams=$1 queues=$2 slots=$3 $(tail -1 gpurun_out/sweep/s$1_q$2_n$3.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["stage_ms_isolated_per_proof"])')"
done
