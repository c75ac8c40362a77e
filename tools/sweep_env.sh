#!/bin/bash
# A/B sweep of an environment switch on the default bench (GPU box):
#   bash tools/sweep_env.sh VAR "v1 v2 ..." [extra bench args]
set -o pipefail
VAR=$1; VALS=$2; shift 2
mkdir -p gpurun_out/sweep
for v in $VALS; do
  LOG=gpurun_out/sweep/${VAR}_$(basename "$v").log
  env $VAR=$v timeout -k 10 150 python -u bench.py --steps 96 --warmup 16 --no-cpu-baseline "$@" > "$LOG" 2>&1 || exit 1
  echo "$VAR=$v $(tail -1 "$LOG" | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["stage_ms_isolated_per_proof"], d["roofline"]["valu"])')"
done
