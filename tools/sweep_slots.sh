#!/bin/bash
# Proof slots x streams per slot x HW queues sweep of the default bench (GPU box).
#   bash tools/sweep_slots.sh STREAMS,QUEUES,SLOTS ...
set -o pipefail
mkdir -p gpurun_out/sweep
for cfg in "$@"; do
  IFS=, read -r S Q N <<< "$cfg"
  LOG=gpurun_out/sweep/s${S}_q${Q}_n${N}.log
  ZKFL_SLOT_STREAMS=$S ZKFL_HW_QUEUES=$Q timeout -k 10 150 python -u bench.py --steps 96 --warmup 16 --slots $N --no-cpu-baseline > $LOG 2>&1 || exit 1
  echo "streams=$S queues=$Q slots=$N $(tail -1 $LOG | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"])')"
done
