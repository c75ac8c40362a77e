#!/bin/bash
# Kernel trace of a short bench.py run + the per-proof serialized breakdown (GPU box).
#   bash tools/profile_breakdown.sh [TAG]   -> gpurun_out/prof_TAG/{breakdown.csv,kernel_stats.csv,bench.log}
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-bd}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ks" -o run -- python3 "$R/bench.py" --steps 32 --warmup 4 --no-cpu-baseline --e2e-steps 0 --c5-rounds 0 --merkle-log2n 0 > "$OUT/bench.log" 2>&1
python3 "$R/tools/rocpd_summary.py" kernels "$OUT/ks/run_results.db" "$OUT/kernel_stats.csv"
python3 "$R/tools/rocpd_summary.py" breakdown "$OUT/ks/run_results.db" "$OUT/breakdown.csv" 6
python3 "$R/tools/rocpd_summary.py" timeline "$OUT/ks/run_results.db" "$OUT/timeline.txt"
rm -rf "$OUT/ks"
cat "$OUT/breakdown.csv"
tail -1 "$OUT/bench.log"
