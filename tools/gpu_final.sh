#!/bin/bash
# Round-end evidence on the GPU box: GPU tests, smoke, the default bench line, then the
# rocprofv3 summaries (tools/profile_round.sh).  Outputs under gpurun_out/final and gpurun_out/prof.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/final
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
bash tools/profile_round.sh
