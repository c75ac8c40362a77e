#!/bin/bash
# SQ (sequencer) counters per kernel for a short single-slot bench run (GPU box):
# issue/wait breakdown of the MSM kernels.  Output: gpurun_out/sq/sq_counters.txt
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/sq
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d "$OUT/db" -o run -- python3 "$R/bench.py" --steps 4 --warmup 1 --slots 1 --no-cpu-baseline > "$OUT/bench.log" 2>&1
python3 - "$OUT/db/run_results.db" > "$OUT/sq_counters.txt" <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select kernel_name, counter_name, count(*), avg(value) from counters_collection group by kernel_name, counter_name").fetchall()
by = {}
for k, n, cnt, v in rows:
    if "msm" in k or "abc" in k or "ntt" in k or "assemble" in k:
        by.setdefault(k.split("(")[0].replace("void zkfl::", ""), {})[n] = v
for k, d in sorted(by.items()):
    wc = d.get("SQ_WAVE_CYCLES", 1) or 1
    print(f"{k[:70]:70s} waves {d.get('SQ_WAVES',0):9.0f} wave_cyc {wc:.3e} wait_inst {d.get('SQ_WAIT_INST_ANY',0)/wc:5.1%} "
          f"wait_any {d.get('SQ_WAIT_ANY',0)/wc:5.1%} active_inst {d.get('SQ_ACTIVE_INST_ANY',0)/wc:5.1%} "
          f"valu_insts {d.get('SQ_INSTS_VALU',0):.3e} busy {d.get('SQ_BUSY_CYCLES',0):.3e}")
PY
rm -rf "$OUT/db"
cat "$OUT/sq_counters.txt"
