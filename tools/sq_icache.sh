#!/bin/bash
# Is the G1 accumulation's SQ_WAIT_INST_ANY an instruction-cache problem or VALU issue contention?
# (VERDICT r01 "What's weak" 5.)  Run on the GPU box; outputs under gpurun_out/sqi/.
#   1. rocprofv3 -L: the counters gfx950 offers (saved for reference)
#   2. SQ issue/wait pass + VALU activity, single-slot bench (kernels one at a time)
#   3. SQC instruction-cache pass (hits / misses) on the same run shape
# PMC dispatch collection serializes kernels, so a "concurrent" per-kernel pass does not exist;
# the single-slot pass already has every kernel alone on the GPU.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/sqi
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
BENCH="$R/bench.py --steps 3 --warmup 1 --slots 1 --no-cpu-baseline --e2e-steps 0 --c5-rounds 0 --merkle-log2n 0 --extra-circuit none"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d "$OUT/sq" -o run -- python3 $BENCH > "$OUT/sq.log" 2>&1
IC=""
for c in SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE; do
  if grep -qw "$c" "$OUT/counters_list.txt"; then IC="$IC $c"; fi
done
if [ -n "$IC" ]; then
  timeout -s KILL 240 rocprofv3 --pmc $IC SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/ic" -o run -- python3 $BENCH > "$OUT/ic.log" 2>&1
fi
python3 - "$OUT" > "$OUT/sq_icache.txt" <<'PY'
import os, sqlite3, sys
out = sys.argv[1]
def load(db):
    if not os.path.exists(db):
        return {}
    c = sqlite3.connect(db)
    by = {}
    for k, n, v in c.execute("select kernel_name, counter_name, avg(value) from counters_collection group by kernel_name, counter_name"):
        if any(t in k for t in ("msm", "abc", "ntt", "assemble")):
            by.setdefault(k.split("(")[0].replace("void zkfl::", ""), {})[n] = v
    return by
sq, ic = load(f"{out}/sq/run_results.db"), load(f"{out}/ic/run_results.db")
print("per launch averages; SQ_* cycle counters in quad-cycles; valu_util = ACTIVE_INST_VALU / WAVE_CYCLES summed over the SIMD's waves")
for k in sorted(set(sq) | set(ic)):
    d, e = sq.get(k, {}), ic.get(k, {})
    wc = d.get("SQ_WAVE_CYCLES", 0) or 1
    line = f"{k[:62]:62s}"
    if d:
        line += (f" waves {d.get('SQ_WAVES',0):7.0f} wait_inst {d.get('SQ_WAIT_INST_ANY',0)/wc:5.1%} wait_any {d.get('SQ_WAIT_ANY',0)/wc:5.1%}"
                 f" active {d.get('SQ_ACTIVE_INST_ANY',0)/wc:5.1%} active_valu {d.get('SQ_ACTIVE_INST_VALU',0)/wc:5.1%}"
                 f" valu_insts {d.get('SQ_INSTS_VALU',0):.3e}")
    if e:
        req = e.get("SQC_ICACHE_REQ") or (e.get("SQC_ICACHE_HITS", 0) + e.get("SQC_ICACHE_MISSES", 0)) or 1
        line += (f" | icache req {req:.3e} hit {e.get('SQC_ICACHE_HITS',0)/req:6.2%} miss {e.get('SQC_ICACHE_MISSES',0)/req:6.3%}"
                 f" miss_dup {e.get('SQC_ICACHE_MISSES_DUPLICATE',0)/req:6.3%} grbm {e.get('GRBM_GUI_ACTIVE',0):.3e}")
    print(line)
PY
rm -rf "$OUT/sq" "$OUT/ic"
cat "$OUT/sq_icache.txt"
