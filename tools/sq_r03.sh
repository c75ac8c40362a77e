#!/bin/bash
# Counter evidence for the SHIPPED MSM accumulation kernels (k_msm_accumulate<FqOps29,3> and
# <Fq2Pair29,2>), the NTT and the bucket sort (VERDICT r02 "Next round" 4): single-slot bench runs so
# every kernel is alone on the GPU (PMC dispatch collection serializes kernels anyway).
#   pass sq   : SQ issue / wait breakdown + VALU activity + GRBM_GUI_ACTIVE (launch cycles, 8 XCDs summed)
#   pass mix  : instruction mix (SALU / LDS / VMEM / VALU subclasses gfx950 offers, from rocprofv3 -L)
# Output: gpurun_out/sq3/sq_r03.txt (+ the raw per-kernel averages as JSON).  Run on the GPU box.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
# SQ_CIRCUIT=M19: the 2^19 leg's key instead of the metric key (output gpurun_out/sq3_M19)
CIRC=${SQ_CIRCUIT:-M}
OUT=$R/gpurun_out/sq3$([ "$CIRC" = M ] || echo "_$CIRC")
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
BENCH="$R/bench.py --circuit $CIRC --steps 3 --warmup 1 --slots 1 --no-cpu-baseline --e2e-steps 0 --c5-rounds 0 --c5-weak-rounds 0 --merkle-log2n 0 --extra-circuit none --split-proofs 0 --cli-runs 0"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/sq" -o run -- python3 $BENCH > "$OUT/sq.log" 2>&1
MIX=""
n=0
for c in SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA; do
  if [ $n -lt 8 ] && grep -qw "$c" "$OUT/counters_list.txt"; then MIX="$MIX $c"; n=$((n + 1)); fi
done
if [ -n "$MIX" ]; then
  timeout -s KILL 180 rocprofv3 --pmc $MIX --kernel-trace -d "$OUT/mix" -o run -- python3 $BENCH > "$OUT/mix.log" 2>&1
fi
export ZKFL_BUILD_ID=$(cd "$R" && python3 -c "import sys; sys.path.insert(0, 'verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd'); from zkfl import native; print(native.build_id())")
python3 - "$OUT" > "$OUT/sq_r03.txt" <<'PY'
import json, os, sqlite3, sys
out = sys.argv[1]
KEYS = ("msm", "ntt", "abc", "assemble")
def load(db):
    if not os.path.exists(db):
        return {}, {}
    c = sqlite3.connect(db)
    by, dur = {}, {}
    for k, n, v in c.execute("select kernel_name, counter_name, avg(value) from counters_collection group by kernel_name, counter_name"):
        if any(t in k for t in KEYS):
            by.setdefault(k.split("(")[0].replace("void zkfl::", ""), {})[n] = v
    try:
        for k, v in c.execute("select name, avg(end - start) from kernels group by name"):
            if any(t in k for t in KEYS):
                dur[k.split("(")[0].replace("void zkfl::", "")] = v
    except sqlite3.Error:
        pass
    return by, dur
def find_db(d):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("results.db"):
                return os.path.join(root, f)
    return ""
sq, dur = load(find_db(f"{out}/sq"))
mix, _ = load(find_db(f"{out}/mix"))
print("per-launch averages, single-slot bench (each kernel alone on the GPU).  SQ_* cycle counters are quad-cycles")
print("(x4 -> cycles); GRBM_GUI_ACTIVE is summed over the 8 XCDs (/8 -> launch cycles); clock = launch cycles / duration;")
print("valu_simd_busy = 4 * SQ_ACTIVE_INST_VALU / (1024 SIMDs * launch cycles): the share of all SIMD cycles in which")
print("some wave was executing a VALU instruction; valu_per_wave = ACTIVE_INST_VALU / WAVE_CYCLES")
res = {}
for k in sorted(set(sq) | set(mix)):
    d, m = sq.get(k, {}), mix.get(k, {})
    wc = d.get("SQ_WAVE_CYCLES", 0) or 1
    grbm = d.get("GRBM_GUI_ACTIVE", 0) / 8.0
    ns = dur.get(k, 0.0)
    r = {"waves": d.get("SQ_WAVES", 0), "duration_us": ns / 1e3, "launch_cycles": grbm,
         "clock_GHz": grbm / ns if ns else None,
         "wait_inst": d.get("SQ_WAIT_INST_ANY", 0) / wc, "wait_any": d.get("SQ_WAIT_ANY", 0) / wc,
         "active_inst": d.get("SQ_ACTIVE_INST_ANY", 0) / wc, "valu_per_wave": d.get("SQ_ACTIVE_INST_VALU", 0) / wc,
         "valu_simd_busy": 4 * d.get("SQ_ACTIVE_INST_VALU", 0) / (1024 * grbm) if grbm else None,
         "insts_valu": d.get("SQ_INSTS_VALU", 0)}
    r.update({c.lower(): v for c, v in m.items()})
    res[k] = r
    line = (f"{k[:58]:58s} dur {r['duration_us']:8.1f}us clk {r['clock_GHz'] or 0:4.2f} waves {r['waves']:8.0f} "
            f"wait_inst {r['wait_inst']:5.1%} wait_any {r['wait_any']:5.1%} active {r['active_inst']:5.1%} "
            f"valu/wave {r['valu_per_wave']:5.1%} valu_simd_busy {(r['valu_simd_busy'] or 0):5.1%} valu_insts {r['insts_valu']:.3e}")
    if m:
        line += " | " + " ".join(f"{c.replace('SQ_', '').lower()} {v:.3e}" for c, v in sorted(m.items()))
    print(line)
bid = os.environ.get("ZKFL_BUILD_ID", "")
json.dump({"build_id": bid or None, "source": "tools/sq_r03.sh (single-slot bench, SQ + GRBM passes)", "kernels": res},
          open(f"{out}/sq_r03.json", "w"), indent=1)
PY
rm -rf "$OUT/sq" "$OUT/mix"
cat "$OUT/sq_r03.txt"
