#!/bin/bash
# Only the metric circuit M runs (the e2e / config-5 / dataset legs are off): the summaries select
# dispatches by kernel name and by position, which other circuits' launches would pollute.
# Reproduce the committed profiles/: rocprofv3 kernel-trace stats of the default bench.py run,
# the exact HBM bytes per launch from the L2's request-size counters (tools/pmc_attrib.sh: three
# separate --pmc passes; FETCH_SIZE counts a 128-B request as 64 B on gfx950) and the SQ counters.
# Run on the GPU box:  bash tools/profile_round.sh   (outputs under gpurun_out/prof/)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ks" -o run -- python3 "$R/bench.py" --no-cpu-baseline --e2e-steps 0 --c5-rounds 0 --merkle-log2n 0 --extra-circuit none --split-proofs 0 --cli-runs 0 > "$OUT/bench_ks.log" 2>&1
python3 "$R/tools/rocpd_summary.py" kernels "$OUT/ks/run_results.db" "$OUT/kernel_stats.csv"
python3 "$R/tools/rocpd_summary.py" roofline "$OUT/ks/run_results.db" "$OUT/bench_ks.log" "$OUT/roofline_pass.json"
bash "$R/tools/pmc_attrib.sh" "$OUT/pmc" > "$OUT/pmc.log" 2>&1
cp "$OUT/pmc/pmc_traffic.json" "$OUT/pmc_traffic.json"
bash "$R/tools/sq_r03.sh" > "$OUT/sq.log" 2>&1
cp "$R/gpurun_out/sq3/sq_r03.json" "$OUT/sq_counters.json"
cp "$R/gpurun_out/sq3/sq_r03.txt" "$OUT/sq_counters.txt"
# the 2^19-domain leg's key (bench.py extra_circuit): its own traffic and clock summaries
bash "$R/tools/pmc_attrib.sh" "$OUT/pmc_m19" M19 > "$OUT/pmc_m19.log" 2>&1
cp "$OUT/pmc_m19/pmc_traffic.json" "$OUT/pmc_traffic_m19.json"
SQ_CIRCUIT=M19 bash "$R/tools/sq_r03.sh" > "$OUT/sq_m19.log" 2>&1
cp "$R/gpurun_out/sq3_M19/sq_r03.json" "$OUT/sq_counters_m19.json"
cp "$R/gpurun_out/sq3_M19/sq_r03.txt" "$OUT/sq_counters_m19.txt"
echo "profiles written to $OUT"
