#!/bin/bash
# Only the metric circuit M runs (the e2e / config-5 / dataset legs are off): the summaries select
# dispatches by kernel name and by position, which other circuits' launches would pollute.
# Reproduce the committed profiles/: rocprofv3 kernel-trace stats of the default bench.py run,
# separate PMC passes for FETCH_SIZE and WRITE_SIZE (MI355X_MICROARCH.md §rocprofv3 PMC slots:
# they cannot share a pass), and the FETCH_SIZE calibration of the MSM gather pattern.
# Run on the GPU box:  bash tools/profile_round.sh   (outputs under gpurun_out/prof/)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ks" -o run -- python3 "$R/bench.py" --no-cpu-baseline --e2e-steps 0 --c5-rounds 0 --merkle-log2n 0 --extra-circuit none --split-proofs 0 > "$OUT/bench_ks.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/fetch" -o run -- python3 "$R/bench.py" --steps 8 --warmup 1 --slots 2 --no-cpu-baseline --e2e-steps 0 --c5-rounds 0 --merkle-log2n 0 --extra-circuit none --split-proofs 0 > "$OUT/fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/write" -o run -- python3 "$R/bench.py" --steps 8 --warmup 1 --slots 2 --no-cpu-baseline --e2e-steps 0 --c5-rounds 0 --merkle-log2n 0 --extra-circuit none --split-proofs 0 > "$OUT/write.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/calib" -o run -- "$R/tools/pmc_calib" > "$OUT/calib.log" 2>&1
python3 "$R/tools/rocpd_summary.py" kernels "$OUT/ks/run_results.db" "$OUT/kernel_stats.csv"
python3 "$R/tools/rocpd_summary.py" roofline "$OUT/ks/run_results.db" "$OUT/bench_ks.log" "$OUT/roofline_pass.json"
BID=$(cd "$R" && python3 -c "import sys; sys.path.insert(0, 'verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd'); from zkfl import native; print(native.build_id())")
python3 "$R/tools/rocpd_summary.py" pmc "$OUT/fetch/run_results.db" "$OUT/write/run_results.db" "$OUT/calib/run_results.db" "$OUT/pmc_traffic.json" "$BID"
bash "$R/tools/sq_r03.sh" > "$OUT/sq.log" 2>&1
cp "$R/gpurun_out/sq3/sq_r03.json" "$OUT/sq_counters.json"
cp "$R/gpurun_out/sq3/sq_r03.txt" "$OUT/sq_counters.txt"
echo "profiles written to $OUT"
