#!/bin/bash
# HBM traffic of the MSM accumulation kernels by request size: three separate
# rocprofv3 --pmc passes (<= 4 TCC counters each, MI355X_MICROARCH.md) over a one-slot ko_probe run
# of the metric circuit, then tools/pmc_attrib.py.  FETCH_SIZE counts a 128-B read request as 64 B
# on gfx950; the 32/64/128-B request counters give the read bytes exactly.  Run on the GPU box:
#   bash tools/pmc_attrib.sh [OUTDIR [CIRCUIT]]   (default gpurun_out/pmc_attrib, M; M19: the 2^19 leg)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=${1:-$R/gpurun_out/pmc_attrib}
mkdir -p "$OUT"
OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
PROBE=("$R/tools/ko_probe.py" --slots 1 --steps 2 --warmup 1 --circuit "${2:-M}")
pass() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o run -- python3 "${PROBE[@]}" \
      > "$OUT/$name.log" 2>&1
}
pass rd TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
pass wr TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
pass hit TCC_HIT_sum TCC_MISS_sum
python3 "$R/tools/pmc_attrib.py" "$OUT" "${2:-M}" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
