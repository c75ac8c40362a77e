#!/bin/bash
# Same-box throughput A/B of library variants (GPU box).  Variants alternate round by round, so a
# drift of the box's clock hits every variant alike; each run is one tools/ko_probe.py line.
#   bash tools/ab.sh TAG ROUNDS VARIANT... [-- PROBE_ARGS...]
# VARIANT: LIB[+VAR=VALUE...]; LIB "cur" = the in-tree libzkfl.so, otherwise build_ab/<LIB>/libzkfl.so
# (tools/build_ab.sh NAME "-DKNOB=..." builds one on the CPU first); +VAR=VALUE sets an environment
# knob for that variant's runs (e.g. cur+ZKFL_STAGGER=1).
# AB_PROBE=tools/c5_probe.py runs that probe instead of tools/ko_probe.py (same one-line output).
# Output: gpurun_out/TAG/ab.log (every line) and a per-variant summary (mean, min, max, spread).
# A run that fails, times out or crashes ends the script (nothing is retried).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; ROUNDS=$2; shift 2
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
PROBE=("$@")
[ ${#PROBE[@]} -eq 0 ] && [ -z "${AB_PROBE:-}" ] && PROBE=(--steps 40 --warmup 6)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for r in $(seq 1 "$ROUNDS"); do
  for v in "${VARS[@]}"; do
    IFS=+ read -r -a parts <<< "$v"
    base=${parts[0]}
    if [ "$base" = cur ]; then lib=""; else lib=build_ab/$base/libzkfl.so; fi
    line=$(env ZKFL_LIB="$lib" "${parts[@]:1}" timeout -k 10 180 python -u "${AB_PROBE:-tools/ko_probe.py}" "${PROBE[@]}" \
           2>>"$OUT/stderr.log" | tail -n 1)
    rc=$?
    [ $rc -ne 0 ] && { echo "$v round $r failed (rc $rc)"; exit $rc; }
    echo "$v $line" | tee -a "$OUT/ab.log"
  done
done
python3 - "$OUT/ab.log" <<'EOF'
import re, sys, collections
runs = collections.defaultdict(list)
for ln in open(sys.argv[1]):
    m = re.match(r"(\S+) .*: ([0-9.]+) (proofs/s|ms median)", ln)
    if m:
        runs[m.group(1)].append((float(m.group(2)), m.group(3)))
for v, xs in runs.items():
    u = xs[0][1]
    xs = [x for x, _ in xs]
    mean = sum(xs) / len(xs)
    print(f"{v}: mean {mean:.3f} {u} over {len(xs)} runs, min {min(xs):.3f}, max {max(xs):.3f}, "
          f"spread {100 * (max(xs) - min(xs)) / mean:.1f}%")
EOF
