#!/bin/bash
# GPU-box driver for this round's checks: each step under its own time limit, output under
# gpurun_out/$TAG/<step>.log.  A step that fails normally (exit 1: test failures) lets the next one
# run; a time limit, abort, segfault or kill (124 / 134 / 137 / 139 / >128) ends the call there.
#   bash tools/gpu_run.sh TAG "name:seconds:command" ...
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
final=0
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "=== $name ($secs s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc in $(( $(date +%s) - start )) s"
  tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then final=$rc; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "=== stopping: $name ended with $rc"; exit $rc; fi
done
exit $final
