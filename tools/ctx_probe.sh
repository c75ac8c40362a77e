#!/bin/bash
# Fresh-process start-up costs (tools/ctx_probe.cc), 5 processes per condition: the HIP runtime
# alone, with libzkfl.so loaded, eager code-object loading, 28 hardware queues, and while another
# process holds a context on the same GPU.  Output: one JSON line per process, tagged.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
LIB=$R/verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd/libzkfl.so
P=$R/tools/ctx_probe
run() {  # tag, then env assignments / args
  local tag=$1; shift
  for i in 1 2 3 4 5; do
    printf '%s ' "$tag"; timeout -k 5 60 env "$@" || { echo "failed: $tag"; return 1; }
  done
}
run runtime_only $P || exit 1
run libzkfl $P $LIB || exit 1
run libzkfl_eager HIP_ENABLE_DEFERRED_LOADING=0 $P $LIB || exit 1
run libzkfl_q28 GPU_MAX_HW_QUEUES=28 $P $LIB || exit 1
# a second process holding a context (and the device awake) for the duration
timeout -k 5 40 python3 -c "
import sys, time; sys.path.insert(0, '$R/verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd')
from zkfl import native; c = native.Context(0); print('holder up', flush=True); time.sleep(25)" &
HOLDER=$!
sleep 8
run libzkfl_beside_holder $P $LIB
wait $HOLDER
