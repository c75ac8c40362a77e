#!/bin/bash
# HIP runtime start-up (tools/ctx_probe, runtime only) under environment variants, 5 processes each.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
P=$R/tools/ctx_probe
echo "kfd topology nodes: $(ls /sys/class/kfd/kfd/topology/nodes | wc -l); gpus with simds: $(grep -l 'simd_count [1-9]' /sys/class/kfd/kfd/topology/nodes/*/properties | wc -l)"
env | grep -E '^(HSA|HIP|ROCR|GPU_|AMD)' | sort
run() {
  local tag=$1; shift
  for i in 1 2 3 4 5; do printf '%s ' "$tag"; timeout -k 5 60 env "$@" $P || return 1; done
}
run default || exit 1
run rocr_visible0 ROCR_VISIBLE_DEVICES=0 || exit 1
run no_sdma HSA_ENABLE_SDMA=0 || exit 1
run no_interrupt HSA_ENABLE_INTERRUPT=0 || exit 1
run legacy_ipc_unset -u HSA_ENABLE_IPC_MODE_LEGACY || exit 1
