#!/bin/bash
# Build an A/B variant of libzkfl.so with extra compile flags (CPU side, before gpurun):
#   bash tools/build_ab.sh NAME "-DKNOB=VALUE ..."   ->  build_ab/NAME/libzkfl.so
# then on the box: ZKFL_LIB=build_ab/NAME/libzkfl.so python bench.py ...  (tools/sweep_env.sh)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
PKG=$R/verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd
NAME=$1; FLAGS=${2:-}
# knock-out builds compute wrong proofs; msm_api.h refuses them without the acknowledgement
case "$FLAGS" in *ZK_KNOCKOUT*) FLAGS="$FLAGS -DZK_KNOCKOUT_AB_ONLY" ;; esac
OUT=$R/build_ab/$NAME
mkdir -p "$OUT"
CXX="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$R/include -I$PKG/csrc -Wno-unused-result $FLAGS"
pids=()
# the library's HIP sources, as the package Makefile lists them
SRCS=$(sed -n 's/^SRCS := //p' "$PKG/Makefile")
for s in $SRCS; do
  $CXX -c -o "$OUT/$s.o" "$PKG/csrc/$s.hip" & pids+=($!)
done
g++ -O2 -fPIC -std=c++17 -I"$R/include" -I"$PKG/csrc" -c -o "$OUT/host_parse.o" "$PKG/csrc/host_parse.cc" & pids+=($!)
echo "const char* zkfl_build_id(void) { return \"ab-$NAME\"; }" > "$OUT/build_id.c"
gcc -O2 -fPIC -c -o "$OUT/build_id.o" "$OUT/build_id.c"
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libzkfl.so" "$OUT"/*.o
rm -f "$OUT"/*.o
echo "built $OUT/libzkfl.so ($FLAGS)"
