#!/bin/bash
# A variant library that differs from the in-tree build in some source files:
# those recompiled with extra flags, every other object reused from build/obj
# (run __graft_entry__.build() first).
#   bash tools/build_variant.sh <out.so> <a.hip[,b.hip...]> -DFLAG=... [more flags]
set -e
cd "$(dirname "$0")/.."
OUT=$1; SRCS=$2; shift 2
S=iwae_replication_project_amd/csrc
mkdir -p "$(dirname "$OUT")" build/var
TAG=$(basename "$OUT" .so)
OBJS=""
for f in iwae_gemm iwae_elem iwae_fused iwae_mega iwae_nring iwae_train iwae_update iwae_dwgrad iwae_model; do
  if [[ ",$SRCS," == *",$f.hip,"* ]]; then
    # (the in-tree build compiles these three without the SLP vectorizer: __graft_entry__.SOURCE_FLAGS)
    NOSLP=""; case $f in iwae_train|iwae_update|iwae_gemm) NOSLP=-fno-slp-vectorize ;; esac
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $NOSLP "$@" -c -o build/var/${f}_${TAG}.o $S/$f.hip
    OBJS="$OBJS build/var/${f}_${TAG}.o"
  else
    OBJS="$OBJS build/obj/$f.o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $OBJS -lrccl
