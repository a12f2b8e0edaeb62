#!/bin/bash
# Debug build of the library into tools/_dbg/ (git-ignored .so; gpurun-ignored too:
# DBG_DIR=dbgx puts it where a gpurun call takes it along), e.g.
#   bash tools/build_debug.sh -DIWAE_GEMM_TRACE      -> tools/_dbg/libiwae_dbg.so
# then run a tool with IWAE_HIP_LIB=tools/_dbg/libiwae_dbg.so.
set -e
cd "$(dirname "$0")/.."
D=${DBG_DIR:-tools/_dbg}; mkdir -p $D
S=iwae_replication_project_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-result \
  -o $D/${OUT:-libiwae_dbg.so} $S/iwae_gemm.hip $S/iwae_elem.hip $S/iwae_fused.hip $S/iwae_mega.hip $S/iwae_nring.hip $S/iwae_train.hip $S/iwae_update.hip $S/iwae_dwgrad.hip $S/iwae_model.hip -lrccl "$@"
