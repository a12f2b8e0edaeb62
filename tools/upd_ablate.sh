#!/bin/bash
# upd_kernel timing ablations: debug builds with -DIWAE_UPD_ABLATE=<mask> (4 no
# operand loads, 8 stop after the reduction, 16 no FX / GX copies, 32 no Adam,
# 64 no reduction; WRONG results) on the bench's train leg; prints the replayed avg.
# Build the libraries first (here, on the CPU):  BUILD=1 bash tools/upd_ablate.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
MASKS=${MASKS:-0 4 8 16 32 64}
if [ "${BUILD:-0}" = 1 ]; then
  for d in $MASKS; do OUT=libiwae_abl$d.so bash tools/build_debug.sh -DIWAE_UPD_ABLATE=$d || exit $?; done
  exit 0
fi
mkdir -p gpurun_out/abl
for d in $MASKS; do
  IWAE_HIP_LIB=tools/_dbg/libiwae_abl$d.so timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --no-cpu --no-nll \
    --no-large-batch --no-c0 > gpurun_out/abl/d$d.json 2> gpurun_out/abl/d$d.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/abl/d$d.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']; print('mask=$d', d['ms_per_step'], {n[:12]: v['avg_us'] for n, v in k.items()})"
done
