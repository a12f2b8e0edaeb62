#!/bin/bash
# upd_kernel timing ablations (IWAE_UPD_DBG bits: 1 no MFMA, 2 no LDS staging,
# 4 no activation loads, 8 stop after the reduction, 32 after the gradient write, 16
# after Adam) on the bench's train leg; prints the replayed avg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abl
for d in ${DBGS:-0 1 2 4 3 7}; do
  IWAE_UPD_DBG=$d timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --no-cpu --no-nll --no-large-batch --no-c0 \
    > gpurun_out/abl/d$d.json 2> gpurun_out/abl/d$d.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/abl/d$d.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']; print('dbg=$d', d['ms_per_step'], {n[:12]: v['avg_us'] for n, v in k.items()})"
done
