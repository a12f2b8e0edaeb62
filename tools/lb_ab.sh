#!/bin/bash
# Large-batch (configs[4] per-GPU share) A/B of env settings: ENVS="A=1 A=0,B=2" bash tools/lb_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lb
i=0
for e in ${ENVS}; do
  i=$((i+1))
  env $(echo "$e" | tr ',' ' ') timeout -k 10 150 python -u bench.py --steps 30 --warmup 5 --no-cpu --no-nll --no-c0 \
    > gpurun_out/lb/b$i.json 2> gpurun_out/lb/b$i.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/lb/b$i.json').read().strip().splitlines()[-1]); print('$e', d['ms_per_step'], d['large_batch']['ms_per_step'])"
done
