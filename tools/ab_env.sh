#!/bin/bash
# A/B of env switches on the bench's configs[1] train leg: ENVS="A=1 A=0,B=1" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
i=0
for e in ${ENVS}; do
  i=$((i+1))
  env $(echo "$e" | tr ',' ' ') timeout -k 10 120 python -u bench.py --steps 300 --warmup 20 --no-cpu --no-nll --no-large-batch \
    > gpurun_out/ab/r$i.json 2> gpurun_out/ab/r$i.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/ab/r$i.json').read().strip().splitlines()[-1]); print('$e', d['ms_per_step'], d['configs0_train']['ms_per_step'], {n[:14]: v['avg_us'] for n, v in d['roofline']['kernels'].items()})"
done
