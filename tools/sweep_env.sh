#!/bin/bash
# Train-step ms/step under different values of one tuning env knob:
#   VAR=IWAE_DW_TARGET VALUES="768 256 128" bash tools/sweep_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in $VALUES; do
  env "$VAR=$v" timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 --no-nll --no-cpu > gpurun_out/sweep_$v.log 2>&1 || exit $?
  echo "$VAR=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sweep_$v.log)"
done
