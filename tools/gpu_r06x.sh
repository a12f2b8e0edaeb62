#!/bin/bash
# Driver-argument bench line (--steps 20 --warmup 5): as is vs after extra
# untimed steps (hot GPU), alternating: is the short timed call slow because
# the GPU is cold?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06x; mkdir -p $O
A="--steps 20 --warmup 5 --no-cpu --no-nll --no-large-batch --no-stats --no-c0"
for i in 1 2 3 4; do
  for arm in cold hot; do
    B=bench.py; [ $arm = hot ] && B=bench_hot_tmp.py
    timeout -k 10 120 python -u $B $A > $O/$arm.$i.json 2> $O/$arm.$i.err || exit $?
    python -c "import json,sys; d=json.loads(open('$O/$arm.$i.json').read().strip().splitlines()[-1]); print('$arm', $i, d['ms_per_step'], d['train_step_calls']['ms_per_step'])"
  done
done
timeout -k 10 120 python -u bench.py --no-cpu --no-nll --no-large-batch --no-stats --no-c0 > $O/default.json 2>&1 || exit $?
python -c "import json,sys; d=json.loads(open('$O/default.json').read().strip().splitlines()[-1]); print('default 200 steps', d['ms_per_step'])"
