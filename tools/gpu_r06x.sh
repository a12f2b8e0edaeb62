#!/bin/bash
# Driver-argument bench line (--steps 20 --warmup 5): is the short timed call
# slow because the GPU is cold?  (1) as is vs after extra untimed steps
# (bench_hot_tmp.py, an experiment copy), headline-only runs; (2) the full
# bench with the headline timed first (--headline-first) vs after the other
# legs (default), alternating.  (Historical: the bench that had --headline-first
# was reverted after this A/B, profiles/r06x_cold_and_leg_order_ab.txt; the hot arm
# needs bench_hot_tmp.py, an experiment copy that is not kept.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06x; mkdir -p $O
A="--steps 20 --warmup 5 --no-cpu --no-nll --no-large-batch --no-stats --no-c0 --headline-first"
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['ms_per_step'], d['train_step_calls']['ms_per_step'], (d.get('large_batch') or {}).get('ms_per_step'), (d.get('nll') or {}).get('value'))"; }
for i in 1 2 3; do
  for arm in cold hot; do
    B=bench.py; [ $arm = hot ] && B=bench_hot_tmp.py
    timeout -k 10 120 python -u $B $A > $O/$arm.$i.json 2> $O/$arm.$i.err || exit $?
    show $O/$arm.$i.json "$arm $i"
  done
done
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --headline-first > $O/first.$i.json 2> $O/first.$i.err || exit $?
  show $O/first.$i.json "first $i"
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/after.$i.json 2> $O/after.$i.err || exit $?
  show $O/after.$i.json "after $i"
done
