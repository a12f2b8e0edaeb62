#!/bin/bash
# A/B of the driver-argument bench line (--steps 20 --warmup 5): graph upload at
# capture (in-tree lib) vs none (var/noupload.so), and the bench's order
# (prepare before warmup: bench.py; after: bench_old_tmp.py), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06v; mkdir -p $O
A="--steps 20 --warmup 5 --no-cpu --no-nll --no-large-batch --no-stats --no-c0"
for i in 1 2 3 4; do
  for arm in new old_lib old_bench; do
    case $arm in
      new) L=""; B=bench.py ;;
      old_lib) L=var/noupload.so; B=bench.py ;;
      old_bench) L=""; B=bench_old_tmp.py ;;
    esac
    if [ -n "$L" ]; then export IWAE_HIP_LIB=$L; else unset IWAE_HIP_LIB; fi
    timeout -k 10 120 python -u $B $A > $O/$arm.$i.json 2> $O/$arm.$i.err || exit $?
    python -c "import json,sys; d=json.loads(open('$O/$arm.$i.json').read().strip().splitlines()[-1]); print('$arm', $i, d['ms_per_step'], d['train_step_calls']['ms_per_step'])"
  done
done
