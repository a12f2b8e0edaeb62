#!/bin/bash
# The N > 1 bench path on the final tree, rehearsed on one GPU: --gpus 2 and
# --gpus 4 under gloo (ranks share the card; the launcher, the per-rank
# shards, the max-over-ranks timing and the NLL merge), with the driver's
# --steps 20 --warmup 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06g2; mkdir -p $O
for n in 2 4; do
  IWAE_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus $n --steps 20 --warmup 5 --no-cpu --no-stats \
    > $O/bench_gpus${n}_gloo.jsonl 2> $O/bench_gpus${n}_gloo.err || { tail -20 $O/bench_gpus${n}_gloo.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_gpus${n}_gloo.jsonl').read().strip().splitlines()[-1]); print($n, d['n_gpus'], d['value'], d['ms_per_step'], d['rccl_world'], d['nll']['images_per_rank'], d['nll']['value'], d['large_batch']['ms_per_step'])"
done
