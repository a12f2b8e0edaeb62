#!/bin/bash
# GPU suite, then the --gpus 2 gloo rehearsal of the bench launcher, then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
IWAE_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 50 --warmup 10 --no-cpu --no-stats \
  > $O/bench_gpus2_gloo.jsonl 2> $O/bench_gpus2_gloo.err || exit $?
tail -c 1500 $O/bench_gpus2_gloo.jsonl
timeout -k 10 400 python -u bench.py > $O/bench.jsonl 2> $O/bench.err || exit $?
tail -1 $O/bench.jsonl
