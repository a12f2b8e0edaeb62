#!/bin/bash
# Edge tests (train_steps, stale rows, ring NLL pin), then a train-only bench + kernel trace of the steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04c}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu --no-nll --no-large-batch --no-stats --no-c0 > $O/bench.jsonl 2> $O/bench.err || exit $?
python -c "import json;d=json.loads(open('$O/bench.jsonl').read().splitlines()[-1]);print(d['ms_per_step'],d['train_step_calls'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python -u bench.py --steps 200 --warmup 20 --no-cpu --no-nll --no-large-batch --no-c0 --no-stats > $O/bench_prof.log 2>&1 || exit $?
