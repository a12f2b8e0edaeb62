#!/bin/bash
# Ring train-forward gate: its parity tests, the configs[4]-share oracle test, NLL tests, then the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-tr}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "weight_ring or configs4 or nll or NLL or wide_engine" > $O/pytest_tr.log 2>&1; rc=$?
tail -3 $O/pytest_tr.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu --steps 50 --no-c0 --no-stats > $O/bench.jsonl 2> $O/bench.err || exit $?
tail -1 $O/bench.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step')}, 'nll', d['nll']['value'], 'lb', d['large_batch']['ms_per_step'])"
