#!/bin/bash
# Ring-kernel gate: the NLL parity tests first, then the whole GPU suite and the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-nring}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "nll or NLL" > $O/pytest_nll.log 2>&1; rc=$?
tail -5 $O/pytest_nll.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench.jsonl 2> $O/bench.err || exit $?
tail -1 $O/bench.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step')}, 'nll', d['nll']['value'], 'lb', d['large_batch']['ms_per_step'])"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
exit $rc
