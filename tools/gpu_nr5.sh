#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-nr5}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "nll or NLL or statistics" > $O/pytest_nll.log 2>&1; rc=$?
tail -2 $O/pytest_nll.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --no-cpu --steps 20 --no-large-batch --no-c0 --no-stats > $O/bench.jsonl 2> $O/bench.err || exit $?
tail -1 $O/bench.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('nll', d['nll']['value'])"
IWAE_HIP_LIB=tools/_dbg/libiwae_nrtrace.so timeout -k 10 120 python -u tools/nr_trace.py > $O/nr_trace.txt 2>&1 || exit $?
grep "^rec" $O/nr_trace.txt
