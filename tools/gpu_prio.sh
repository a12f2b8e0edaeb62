#!/bin/bash
# NLL A/B of debug builds (tools/_dbg/*.so) against the release library: bench NLL leg only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-prio}
mkdir -p $O
for lib in "" ${LIBS}; do
  env ${lib:+IWAE_HIP_LIB=$lib} timeout -k 10 200 python -u bench.py --no-cpu --steps 20 --no-large-batch --no-c0 --no-stats > $O/bench_$(basename x$lib).jsonl 2> $O/bench_$(basename x$lib).err || exit $?
  tail -1 $O/bench_$(basename x$lib).jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lib=$lib nll', d['nll']['value'], 'step', d['ms_per_step'])"
done
