#!/bin/bash
# ring-kernel ablations (timing only): no weight DMA, no MFMAs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-nr4}
mkdir -p $O
for lib in "" tools/_dbg/libiwae_NODMA.so tools/_dbg/libiwae_NOMMA.so; do
  env ${lib:+IWAE_HIP_LIB=$lib} timeout -k 10 200 python -u bench.py --no-cpu --steps 20 --no-large-batch --no-c0 --no-stats > $O/bench_$(basename x$lib).jsonl 2> $O/bench_$(basename x$lib).err || exit $?
  tail -1 $O/bench_$(basename x$lib).jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lib=$lib nll', d['nll']['value'])"
done
IWAE_HIP_LIB=tools/_dbg/libiwae_nrtrace.so timeout -k 10 120 python -u tools/nr_trace.py > $O/nr_trace.txt 2>&1 || exit $?
grep "^rec" $O/nr_trace.txt
