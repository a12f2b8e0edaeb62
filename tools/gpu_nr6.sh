#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-nr6}
mkdir -p $O
for lib in tools/_dbg/libiwae_g4.so ""; do
  env ${lib:+IWAE_HIP_LIB=$lib} timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -q -x --timeout 120 --timeout-method thread -k "weight_ring or k5000_single" > $O/pt_$(basename x$lib).log 2>&1
  echo "lib=$lib rc=$?"; tail -1 $O/pt_$(basename x$lib).log
  env ${lib:+IWAE_HIP_LIB=$lib} timeout -k 10 200 python -u bench.py --no-cpu --steps 20 --no-large-batch --no-c0 --no-stats > $O/bench_$(basename x$lib).jsonl 2> $O/bench_$(basename x$lib).err || exit $?
  tail -1 $O/bench_$(basename x$lib).jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lib=$lib nll', d['nll']['value'])"
done
