#!/bin/bash
# Few-row launches on the narrow (MU = 2, staging specialized) instantiations vs
# the generic ones (variant library built with -DIWAE_SM_NARROW=0): the GPU
# suite on the in-tree library, then B=20 bench train legs alternating.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05n}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for rep in 1 2 3; do
  for lib in "" tools/dbgx/libsmw.so; do
    if [ -n "$lib" ]; then export IWAE_HIP_LIB=$lib; else unset IWAE_HIP_LIB; fi
    timeout -k 10 150 python -u bench.py --steps 300 --warmup 20 --no-cpu --no-nll --no-large-batch > $O/b.json 2> $O/b.err || exit $?
    python -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('${lib:-in-tree}', d['ms_per_step'], d['configs0_train']['ms_per_step'])"
  done
done
unset IWAE_HIP_LIB
SP_TUNE="" bash tools/gpu_sptrace.sh ${TAG:-r05n}_tr tools/dbgx/libsmw.so | grep -E "==|smallm"
