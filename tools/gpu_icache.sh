#!/bin/bash
# I-cache counters of the train step (short train-only bench), then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-icache}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d $O/ic -o run -- python -u bench.py --steps 20 --warmup 5 --no-nll --no-cpu --no-c0 --no-large-batch --no-stats > $O/ic.log 2>&1; echo "icache pass rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_IFETCH --output-format csv -d $O/sq -o run -- python -u bench.py --steps 20 --warmup 5 --no-nll --no-cpu --no-c0 --no-large-batch --no-stats > $O/sq.log 2>&1; echo "sq pass rc=$?"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 $O/pytest.log
