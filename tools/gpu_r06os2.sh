#!/bin/bash
# The tree with the train engine compiled -Os: GPU suite, smoke, bench line,
# then one PMC pass of instruction-cache counters over the k=5000 NLL leg
# (nring_kernel is 66 KB of code against the 64 KB instruction cache).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06os2; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench.jsonl 2> $O/bench.err || exit $?
python -c "import json; d=json.loads(open('$O/bench.jsonl').read().strip().splitlines()[-1]); print('b20', d['ms_per_step'], 'calls', d['train_step_calls']['ms_per_step'], 'nll', d['nll']['value'], 'b512', d['large_batch']['ms_per_step'], 'c0', d['configs0_train']['ms_per_step'], 'tcu', d['roofline']['avg_us'])"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
  --output-format csv -d $O/icache_nll -o run -- python -u tools/nll_time.py 2000 > $O/icache_nll.log 2>&1; echo "icache pass rc=$?"
P=$(find $O/icache_nll -name "*counter_collection.csv" | head -1); [ -n "$P" ] && python tools/pmc_kernel.py "$P" nring_kernel > $O/icache_nll.txt 2>&1; head -20 $O/icache_nll.txt
