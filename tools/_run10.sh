set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt10.log 2>&1; rc=$?
tail -5 gpurun_out/pt10.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2 || exit $?
timeout -k 10 300 python -u tools/snr_c4.py 1000 > gpurun_out/snr10.txt 2>&1 || exit $?
cat gpurun_out/snr10.txt | grep -v amdgpu.ids
timeout -k 10 400 python -u bench.py > gpurun_out/bench10.jsonl 2> gpurun_out/bench10.err || exit $?
tail -1 gpurun_out/bench10.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step')}, 'nll', d['nll']['value'], 'lb', d['large_batch']['ms_per_step'], 'stats', d['training_statistics'], 'c0', d['configs0_train']['ms_per_step'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['threads_curve'])"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dp10 -o run -- python -u tools/dp_timeline.py > gpurun_out/dp10.log 2>&1 || exit $?
T=$(find gpurun_out/dp10 -name "*kernel_trace.csv" | head -1); python tools/step_timeline.py "$T" 14 "smallm_kernel<false>" > gpurun_out/dp10_timeline.txt; cat gpurun_out/dp10_timeline.txt
for lib in "" tools/_dbg/libiwae_mgold.so; do
  env ${lib:+IWAE_HIP_LIB=$lib} timeout -k 10 150 python -u bench.py --steps 50 --warmup 10 --no-cpu --no-large-batch --no-c0 --no-stats > gpurun_out/nll10_$(basename x$lib).json 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/nll10_$(basename x$lib).json').read().strip().splitlines()[-1]); print('lib=$lib nll', d['nll']['value'])"
done
