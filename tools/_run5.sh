set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PMC_OUT=gpurun_out/pmc5 bash tools/pmc_passes.sh python -u tools/train_large.py 512 5 || exit $?
python tools/pmc_summary.py gpurun_out/pmc5 > gpurun_out/pmc5_summary.txt
grep -A12 'tc_kernel<4>\|tc_kernel<2>\|dw_kernel' gpurun_out/pmc5_summary.txt | head -80
for lib in "" tools/_dbg/libiwae_uncond.so; do
  env ${lib:+IWAE_HIP_LIB=$lib} timeout -k 10 150 python -u bench.py --steps 300 --warmup 20 --no-cpu --no-nll --large-batch-steps 20 > gpurun_out/ab5_$(basename x$lib).json 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab5_$(basename x$lib).json').read().strip().splitlines()[-1]); print('lib=$lib', d['ms_per_step'], d['configs0_train']['ms_per_step'], d['large_batch']['ms_per_step'], {n[:14]: v['avg_us'] for n, v in d['roofline']['kernels'].items()})"
done
