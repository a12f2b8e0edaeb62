set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "" tools/_dbg/libiwae_nostore.so; do
  env ${lib:+IWAE_HIP_LIB=$lib} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p9$(basename x$lib) -o lb -- python -u tools/train_large.py 512 10 > gpurun_out/p9.log 2>&1 || exit $?
  T=$(find gpurun_out/p9$(basename x$lib) -name "*kernel_trace.csv" | head -1); echo "== $lib"; python tools/kernel_by_grid.py "$T" | head -5
done
