set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r04k; mkdir -p $O
for lib in none dbg/libdw1.so dbg/libdw2.so dbg/libdw4.so dbg/libdw12.so; do
  if [ $lib = none ]; then L=""; else L="IWAE_HIP_LIB=$lib"; fi
  timeout -k 10 120 env $L rocprofv3 --kernel-trace --output-format csv -d $O/p_$(basename $lib) -o run -- python -u tools/train_large.py 512 6 auto dw_wide=1 > $O/l_$(basename $lib).log 2>&1 || exit $?
  F=$(find $O/p_$(basename $lib) -name "*kernel_trace.csv" | head -1); echo "== $lib"; python tools/kernel_by_grid.py "$F" dw_kernel
done
