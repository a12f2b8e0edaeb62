#!/bin/bash
# Run-to-run bitwise reproducibility of the final tree (tools/determinism_stress.py):
# B = 20 (the combined launch with the write-through hand-off), B = 512 (ring
# kernels), B = 100 (configs[0]-sized rows on the 2L model), fresh models.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06det; mkdir -p $O
timeout -k 10 300 python -u tools/determinism_stress.py 20 100 6 > $O/b20.txt 2>&1 || { tail $O/b20.txt; exit 1; }
grep -v amdgpu.ids $O/b20.txt | tail -3
timeout -k 10 300 python -u tools/determinism_stress.py 512 60 6 > $O/b512.txt 2>&1 || { tail $O/b512.txt; exit 1; }
grep -v amdgpu.ids $O/b512.txt | tail -3
timeout -k 10 300 python -u tools/determinism_stress.py 100 60 6 > $O/b100.txt 2>&1 || { tail $O/b100.txt; exit 1; }
grep -v amdgpu.ids $O/b100.txt | tail -3
