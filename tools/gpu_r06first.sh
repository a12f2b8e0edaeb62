#!/bin/bash
# First replay of a prepared train_steps graph vs its later replays, and 20
# steps as five 4-step graph launches (tools/steps_warm.py first), three
# processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06first; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/steps_warm.py first > $O/first.$i.txt 2>&1 || { tail $O/first.$i.txt; exit 1; }
  grep -v amdgpu.ids $O/first.$i.txt
done
