#!/bin/bash
# Update-kernel LDS swizzle gate: wave-count parity + the train tests, then the step A/B and one PMC pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-swz}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
EXTRA="--no-large-batch --no-c0 --no-stats" TUNES="default default" bash tools/ab_tune.sh || exit $?
TUNES="default" bash tools/lb_ab.sh || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc -o run -- python -u bench.py --steps 20 --warmup 5 --no-nll --no-cpu --no-c0 --no-large-batch --no-stats > $O/pmc.log 2>&1; echo "pmc rc=$?"
python - "$O" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True)
tot = collections.defaultdict(float)
for row in csv.DictReader(open(f[0])):
    if "upd_kernel" in row.get("Kernel_Name", ""):
        tot[row["Counter_Name"]] += float(row["Counter_Value"])
print({k: v for k, v in tot.items()})
PY
