#!/bin/bash
# round 4, seventeenth GPU pass: the fp64 CenterStretch / CenterContract in-range paths with one division for the
# ladj, 1/b as a record, and the contract's y as one log1p (expm1 form): the whole GPU suite (the wide-range per-
# element centre tests among them), then the fp64 centre patterns at D = 2 and D = 32 (settled)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_gpu_17.txt 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r4_pytest_gpu_17.txt; exit 1; }
tail -2 gpurun_out/r4_pytest_gpu_17.txt
P=gpurun_out/r4_patterns17.jsonl
for pat in C K JC KJKJ CHS SHK; do
  $T 120 python bench.py --pattern $pat --D 2 --N 1000000 --dtype f64 --no-cpu --no-train --no-pmc --steps 20 >> $P 2>>gpurun_out/r4_patterns17.err || exit 1
done
for pat in C K; do
  $T 120 python bench.py --pattern $pat --N 5000000 --dtype f64 --no-cpu --no-train --no-pmc --steps 20 >> $P 2>>gpurun_out/r4_patterns17.err || exit 1
done
echo ALLDONE
