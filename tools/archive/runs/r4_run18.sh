#!/bin/bash
# round 4, eighteenth GPU pass: the fp32 CenterStretch / CenterContract steps with fewer transcendentals (the ladj
# from inner / e1, e2 instead of two more exp2; the contract's output as one log2 of a product): the whole GPU suite,
# then the fp32 D = 32 centre patterns (settled)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_gpu_18.txt 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r4_pytest_gpu_18.txt; exit 1; }
tail -2 gpurun_out/r4_pytest_gpu_18.txt
P=gpurun_out/r4_patterns18.jsonl
for pat in C K JC KJKJ CHS SHK; do
  $T 120 python bench.py --pattern $pat --no-cpu --no-train --no-pmc --steps 20 >> $P 2>>gpurun_out/r4_patterns18.err || exit 1
done
echo ALLDONE
