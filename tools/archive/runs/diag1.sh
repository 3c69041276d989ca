#!/bin/bash
# Diagnostics: issue-cost microbench, debug-mode timings (interpreter), spec A/B, PMC issue counters.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 5 120 ./tools/microbench2 > gpurun_out/microbench2.txt 2>&1 || { echo "microbench2 failed"; exit 1; }
cat gpurun_out/microbench2.txt
PATS="HJHJHJHJ JJJJJJJJ HHHHHHHH" bash tools/dbgmodes.sh || exit 1
PATS="HJHJHJHJ" bash tools/spec_ab.sh || exit 1
LIST=1 bash tools/pmc.sh || exit 1
python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt 2>&1; cat gpurun_out/pmc_summary.txt
