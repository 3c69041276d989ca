#!/bin/bash
# Diagnostic timings: normal / synthesized input (no loads) / compute only (no loads, no stores)
cd "${GRAFT_REPO_ROOT:-.}"
for P in ${PATS:-HJHJHJHJ JJJJJJJJ H}; do
  for M in 0 1 2; do
    r=$(ENF_DEBUG_MODE=$M timeout -k 5 120 python bench.py --no-cpu --steps 20 --pattern $P 2>/dev/null) || { echo "$P $M failed"; exit 1; }
    echo "$P mode=$M $(echo "$r" | python -c 'import json,sys; d=json.load(sys.stdin); print("kernel %.4f ms" % d["roofline"]["kernel_ms"])')"
  done
done | tee gpurun_out/dbgmodes.txt
