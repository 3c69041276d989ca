#!/bin/bash
# Time diagnostic layer patterns through the flow kernel (one process each).
cd "${GRAFT_REPO_ROOT:-.}"
for P in ${PATS:-HJHJHJHJ HHHHHHHH JJJJJJJJ H J HJ}; do
  r=$(timeout -k 5 120 python bench.py --no-cpu --steps 20 --pattern $P ${BENCH_ARGS:-} 2>/dev/null) || { echo "$P failed"; exit 1; }
  echo "$P $(echo "$r" | python -c 'import json,sys; d=json.load(sys.stdin); print("kernel %.4f ms  %.1f GB/s" % (d["roofline"]["kernel_ms"], d["roofline"]["achieved"]))')"
done | tee gpurun_out/patterns.txt
