#!/bin/bash
# A/B: compiled (H o J)^n program vs the interpreter, HJ patterns
cd "${GRAFT_REPO_ROOT:-.}"
for P in ${PATS:-HJHJHJHJ HJ HJHJ}; do
  for S in 0 1; do
    r=$(ENF_NO_SPECIALIZE=$S timeout -k 5 120 python bench.py --no-cpu --steps 20 --pattern $P 2>/dev/null) || { echo "$P $S failed"; exit 1; }
    echo "$P nospec=$S $(echo "$r" | python -c 'import json,sys; d=json.load(sys.stdin); print("kernel %.4f ms  %.1f GB/s" % (d["roofline"]["kernel_ms"], d["roofline"]["achieved"]))')"
  done
done | tee gpurun_out/spec_ab.txt
