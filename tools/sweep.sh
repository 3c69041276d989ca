#!/bin/bash
# Tuning sweep of the fused flow kernel knobs (ENF_FRAG_U, ENF_BLOCKS_PER_CU); one process per point.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for U in ${US:-4 2 8}; do
  for B in ${BS:-0 2 3 4}; do
    r=$(ENF_FRAG_U=$U ENF_BLOCKS_PER_CU=$B timeout -k 5 120 python bench.py --no-cpu --steps 20 ${BENCH_ARGS:-} 2>/dev/null)
    rc=$?
    [ $rc -eq 0 ] || { echo "U=$U B=$B failed rc=$rc"; exit $rc; }
    echo "U=$U B=$B $(echo "$r" | python -c 'import json,sys; d=json.load(sys.stdin); print("%.4e samples/s kernel %.4f ms frac %.3f" % (d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"]))')"
  done
done | tee gpurun_out/sweep.txt
