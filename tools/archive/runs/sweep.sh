#!/bin/bash
# Tuning sweep of the fused flow kernel knobs; one process per point. POINTS = "U:OCC:BLOCKS_PER_CU ..."
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for P in ${POINTS:-4:1:0 2:1:0 2:6:0 2:8:0 4:5:0}; do
  IFS=: read U O B <<< "$P"
  r=$(ENF_FRAG_U=$U ENF_FRAG_OCC=$O ENF_BLOCKS_PER_CU=$B timeout -k 5 120 python bench.py --no-cpu --steps 20 ${BENCH_ARGS:-} 2>/dev/null)
  rc=$?
  [ $rc -eq 0 ] || { echo "U=$U OCC=$O B=$B failed rc=$rc"; exit $rc; }
  echo "U=$U OCC=$O B=$B $(echo "$r" | python -c 'import json,sys; d=json.load(sys.stdin); print("%.4e samples/s kernel %.4f ms frac %.3f" % (d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"]))')"
done | tee gpurun_out/sweep.txt
