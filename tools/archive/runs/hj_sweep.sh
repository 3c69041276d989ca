#!/bin/bash
# Sweep the compiled (J o H)^n kernel variants: ENF_HJ_U / ENF_HJ_OCC / ENF_BLOCKS_PER_CU.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for P in ${POINTS:-8:0:0 4:0:0 16:0:0 8:1:0 4:1:0}; do
  IFS=: read U O B <<< "$P"
  r=$(ENF_HJ_R=$U ENF_HJ_U2=$O ENF_BLOCKS_PER_CU=$B timeout -k 5 120 python bench.py --no-cpu --steps 20 ${BENCH_ARGS:-} 2>/dev/null)
  rc=$?
  [ $rc -eq 0 ] || { echo "R=$U U2=$O B=$B failed rc=$rc"; exit $rc; }
  echo "R=$U U2=$O B=$B $(echo "$r" | python -c 'import json,sys; d=json.load(sys.stdin); print("%.4e samples/s kernel %.4f ms frac %.3f" % (d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"]))')"
done | tee gpurun_out/hj_sweep.txt
