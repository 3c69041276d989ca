#!/bin/bash
# A/B of two env settings, interleaved (thermal drift affects both): AB_A / AB_B env strings.
cd "${GRAFT_REPO_ROOT:-.}"
for i in 1 2 3; do
  for V in "${AB_A:-X=0}" "${AB_B:-X=1}"; do
    r=$(env $V timeout -k 5 120 python bench.py --no-cpu --steps 30 ${BENCH_ARGS:-} 2>/dev/null) || { echo "failed: $V"; exit 1; }
    echo "[$V] $(echo "$r" | python -c 'import json,sys; d=json.load(sys.stdin); print("%.4e samples/s kernel %.4f ms" % (d["value"], d["roofline"]["kernel_ms"]))')"
  done
done | tee gpurun_out/ab.txt
