#!/bin/bash
# NOTE: the dispatch knob this script sets was measured and then removed from the library (no variant
# beat the default; results under profiles/). Re-add the knob to the dispatcher to reproduce.
# A/B of the D = 64 compiled-program layouts (ENF_HJ64: 0 = R8 U2, 1 = R16 U1, 2 = R16 U2) on the
# config-4 shard (D = 64, N = 1.25e7 per GPU, 4 x (J o H), fp32).
cd "${GRAFT_REPO_ROOT:-.}"
for v in 0 1 2 0 1 2; do
  ENF_HJ64=$v timeout -k 5 120 python bench.py --no-cpu --D 64 --N 12500000 --pairs 4 --steps 20 2>/dev/null \
    | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('ENF_HJ64=$v', round(d['roofline']['kernel_ms'],4), 'ms', round(d['roofline']['frac'],3))" \
    || { echo "failed $v"; exit 1; }
done
