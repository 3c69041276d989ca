#!/bin/bash
# NOTE: the dispatch knob this script sets was measured and then removed from the library (no variant
# beat the default; results under profiles/). Re-add the knob to the dispatcher to reproduce.
# A/B of the config-3 compiled program at higher occupancy: ENF_HJ_U1OCC = 0 (default R8 U2, 4
# waves/SIMD), 1 (R8 U1, 88 VGPRs, 5 waves), 6 / 8 (R8 U1 forced to 6 / 8 waves, spills), 9 (R8 U2
# forced to 5 waves, spills).
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
for v in 0 1 6 8 9; do
  ENF_HJ_U1OCC=$v timeout -k 5 120 python bench.py --no-cpu --steps 20 2>/dev/null \
    | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('ENF_HJ_U1OCC=$v', round(d['roofline']['kernel_ms'],4), 'ms', round(d['roofline']['frac'],3))" \
    || { echo "failed $v"; exit 1; }
done
done
