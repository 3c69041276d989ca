#!/bin/bash
# NOTE: the dispatch knob this script sets was measured and then removed from the library (no variant
# beat the default; results under profiles/). Re-add the knob to the dispatcher to reproduce.
# A/B of the D = 2 fragment-kernel variants (ENF_D2_VARIANT: 0 = U4, 1 = U2, 2 = U4 occ4,
# 3 = U2 occ4, 4 = U1 occ4) on config 2 (J o H, D = 2, N = 1e6, fp64) and its fp32 twin.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in 0 1 2 3 4; do
  for dt in f64 f32; do
    ENF_D2_VARIANT=$v timeout -k 5 120 python bench.py --no-cpu --D 2 --N 1000000 --pairs 1 --dtype $dt --steps 200 2>/dev/null \
      | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('variant $v $dt', round(d['roofline']['kernel_ms']*1e3,2), 'us', round(d['roofline']['frac'],3))" \
      || { echo "failed variant $v $dt"; exit 1; }
  done
done
