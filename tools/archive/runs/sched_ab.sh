#!/bin/bash
# A/B of compiler scheduling variants of the compiled (J o H)^n program (design probe): each
# euclidiannormalizingflows.jl_amd/libenf_altN.so differs from libenf.so only in enf_flow_hj.hip's
# LLVM scheduler options (1: max-ilp, 2: schedule-metric-bias=100, 3: max-memory-clause). Runs in the
# gpurun snapshot, swapping the library file there. The alternative libraries are built by hand
# (hipcc with the extra -mllvm option on enf_flow_hj.hip, linked with the other objects) and were
# deleted after the measurement (profiles/r01_sched_variants.txt).
cd "${GRAFT_REPO_ROOT:-.}"
L=euclidiannormalizingflows.jl_amd
cp $L/libenf.so $L/libenf_base.so
for rep in 1 2; do
  for v in base alt1 alt2 alt3; do
    cp $L/libenf_$v.so $L/libenf.so
    timeout -k 5 120 python bench.py --no-cpu --steps 20 2>/dev/null \
      | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', round(d['roofline']['kernel_ms'],4), 'ms', round(d['roofline']['frac'],3))" \
      || { echo "failed $v"; exit 1; }
  done
done
cp $L/libenf_base.so $L/libenf.so
