#!/bin/bash
# Config 5: the fused gradient kernel with its transcendentals grouped at wave priority 3 (diagnostics build,
# ENF_GRAD_PRIO=1) against the shipped schedule; bench_train.py --diag, interleaved; negll_last must agree bit for
# bit (same operations). gpurun_out/gradprio.txt
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  for V in ENF_GRAD_PRIO=0 ENF_GRAD_PRIO=1; do
    r=$(env $V timeout -k 5 120 python bench_train.py --diag 2>/dev/null) || { echo "failed: $V"; exit 1; }
    echo "[$V] $(echo "$r" | python -c 'import json,sys; d=json.load(sys.stdin); print("%.0f steps/s  %.2f us/step  negll_last %r" % (d["value"], d["ms_per_step"] * 1e3, d["negll_last"]))')"
  done
done | tee gpurun_out/gradprio.txt
