#!/bin/bash
# Config-5 step time A/B on the diagnostics library (bench_train.py --diag): fused-gradient kernel
# variants by ENF_* knobs (ENF_GRAD_RU: columns per lane per tile of hj_grad_reg_kernel; ENF_GRAD_BPC:
# blocks per CU). Interleaved twice. gpurun_out/train_ab.txt
set -u
cd "${GRAFT_REPO_ROOT:-.}"
for i in 1 2; do
  for V in ${VARIANTS:-"ENF_GRAD_RU=1" "ENF_GRAD_RU=2"}; do
    r=$(env ${V//,/ } timeout -k 5 120 python bench_train.py --diag ${ARGS:-} 2>/dev/null) || { echo "failed: $V"; exit 1; }
    echo "[$V] $(echo "$r" | python -c 'import json,sys; d=json.load(sys.stdin); print("%.0f steps/s  %.2f us/step" % (d["value"], d["ms_per_step"] * 1e3))')"
  done
done | tee gpurun_out/train_ab.txt
