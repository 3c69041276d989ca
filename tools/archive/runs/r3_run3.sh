#!/bin/bash
# Round 3: C2 prefetch-depth variants (ENF_D2_P / ENF_D2_U / ENF_BLOCKS_PER_CU on the diagnostics library)
# and the headline kernel under the iterative-ILP LLVM scheduler (diagnostics library built with
# HJ_SCHED=iterative-ilp) against the product, interleaved. Stops at a failure.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r3c
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # tag, env, extra args
  local tag=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python tools/flow_time.py --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 50 "$@" > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$tag/run_kernel_stats.csv')):
    if 'flow_' in r['Name']: print('$tag', r['Name'][:52], r['Calls'], 'avg_us %.2f' % (float(r['AverageNs']) / 1e3), 'min_us %.2f' % (float(r['MinNs']) / 1e3))
"
}
run product ENF_NONE=0 --product
for v in p2:ENF_D2_P=2 p3:ENF_D2_P=3 p4:ENF_D2_P=4 p3_bpc3:ENF_D2_P=3,ENF_BLOCKS_PER_CU=3 u1p4_bpc4:ENF_D2_U=1,ENF_D2_P=4,ENF_BLOCKS_PER_CU=4 product2:ENF_NONE=0; do
  tag=${v%%:*}; kv=${v#*:}; kv=${kv//,/ }
  if [ "$tag" = product2 ]; then run $tag "$kv" --product; else run $tag "$kv"; fi
done
REPS=3 TAG=r3c/hjab VARIANTS="iterilp:ENF_HJ_VAR=0" bash tools/r3_hj_ab.sh
