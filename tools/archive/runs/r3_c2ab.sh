#!/bin/bash
# Round 3: C2 (J o H, D=2, fp64, N=1e6) kernel durations by rocprofv3 for blocks-per-CU / columns-per-lane
# variants of the compiled D=2 program on the diagnostics library, and the product. Stops at a failure.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r3c2
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # tag, env, extra args
  local tag=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python tools/flow_time.py --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 50 "$@" > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$tag/run_kernel_stats.csv')):
    if 'flow_' in r['Name']: print('$tag', r['Name'][:48], r['Calls'], 'avg_us %.2f' % (float(r['AverageNs']) / 1e3), 'min_us %.2f' % (float(r['MinNs']) / 1e3))
"
}
run product ENF_NONE=0 --product
for v in u2_bpc2:ENF_D2_U=2,ENF_BLOCKS_PER_CU=2 u2_bpc3:ENF_D2_U=2,ENF_BLOCKS_PER_CU=3 u2_bpc4:ENF_D2_U=2,ENF_BLOCKS_PER_CU=4 u1_bpc4:ENF_D2_U=1,ENF_BLOCKS_PER_CU=4 u1_bpc6:ENF_D2_U=1,ENF_BLOCKS_PER_CU=6 u1_bpc8:ENF_D2_U=1,ENF_BLOCKS_PER_CU=8 compute:ENF_D2_DBG=2; do
  tag=${v%%:*}; kv=${v#*:}; kv=${kv//,/ }
  run $tag "$kv"
done
