#!/bin/bash
# Round 3: C2 per-block-prologue variants against the product (P = 4), and the instruction-mix probe with
# larger transcendental groups. Stops at a failure.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r3d
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # tag, env, extra args
  local tag=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python tools/flow_time.py --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 50 "$@" > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$tag/run_kernel_stats.csv')):
    if 'flow_' in r['Name']: print('$tag', r['Name'][:56], r['Calls'], 'avg_us %.2f' % (float(r['AverageNs']) / 1e3), 'min_us %.2f' % (float(r['MinNs']) / 1e3))
"
}
for rep in 1 2; do
  run product$rep ENF_NONE=0 --product
  for v in p2:ENF_D2_P=2 p4pb:ENF_D2_P=4,ENF_D2_PB=1 p2pb:ENF_D2_P=2,ENF_D2_PB=1; do
    tag=${v%%:*}$rep; kv=${v#*:}; kv=${kv//,/ }
    run $tag "$kv"
  done
done
run compute_pb ENF_D2_DBG=2,ENF_D2_PB=1
run compute ENF_D2_DBG=2
timeout -k 5 60 ./tools/microbench16 4 > $OUT/mb16.txt 2>&1; rc=$?; cat $OUT/mb16.txt; exit $rc
