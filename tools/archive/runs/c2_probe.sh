#!/bin/bash
# C2 (J o H, D = 2, fp64) latency decomposition: rocprofv3 kernel durations of the shipping kernel
# at several N and of the diagnostics variants (ENF_FRAG_DBG: 1 synthesized tile, 2 also no stores,
# 4 prologue only). Writes gpurun_out/c2_<tag>.csv summaries.
set -u
OUT=gpurun_out/c2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # tag, env, args
  local tag=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python tools/flow_time.py "$@" > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
  f=$(find $OUT/$tag -name '*kernel_stats.csv' | head -1)
  echo "== $tag"; grep -i "flow_frag\|flow_hj" $f | cut -d, -f1-5 | cut -c1-60,200-400
}
for N in ${NS:-100000 1000000 16000000}; do
  run prod_N$N ENF_NONE=0 --D 2 --N $N --pairs 1 --dtype f64 --steps 50 --product
done
for v in ${DBGS:-}; do
  run dbg$v ENF_FRAG_DBG=$v --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 50
done
for b in ${BPCS:-}; do
  run bpc$b ENF_BLOCKS_PER_CU=$b --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 50
done
for u in ${US:-2 1}; do
  run u$u ENF_FRAG_HJU=$u --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 50
done
for d in $OUT/*/; do
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$d/run_kernel_stats.csv')):
    if 'flow_' in r['Name']: print('$(basename $d)', r['Calls'], 'avg_us %.2f'%(float(r['AverageNs'])/1e3), 'min_us %.2f'%(float(r['MinNs'])/1e3))
"
done
