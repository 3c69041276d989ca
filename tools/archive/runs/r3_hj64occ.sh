#!/bin/bash
# fp64 (J o H)^4 compiled program: register allocation capped for 4 waves per SIMD (diagnostics build,
# ENF_HJ64_OCC=4: 128 VGPRs, 7-8 spilled) against the product's 140 VGPRs / 3 waves. rocprofv3 kernel
# averages, interleaved passes. gpurun_out/hj64occ/.
set -u
OUT=gpurun_out/hj64occ
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # tag, env, args
  local tag=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python tools/flow_time.py --dtype f64 --pairs 4 --steps 30 "$@" > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$tag/run_kernel_stats.csv')):
    if 'flow_' in r['Name']: print('$tag', r['Name'][:60], r['Calls'], 'avg_ms %.4f' % (float(r['AverageNs']) / 1e6), 'min_ms %.4f' % (float(r['MinNs']) / 1e6))
" | tee -a $OUT/summary.txt
}
for pass in 1 2; do
  run d32_base$pass ENF_HJ64_OCC=1 --D 32 --N 10000000
  run d32_occ4_$pass ENF_HJ64_OCC=4 --D 32 --N 10000000
  run d64_base$pass ENF_HJ64_OCC=1 --D 64 --N 5000000
  run d64_occ4_$pass ENF_HJ64_OCC=4 --D 64 --N 5000000
done
