#!/bin/bash
# Config 2: load order A/B (diagnostics build, ENF_D2_LO=1: only the first tile's load ahead of the wave
# prologue, the other tiles after it) against the shipped order (all P tiles ahead), warm and cold,
# interleaved passes. gpurun_out/c2lo/.
set -u
OUT=gpurun_out/c2lo
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {
  local tag=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python tools/flow_time.py --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 300 "$@" > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$tag/run_kernel_stats.csv')):
    if 'flow_' in r['Name']: print('$tag', r['Name'][:56], r['Calls'], 'avg_us %.2f' % (float(r['AverageNs']) / 1e3), 'min_us %.2f' % (float(r['MinNs']) / 1e3))
" | tee -a $OUT/summary.txt
}
for pass in 1 2; do
  run base_$pass ENF_D2_LO=0
  run lo1_p4_$pass ENF_D2_LO=1
  run lo1_p3_$pass "ENF_D2_LO=1 ENF_D2_P=3"
  run base_cold_$pass ENF_D2_LO=0 --flush-mb 512
  run lo1_p4_cold_$pass ENF_D2_LO=1 --flush-mb 512
done
