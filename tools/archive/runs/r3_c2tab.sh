#!/bin/bash
# Config 2: log table index bits of the compiled D = 2 kernel (ENF_D2_TABB 5 / 7 / 8, diagnostics build):
# rocprofv3 kernel averages, interleaved A/B/C rounds. gpurun_out/c2tab/.
set -u
OUT=gpurun_out/c2tab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # tag, env
  local tag=$1; shift
  env $1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python tools/flow_time.py --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 200 > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$tag/run_kernel_stats.csv')):
    if 'flow_' in r['Name']: print('$tag', r['Name'][:60], r['Calls'], 'avg_us %.2f' % (float(r['AverageNs']) / 1e3), 'min_us %.2f' % (float(r['MinNs']) / 1e3), flush=True)
"
}
for rep in 1 2 3; do
  for b in 5 7 8; do run tab${b}_r$rep ENF_D2_TABB=$b || exit 1; done
done
run compute_tab5 ENF_D2_DBG=2 || exit 1
run compute_tab8 "ENF_D2_DBG=2 ENF_D2_TABB=8" || exit 1
