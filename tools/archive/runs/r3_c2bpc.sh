#!/bin/bash
# Config 2 (J o H, D = 2, fp64, N = 1e6): kernel time against resident blocks per CU (diagnostics build,
# ENF_BLOCKS_PER_CU) for U = 2 and U = 1 columns per lane per tile, product library beside it, warm and
# cold (512 MB written between calls). rocprofv3 kernel averages; gpurun_out/c2bpc/<tag>.
set -u
OUT=gpurun_out/c2bpc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # tag, env, extra args
  local tag=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python tools/flow_time.py --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 300 "$@" > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$tag/run_kernel_stats.csv')):
    if 'flow_' in r['Name']: print('$tag', r['Name'][:48], r['Calls'], 'avg_us %.2f' % (float(r['AverageNs']) / 1e3), 'min_us %.2f' % (float(r['MinNs']) / 1e3))
" | tee -a $OUT/summary.txt
}
for pass in 1 2; do
run product$pass ENF_NONE=0 --product
for b in 2 3 4 5; do run u2_bpc${b}_$pass ENF_BLOCKS_PER_CU=$b; done
for b in 4 6 8; do run u1_bpc${b}_$pass "ENF_D2_U=1 ENF_BLOCKS_PER_CU=$b"; done
done
run product_cold ENF_NONE=0 --product --flush-mb 512
for b in 2 3 4; do run u2_bpc${b}_cold ENF_BLOCKS_PER_CU=$b --flush-mb 512; done
run u1_bpc6_cold "ENF_D2_U=1 ENF_BLOCKS_PER_CU=6" --flush-mb 512
