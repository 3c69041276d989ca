#!/bin/bash
# Config 2 after the switch to 3 blocks per CU: the C2 GPU tests, then the product kernel's rocprofv3 time warm
# (twice) and cold (512 MB written between calls). gpurun_out/c2bpc3/.
set -u
OUT=gpurun_out/c2bpc3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_gpu_c2.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_c2.txt 2>&1 || { tail -20 $OUT/pytest_c2.txt; exit 1; }
tail -2 $OUT/pytest_c2.txt
run() {
  local tag=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python tools/flow_time.py --product --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 300 "$@" > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$tag/run_kernel_stats.csv')):
    if 'flow_' in r['Name']: print('$tag', r['Name'][:48], r['Calls'], 'avg_us %.2f' % (float(r['AverageNs']) / 1e3), 'min_us %.2f' % (float(r['MinNs']) / 1e3))
" | tee -a $OUT/summary.txt
}
run warm1
run cold1 --flush-mb 512
run warm2
run cold2 --flush-mb 512
