#!/bin/bash
# Round 3, second GPU session: the new fp64 paths' tests, C2 and fp64-C3 kernel times (rocprofv3), and the
# headline-kernel A/B. Stops at the first crash / time limit.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r3b
mkdir -p $OUT
export TMPDIR=/tmp
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
echo "== pytest (round-3 + C2 modules)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_round3.py tests/test_gpu_c2.py -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?; tail -6 $OUT/pytest.txt; ok $rc || { echo "pytest crashed rc=$rc"; exit $rc; }
prof() {  # tag, flow_time args
  local tag=$1; shift
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python tools/flow_time.py --product "$@" > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$tag/run_kernel_stats.csv')):
    if 'flow_' in r['Name']: print('$tag', r['Name'][:60], r['Calls'], 'avg_us %.2f' % (float(r['AverageNs']) / 1e3), 'min_us %.2f' % (float(r['MinNs']) / 1e3))
"
  grep '^{' $OUT/$tag.log | tail -1
}
echo "== C2 and fp64 C3 kernel times"
prof c2 --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 50
prof c3f64 --D 32 --N 10000000 --pairs 4 --dtype f64 --steps 10
prof c4f64 --D 64 --N 5000000 --pairs 4 --dtype f64 --steps 10
echo "== headline A/B"
REPS=2 TAG=r3b/hjab bash tools/r3_hj_ab.sh
