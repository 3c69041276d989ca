#!/bin/bash
# Config 2: the compiled D = 2 kernel with the parameter / table loads issued ahead of the first tiles, the
# uniform group loop and one-line dummy loads (diagnostics build) vs the shipping library's previous
# version (--product), interleaved, warm (repeated call) and cold (512 MB written before every call).
set -u
OUT=gpurun_out/c2pro
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # tag, env [flow_time args]
  local tag=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python tools/flow_time.py --D 2 --N ${N:-1000000} --pairs 1 --dtype f64 --steps 200 "$@" > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
  python3 -c "
import csv, json
for r in csv.DictReader(open('$OUT/$tag/run_kernel_stats.csv')):
    if 'flow_' in r['Name']: print('$tag', r['Name'][:60], r['Calls'], 'avg_us %.2f' % (float(r['AverageNs']) / 1e3), 'min_us %.2f' % (float(r['MinNs']) / 1e3), [json.loads(l)['out_sha1'] for l in open('$OUT/$tag.log') if l.startswith('{')][-1], flush=True)
"
}
for rep in 1 2 3; do
  run old_r$rep ENF_X=0 --product || exit 1
  run new_r$rep ENF_X=0 || exit 1
  run old_cold_r$rep ENF_X=0 --product --flush-mb 512 || exit 1
  run new_cold_r$rep ENF_X=0 --flush-mb 512 || exit 1
done
run new_memonly ENF_D2_DBG=3 || exit 1
run new_nt2 ENF_D2_NT=2 || exit 1
run new_grid0 ENF_D2_GRID=0 || exit 1
run new_grid0_b ENF_D2_GRID=0 || exit 1
run new_b ENF_X=0 || exit 1
for n in 200000 4000000; do
  N=$n run old_N$n ENF_X=0 --product || exit 1
  N=$n run new_N$n ENF_X=0 || exit 1
done
