#!/bin/bash
# Config 2 (J o H, D = 2, fp64, N = 1e6) kernel durations by rocprofv3: the shipping library (compiled
# D = 2 program, enf_flow_d2.hip) and diagnostics variants (ENF_NO_D2=1: the step-table interpreter;
# ENF_D2_U=1: one column per lane per tile; ENF_D2_DBG=2: no loads / stores). gpurun_out/c2ab/<tag>.
set -u
OUT=gpurun_out/c2ab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # tag, env, extra args
  local tag=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python tools/flow_time.py --D 2 --N ${N:-1000000} --pairs 1 --dtype f64 --steps 50 "$@" > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$tag/run_kernel_stats.csv')):
    if 'flow_' in r['Name']: print('$tag', r['Name'][:48], r['Calls'], 'avg_us %.2f' % (float(r['AverageNs']) / 1e3), 'min_us %.2f' % (float(r['MinNs']) / 1e3))
"
}
run product ENF_NONE=0 --product
run d2_u2 ENF_NONE=0
run d2_u1 ENF_D2_U=1
run d2_compute ENF_D2_DBG=2
run interp ENF_NO_D2=1
run interp_prologue "ENF_NO_D2=1 ENF_FRAG_DBG=4"
for b in ${BPCS:-}; do run d2_bpc$b ENF_BLOCKS_PER_CU=$b; done
