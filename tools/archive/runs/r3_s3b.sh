#!/bin/bash
# bench.py with its in-run rocprofv3 PMC and kernel-stats passes (one GPU), timed end to end.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/s3b
mkdir -p $OUT
export TMPDIR=/tmp
s=$(date +%s)
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc wall $(( $(date +%s) - s )) s"; cut -c1-300 $OUT/bench.json; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']
print('frac', r['frac'], 'kernel_ms', r['kernel_ms'], 'traffic', r['traffic'], r['traffic_source']); print('rocprof', r['rocprof_kernel_stats']); print('valu', d['valu'])"
