#!/bin/bash
# bench.py after the PMC time budget (in-run PMC still collected), then the occupancy-5 slab variant with the
# wave-priority schedule (ENF_HJ_VAR=1) against the shipped kernel (tools/r3_prio5.sh).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/s3g
export TMPDIR=/tmp
s=$(date +%s)
timeout -k 10 900 python bench.py > gpurun_out/s3g/bench.json 2> gpurun_out/s3g/bench.err
rc=$?; echo "bench rc=$rc wall $(( $(date +%s) - s )) s"; [ $rc -eq 0 ] || { tail -5 gpurun_out/s3g/bench.err; exit $rc; }
python3 -c "
import json; d=json.load(open('gpurun_out/s3g/bench.json')); r=d['roofline']
print('value %.4g frac %.4f kernel_ms %.4f traffic %s src %s' % (d['value'], r['frac'], r['kernel_ms'], r['traffic'], r['traffic_source'][:20]))"
bash tools/r3_prio5.sh
