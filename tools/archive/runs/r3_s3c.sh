#!/bin/bash
# Round-3 third-session evidence: the box's CPU quota, GPU suite (-x, unserialised), smoke, bench (in-run PMC,
# CPU baseline sized by the cgroup quota, config-5 train object).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/s3c
mkdir -p $OUT
export TMPDIR=/tmp
{ echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; echo "nproc: $(nproc)"; echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-}"; } | tee $OUT/host.txt
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.txt; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
rc=$?; tail -1 $OUT/smoke.txt; [ $rc -eq 0 ] || exit $rc
echo "== bench"
s=$(date +%s)
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc wall $(( $(date +%s) - s )) s"; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']
print('value %.4g frac %.4f kernel_ms %.4f rocprof %s' % (d['value'], r['frac'], r['kernel_ms'], r['rocprof_kernel_stats']['average_ms'] if r['rocprof_kernel_stats'] else None))
print('traffic', r['traffic'], r['traffic_source']); c=d['cpu_baseline']; print('cpu', c['value'], c['cores'], c['single_thread']['value'], c['host'])
print('train', d['train'].get('value'), d['train'].get('ms_per_step'))"
