#!/bin/bash
# The s_setprio schedule in the product: GPU suite, then an interleaved A/B on the same box -- product libenf.so
# (priority 3 around the transcendental groups) against the diagnostics build compiled the product's way
# (iterative-ILP scheduler) with ENF_HJ_VAR=4 (the previous schedule) -- then bench.py (in-run PMC).
set -u
OUT=gpurun_out/prio2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.txt; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
for pass in 1 2 3; do
  timeout -k 10 120 python tools/flow_time.py --product --steps 40 --tag product_prio_$pass >> $OUT/ab.jsonl 2>> $OUT/err.txt || { tail -3 $OUT/err.txt; exit 1; }
  ENF_HJ_VAR=4 timeout -k 10 120 python tools/flow_time.py --steps 40 --tag ilp_noprio_$pass >> $OUT/ab.jsonl 2>> $OUT/err.txt || { tail -3 $OUT/err.txt; exit 1; }
  ENF_HJ_VAR=0 timeout -k 10 120 python tools/flow_time.py --steps 40 --tag ilp_prio_diag_$pass >> $OUT/ab.jsonl 2>> $OUT/err.txt || { tail -3 $OUT/err.txt; exit 1; }
  timeout -k 10 120 python tools/flow_time.py --product --D 64 --N 5000000 --steps 40 --tag product_prio_d64_$pass >> $OUT/ab.jsonl 2>> $OUT/err.txt || { tail -3 $OUT/err.txt; exit 1; }
  ENF_HJ_VAR=4 timeout -k 10 120 python tools/flow_time.py --D 64 --N 5000000 --steps 40 --tag ilp_noprio_d64_$pass >> $OUT/ab.jsonl 2>> $OUT/err.txt || { tail -3 $OUT/err.txt; exit 1; }
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print(d['tag'], '%.4f ms' % d['kernel_ms'], 'frac %.4f' % d['hbm_frac'])"
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']
print('value %.4g frac %.4f kernel_ms %.4f rocprof %s' % (d['value'], r['frac'], r['kernel_ms'], r['rocprof_kernel_stats']))
print('valu', d['valu']); print('train', d['train'].get('value'))"
