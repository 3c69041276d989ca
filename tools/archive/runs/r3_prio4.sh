#!/bin/bash
# Where the raised priority pays: around both transcendental groups (shipped, ENF_HJ_VAR=0), only the sqrt group
# (16), only the log2 group (32), both groups and the ladj log2 (64), none (4); diagnostics build compiled the
# product's way (iterative-ILP), interleaved passes, HIP-event kernel time (flow_time.py). gpurun_out/prio4/.
set -u
OUT=gpurun_out/prio4
mkdir -p $OUT
export TMPDIR=/tmp
for pass in 1 2 3; do
  for v in 0 128 192 64; do
    ENF_HJ_VAR=$v timeout -k 10 120 python tools/flow_time.py --steps 40 --tag var${v}_$pass >> $OUT/ab.jsonl 2>> $OUT/err.txt || { tail -3 $OUT/err.txt; exit 1; }
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print(d['tag'], '%.4f ms' % d['kernel_ms'], 'frac %.4f' % d['hbm_frac'])"
