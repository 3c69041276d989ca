#!/bin/bash
# Headline kernel: s_setprio around the transcendental groups (diagnostics build, ENF_HJ_VAR=4: priority 3 while
# a wave issues its sqrt / log2 group; 8: priority lowered there instead) against the shipped schedule,
# streaming and compute-only (ENF_DEBUG_MODE=2), interleaved passes; flow_time.py lines (HIP events).
set -u
OUT=gpurun_out/prio
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for pass in 1 2 3; do
  for v in 0 4 8; do
    ENF_HJ_VAR=$v timeout -k 10 120 python tools/flow_time.py --steps 40 --tag var${v}_$pass >> $OUT/ab.jsonl 2>> $OUT/err.txt || { tail -3 $OUT/err.txt; exit 1; }
    ENF_HJ_VAR=$v ENF_DEBUG_MODE=2 timeout -k 10 120 python tools/flow_time.py --steps 40 --tag var${v}_compute_$pass >> $OUT/ab.jsonl 2>> $OUT/err.txt || { tail -3 $OUT/err.txt; exit 1; }
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print(d['tag'], d['knobs'], '%.4f ms' % d['kernel_ms'], 'frac %.4f' % d['hbm_frac'])"
