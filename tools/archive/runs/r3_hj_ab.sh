#!/bin/bash
# Round 3: interleaved A/B of headline-kernel variants on the diagnostics library (tools/flow_time.py;
# ENF_HJ_VAR, ENF_DEBUG_MODE knobs, enf_flow_hj.hip) plus the product library, REPS rounds so clock
# drift averages out. VARIANTS="tag:KNOB=v,KNOB=v ..." Stops at a crash / time limit.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r3ab}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-base:ENF_HJ_VAR=0 slab5:ENF_HJ_VAR=1 nolds:ENF_HJ_VAR=2 slab5_nolds:ENF_HJ_VAR=3 base_compute:ENF_DEBUG_MODE=2 slab5_compute:ENF_DEBUG_MODE=2,ENF_HJ_VAR=1}; do
    tag=${v%%:*}; kv=${v#*:}; kv=${kv//,/ }
    env $kv timeout -k 10 120 python tools/flow_time.py --tag $tag ${FLOW_ARGS:-} >> $OUT/ab.jsonl 2>> $OUT/ab.err
    rc=$?; [ $rc -eq 0 ] || { echo "flow_time $tag failed rc=$rc"; tail -5 $OUT/ab.err; exit $rc; }
  done
  timeout -k 10 120 python tools/flow_time.py --product --tag product ${FLOW_ARGS:-} >> $OUT/ab.jsonl 2>> $OUT/ab.err || exit $?
done
python - <<PY
import json, collections
d = collections.defaultdict(list)
for l in open("$OUT/ab.jsonl"):
    r = json.loads(l); d[r["tag"]].append(r["kernel_ms"])
for k, v in d.items(): print(f"{k:16s} ms {' '.join(f'{x:.4f}' for x in v)}  min {min(v):.4f}")
PY
