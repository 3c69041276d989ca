#!/bin/bash
# round 6, GPU pass 4: the epilogue written out in both branches of the redo test (no vmcnt(0) at the join on
# every tile) against the first folded build (tools/ab/libenf_fold1.so) and round 5's, interleaved, config 3 / 4
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6/epi_ab_v1.jsonl
for i in 1 2 3; do
  $T 120 python tools/flow_time.py --lib tools/ab/libenf_r5.so --D 32 --N 10000000 --pairs 4 --steps 100 --tag r5 >> $P || exit 1
  $T 120 python tools/flow_time.py --lib tools/ab/libenf_fold1.so --D 32 --N 10000000 --pairs 4 --steps 100 --tag fold1 >> $P || exit 1
  $T 120 python tools/flow_time.py --product --D 32 --N 10000000 --pairs 4 --steps 100 --tag epi2 >> $P || exit 1
done
$T 120 python tools/flow_time.py --lib tools/ab/libenf_fold1.so --D 64 --N 12500000 --pairs 4 --steps 50 --tag fold1 >> $P || exit 1
$T 120 python tools/flow_time.py --product --D 64 --N 12500000 --pairs 4 --steps 50 --tag epi2 >> $P || exit 1
python -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$P'):
    r=json.loads(l); d[(r['tag'],r['D'])].append(r['kernel_ms'])
for k,v in sorted(d.items()): print(k, ['%.4f'%x for x in v])
"
