#!/bin/bash
# round 6, GPU pass 21: the practical copy ceiling at small sizes (cold, graph-replayed) beside config 2's flow on the
# same box -- what a D = 2 fp64 flow of 40 MB can be held against
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 200 python tools/copy_sizes.py --sizes-mb 20,40,80,320,1280 > gpurun_out/r6/copy_sizes_v1.jsonl || exit 1
cat gpurun_out/r6/copy_sizes_v1.jsonl
for pat in HJ S; do
  $T 200 python bench.py --no-cpu --no-train --no-pmc --pattern $pat --D 2 --N 1000000 --dtype f64 --cache both --steps 50 --warmup 5 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"f64_D2_$pat\"}\t/" >> gpurun_out/r6/c2_beside_copy_v1.jsonl || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/r6/c2_beside_copy_v1.jsonl'):
    t,j=l.split('\t',1); r=json.loads(j)
    print(t, r['roofline']['kernel_ms']*1e3, 'us', round(r['roofline']['frac'],3), (r.get('warm') or {}).get('kernel_ms'))
"
