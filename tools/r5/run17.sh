#!/bin/bash
# round 5, seventeenth GPU pass: refreshed single-layer / example-flow numbers on the round-5 build -- D = 32 fp32
# N = 1e7 (cold by size) and D = 2 fp64 N = 1e6 (cold and warm legs), the fp64 C3 program and its inverse, the
# D = 64 config-4 shard; one JSON line each
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5/patterns_v2.jsonl
for pat in S C K J I H4 CJ JKJK SHC KHS; do
  $T 200 python bench.py --no-cpu --no-train --no-pmc --pattern $pat --steps 20 --warmup 3 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"f32_D32_$pat\"}\t/" >> $P || exit 1
done
for pat in HJ S C K J CJ JKJK SHC KHS; do
  $T 200 python bench.py --no-cpu --no-train --no-pmc --pattern $pat --D 2 --N 1000000 --dtype f64 --cache both --steps 50 --warmup 5 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"f64_D2_$pat\"}\t/" >> $P || exit 1
done
$T 300 python bench.py --no-cpu --no-train --no-pmc --dtype f64 --steps 20 --warmup 3 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"f64_C3\"}\t/" >> $P || exit 1
$T 300 python bench.py --no-cpu --no-train --no-pmc --dtype f64 --inverse --steps 20 --warmup 3 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"f64_C3_inverse\"}\t/" >> $P || exit 1
$T 300 python bench.py --no-cpu --no-train --no-pmc --inverse --steps 20 --warmup 3 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"f32_C3_inverse\"}\t/" >> $P || exit 1
$T 300 python bench.py --no-cpu --no-train --no-pmc --D 64 --N 12500000 --steps 20 --warmup 3 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"f32_C4_shard\"}\t/" >> $P || exit 1
echo ALLDONE
