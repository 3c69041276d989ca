#!/bin/bash
# round 6, GPU pass 5: (1) the duplicated epilogue A/B (round 5 / first fold / current, interleaved, configs 3 and 4),
# (2) the round-6 tests (the similar_fill quirk as default through ENF_NEGLL_ZYGOTE, ties, cross-lane primitives,
# workspace, elementwise report), (3) the whole GPU suite
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
$T 600 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_round6.py \
  > gpurun_out/r6/pytest_run5_round6.txt 2>&1 || { tail -40 gpurun_out/r6/pytest_run5_round6.txt; exit 1; }
grep -E "elementwise|golden|PASS|FAIL" gpurun_out/r6/pytest_run5_round6.txt | tail -40
$T 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests \
  > gpurun_out/r6/pytest_run5_full.txt 2>&1 || { tail -40 gpurun_out/r6/pytest_run5_full.txt; exit 1; }
tail -3 gpurun_out/r6/pytest_run5_full.txt
echo ALLDONE
