#!/bin/bash
# round 6, GPU pass 11: (1) the folded inverse program -- its parity tests (inverse vs oracle, round trips, edge values)
# and an interleaved A/B against round 5 on the forward's outputs (bench.py --inverse's workload); (2) the gradient
# kernel's shape at the 8-rank share now that the all-reduce carries its rows (diagnostics ENF_HJG_VARIANT 0/5/4/3)
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_round4.py tests/test_gpu_parity.py \
  tests/test_gpu_round3.py > gpurun_out/r6/pytest_run11.txt 2>&1 || { tail -30 gpurun_out/r6/pytest_run11.txt; exit 1; }
tail -1 gpurun_out/r6/pytest_run11.txt
P=gpurun_out/r6/inv_ab_v1.jsonl
for i in 1 2 3; do
  $T 120 python tools/flow_time.py --lib tools/ab/libenf_r5.so --inverse --D 32 --N 10000000 --pairs 4 --steps 100 --tag r5_inv >> $P || exit 1
  $T 120 python tools/flow_time.py --product --inverse --D 32 --N 10000000 --pairs 4 --steps 100 --tag r6_inv >> $P || exit 1
done
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$P'):
    r=json.loads(l); d[r['tag']].append((r['kernel_ms'], r['hbm_frac']))
for k,v in sorted(d.items()): print(k, ['%.4f/%.3f'%x for x in v])
"
P=gpurun_out/r6/c5_share_variants_v1.jsonl
for i in 1 2; do
  for v in 0 5 4 3; do
    ENF_HJG_VARIANT=$v $T 200 python bench_train.py --diag --steps 100 --emulate-world 8 > gpurun_out/r6/v.json 2> gpurun_out/r6/v.err || { tail -5 gpurun_out/r6/v.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r6/v.json').read().strip().splitlines()[-1]); print(json.dumps({'variant': $v, 'ms_per_step': d['ms_per_step']}))" >> $P
  done
done
cat $P
