#!/bin/bash
# round 6, GPU pass 20: VERDICT r05 item 7 -- the table-driven fp64 exp / expm1 (enf_math64.h exp64_tab /
# expm1_64_tab) in the fp64 Center forward forms: D = 2 fp64 N = 1e6 example-flow patterns, cold and warm,
# product vs the ENF_EXP_TAB=1 build (tools/ab/libenf_exptab.so, copied over libenf.so for its legs; the box is
# scratch), interleaved; then the fp64 parity tests on the variant
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=euclidiannormalizingflows.jl_amd/libenf.so
cp $L gpurun_out/r6/libenf_product.so.bak
P=gpurun_out/r6/exptab_patterns_v1.jsonl
for i in 1 2; do
  for v in product exptab; do
    if [ $v = exptab ]; then cp tools/ab/libenf_exptab.so $L; else cp gpurun_out/r6/libenf_product.so.bak $L; fi
    for pat in C K CJ KHS SHC JKJK; do
      $T 200 python bench.py --no-cpu --no-train --no-pmc --pattern $pat --D 2 --N 1000000 --dtype f64 --cache both --steps 50 --warmup 5 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"${v}_f64_D2_$pat\"}\t/" >> $P || exit 1
    done
  done
done
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$P'):
    t,j=l.split('\t',1); r=json.loads(j)
    d[json.loads(t)['tag']].append('%.3f/%.3f'%(r['roofline']['frac'], (r.get('warm') or {}).get('frac',0)))
for k,v in sorted(d.items()): print(k, v)
"
cp tools/ab/libenf_exptab.so $L
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_round4.py tests/test_gpu_round3.py \
  tests/test_gpu_c2.py > gpurun_out/r6/pytest_run20_exptab.txt 2>&1 || { tail -30 gpurun_out/r6/pytest_run20_exptab.txt; exit 1; }
tail -1 gpurun_out/r6/pytest_run20_exptab.txt
cp gpurun_out/r6/libenf_product.so.bak $L
rm -f gpurun_out/r6/libenf_product.so.bak
