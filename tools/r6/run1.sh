#!/bin/bash
# round 6, GPU pass 1: the folded (J o H)^n program (enf_hj.h) -- the whole GPU suite, then an interleaved A/B
# of the headline flow (config 3) and the config-4 shard against the round-5 library (tools/ab/libenf_r5.so)
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests \
  > gpurun_out/r6/pytest_run1.txt 2>&1 || { tail -30 gpurun_out/r6/pytest_run1.txt; exit 1; }
tail -2 gpurun_out/r6/pytest_run1.txt
P=gpurun_out/r6/fold_ab_v1.jsonl
for i in 1 2 3; do
  $T 120 python tools/flow_time.py --lib tools/ab/libenf_r5.so --D 32 --N 10000000 --pairs 4 --steps 100 --tag r5 >> $P || exit 1
  $T 120 python tools/flow_time.py --product --D 32 --N 10000000 --pairs 4 --steps 100 --tag r6 >> $P || exit 1
done
for i in 1 2; do
  $T 120 python tools/flow_time.py --lib tools/ab/libenf_r5.so --D 64 --N 12500000 --pairs 4 --steps 50 --tag r5 >> $P || exit 1
  $T 120 python tools/flow_time.py --product --D 64 --N 12500000 --pairs 4 --steps 50 --tag r6 >> $P || exit 1
  $T 120 python tools/flow_time.py --lib tools/ab/libenf_r5.so --D 32 --N 10000000 --pattern IHIHIHIH --steps 50 --tag r5_inv >> $P || exit 1
  $T 120 python tools/flow_time.py --product --D 32 --N 10000000 --pattern IHIHIHIH --steps 50 --tag r6_inv >> $P || exit 1
done
cat $P
echo ALLDONE
