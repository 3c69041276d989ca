#!/bin/bash
# round 6, GPU pass 7: the per-column ballot redo test and the LM-1 store trim (product) against round 5, interleaved;
# one dot chain per column (diagnostics ENF_HJ_VAR=3) against two; VALU count of the product kernel (PMC); the
# hj-program parity / accuracy tests
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_fp32_accuracy.py tests/test_gpu_round4.py > gpurun_out/r6/pytest_run7.txt 2>&1 || { tail -30 gpurun_out/r6/pytest_run7.txt; exit 1; }
tail -1 gpurun_out/r6/pytest_run7.txt
P=gpurun_out/r6/ballot_ab_v1.jsonl
for i in 1 2 3; do
  $T 120 python tools/flow_time.py --lib tools/ab/libenf_r5.so --D 32 --N 10000000 --pairs 4 --steps 100 --tag r5 >> $P || exit 1
  $T 120 python tools/flow_time.py --product --D 32 --N 10000000 --pairs 4 --steps 100 --tag r6b >> $P || exit 1
  ENF_HJ_VAR=0 $T 120 python tools/flow_time.py --D 32 --N 10000000 --pairs 4 --steps 100 --tag diag_var0 >> $P || exit 1
  ENF_HJ_VAR=3 $T 120 python tools/flow_time.py --D 32 --N 10000000 --pairs 4 --steps 100 --tag diag_var3 >> $P || exit 1
done
python -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$P'):
    r=json.loads(l); d[(r['tag'],r['D'])].append(r['kernel_ms'])
for k,v in sorted(d.items()): print(k, ['%.4f'%x for x in v])
"
for m in prod var3; do
  if [ $m = prod ]; then A="--product"; V=0; else A=""; V=3; fi
  ENF_HJ_VAR=$V timeout -k 10 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES \
    --output-format csv -d gpurun_out/r6/pmc7_$m -o run -- python3 tools/flow_time.py $A --D 32 --N 10000000 --pairs 4 \
    --steps 30 --tag pmc > gpurun_out/r6/pmc7_$m.log 2>&1 || { tail -5 gpurun_out/r6/pmc7_$m.log; exit 1; }
done
python3 tools/r6/clk_summary.py gpurun_out/r6/pmc7_prod gpurun_out/r6/pmc7_var3
