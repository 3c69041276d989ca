#!/bin/bash
# fused gradient tail (enf_grad_tail.h): training / VJP / round-3 GPU tests, then the config-5 step A/B
# (diagnostics library, ENF_GRAD_FUSED_TAIL=1 / 0, graph-captured fused step) and the product's bench_train.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s2e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_semantics.py tests/test_gpu_vjp.py tests/test_gpu_round3.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_train.txt 2>&1
rc=$?; tail -4 $O/pytest_train.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for V in ENF_GRAD_FUSED_TAIL=1 ENF_GRAD_FUSED_TAIL=0; do
    r=$(env $V timeout -k 5 120 python bench_train.py --diag 2>>$O/train_ab.err) || { echo "failed: $V"; tail -5 $O/train_ab.err; exit 1; }
    echo "[$V] $(echo "$r" | python -c 'import json,sys; d=json.load(sys.stdin); print("%.0f steps/s  %.2f us/step" % (d["value"], d["ms_per_step"] * 1e3))')"
  done
done | tee $O/train_ab.txt
timeout -k 5 120 python bench_train.py > $O/bench_train.json 2>> $O/train_ab.err || exit 1
cat $O/bench_train.json
# compiled (J o H)^n program on the padded layout and at D = 128 (round 3)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "hj_program or config3_pattern or padded" > $O/pytest_hjpad.txt 2>&1
rc=$?; tail -4 $O/pytest_hjpad.txt; [ $rc -eq 0 ] || exit $rc
for d in "24 13333333" "36 8888888" "100 3200000" "128 2500000"; do
  set -- $d
  timeout -k 10 120 python tools/flow_time.py --product --D $1 --N $2 --tag hjpad_D$1 >> $O/hjpad.jsonl 2>> $O/hjpad.err || { echo "flow_time D$1 failed"; tail -5 $O/hjpad.err; exit 1; }
done
cat $O/hjpad.jsonl
