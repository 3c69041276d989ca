#!/bin/bash
# Round 2, step 1: fp32 accuracy tests + parity suite, then A/B kernel time of the accurate vs the
# fast small-|z| asinh (diagnostics library), then the product bench. Stops at a crash / timeout
# (exit codes other than 0 = pass and 1 = test failures).
set -u
OUT=gpurun_out
mkdir -p $OUT
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
echo "== pytest accuracy + parity"
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fp32_accuracy.py tests/test_gpu_parity.py ${PYTEST_ARGS:-} > $OUT/r2_pytest_acc.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/r2_pytest_acc.txt | tail -30; ok $rc || { echo "pytest crashed rc=$rc"; exit $rc; }
echo "== A/B flow time"
for v in "acc:" "fast:ENF_HJ_ASINH=0"; do
  tag=${v%%:*}; kv=${v#*:}
  env $kv timeout -k 10 120 python tools/flow_time.py --tag $tag >> $OUT/r2_ab_asinh.jsonl 2>> $OUT/r2_ab.err
  rc=$?; [ $rc -eq 0 ] || { echo "flow_time failed rc=$rc"; tail $OUT/r2_ab.err; exit $rc; }
done
timeout -k 10 120 python tools/flow_time.py --product --tag product >> $OUT/r2_ab_asinh.jsonl 2>> $OUT/r2_ab.err || exit $?
cat $OUT/r2_ab_asinh.jsonl
echo "== bench"
timeout -k 10 300 python bench.py --no-cpu > $OUT/r2_bench_acc.json 2> $OUT/r2_bench_acc.err
rc=$?; cat $OUT/r2_bench_acc.json; tail -3 $OUT/r2_bench_acc.err; exit $rc
