#!/bin/bash
# Round 2: accuracy + parity tests, then kernel-time A/B of the headline flow on the diagnostics
# library (accurate vs fast small-|z| asinh, compute-only DEBUG_MODE=2, synthesized loads =1), the
# shipping library, and the product bench. Stops at a crash / timeout.
set -u
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r2}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== pytest ${TESTS:-accuracy + parity}"
  timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    ${TESTS:-tests/test_gpu_fp32_accuracy.py tests/test_gpu_parity.py} > $OUT/${TAG}_pytest.txt 2>&1
  rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/${TAG}_pytest.txt | tail -30; ok $rc || { echo "pytest crashed rc=$rc"; exit $rc; }
fi
echo "== A/B flow time"
# variants "tag:KNOB=v,KNOB=v" (comma-separated knobs)
for v in ${VARIANTS:-merge: med3:ENF_HJ_ASINH=2 fast:ENF_HJ_ASINH=0 merge_compute:ENF_DEBUG_MODE=2 med3_compute:ENF_HJ_ASINH=2,ENF_DEBUG_MODE=2}; do
  tag=${v%%:*}; kv=${v#*:}; kv=${kv//,/ }
  env $kv timeout -k 10 120 python tools/flow_time.py --tag $tag ${FLOW_ARGS:-} >> $OUT/${TAG}_ab.jsonl 2>> $OUT/${TAG}_ab.err
  rc=$?; [ $rc -eq 0 ] || { echo "flow_time failed rc=$rc"; tail $OUT/${TAG}_ab.err; exit $rc; }
done
timeout -k 10 120 python tools/flow_time.py --product --tag product ${FLOW_ARGS:-} >> $OUT/${TAG}_ab.jsonl 2>> $OUT/${TAG}_ab.err || exit $?
cat $OUT/${TAG}_ab.jsonl
[ "${SKIP_BENCH:-0}" = "1" ] && exit 0
echo "== bench"
timeout -k 10 300 python bench.py ${BENCH_ARGS:---no-cpu} > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err
rc=$?; cat $OUT/${TAG}_bench.json; tail -3 $OUT/${TAG}_bench.err; exit $rc
