#!/bin/bash
# fp64 compiled (J o H)^n program on the padded layout and at D = 128: tests, then timings (product library)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s2f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_round3.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "hj64 or hj_program or config3_pattern or padded" > $O/pytest.txt 2>&1
rc=$?; tail -4 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for d in "24 6666666" "32 5000000" "100 1600000" "128 1250000"; do
  set -- $d
  timeout -k 10 120 python tools/flow_time.py --product --dtype f64 --D $1 --N $2 --tag hj64_D$1 >> $O/hj64.jsonl 2>> $O/hj64.err || { echo "flow_time D$1 failed"; tail -5 $O/hj64.err; exit 1; }
done
cat $O/hj64.jsonl
