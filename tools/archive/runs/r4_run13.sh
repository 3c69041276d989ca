#!/bin/bash
# round 4, thirteenth GPU pass: the fp64 forward program on a B = 6 log table (one FMA fewer per log, more LDS
# bank conflicts) against the product's B = 5, interleaved on the diagnostics library (ENF_HJ64_TB), plus the
# B = 6 functions' ulps
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 120 ./tools/asinh64_tab_check > gpurun_out/r4_asinh64_tab_check_13.txt 2>&1 || exit 1
cat gpurun_out/r4_asinh64_tab_check_13.txt
P=gpurun_out/r4_hj64_tb_ab_13.jsonl
for pass in 1 2 3; do
  for tb in 5 6; do
    ENF_HJ64_TB=$tb $T 200 python tools/flow_time.py --dtype f64 --steps 30 --tag tb$tb >> $P 2>> gpurun_out/r4_hj64_tb_ab_13.err || exit 1
  done
done
for tb in 5 6; do
  ENF_HJ64_TB=$tb $T 200 python tools/flow_time.py --dtype f64 --D 64 --N 5000000 --steps 30 --tag tb${tb}_d64 >> $P 2>> gpurun_out/r4_hj64_tb_ab_13.err || exit 1
done
echo ALLDONE
