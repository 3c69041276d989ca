#!/bin/bash
# round 5, fourth GPU pass: where the reduction's ~5 us go (launch-floor probes, device kernargs), the D = 2 legs'
# kernel times cold vs warm under rocprofv3, the examples' training legs, and the new oracle-reverse-pass tests
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_round5.py \
  > gpurun_out/r5/pytest_run4.txt 2>&1 || { tail -30 gpurun_out/r5/pytest_run4.txt; exit 1; }
tail -2 gpurun_out/r5/pytest_run4.txt
$T 300 python bench_train.py --example 1d > gpurun_out/r5/example_1d.json 2> gpurun_out/r5/example.err || exit 1
$T 300 python bench_train.py --example 2d > gpurun_out/r5/example_2d.json 2>> gpurun_out/r5/example.err || exit 1
echo EXAMPLES_DONE
for dbg in 1 2; do
  ENF_RED_DBG=$dbg $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof4_reddbg$dbg -o c5 -- python3 bench_train.py --diag --steps 100 --warmup 10 --emulate-world 8 --graph 0 > /dev/null 2>&1 || exit 1
done
for k in 0 1; do
  HIP_FORCE_DEV_KERNARG=$k $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof4_kernarg$k -o c5 -- python3 bench_train.py --steps 100 --warmup 10 --emulate-world 8 --graph 0 > /dev/null 2>&1 || exit 1
  HIP_FORCE_DEV_KERNARG=$k $T 120 python bench_train.py --steps 200 --warmup 20 --emulate-world 8 2>/dev/null | tail -1 > gpurun_out/r5/kernarg${k}_share8.json || exit 1
done
echo PROBES_DONE
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof4_d2 -o d2 -- python3 bench.py --pattern HJ --D 2 --N 1000000 --dtype f64 --no-cpu --no-train --no-pmc --steps 50 --warmup 5 > gpurun_out/r5/d2_hj_prof.json 2>/dev/null || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof4_d2cj -o d2 -- python3 bench.py --pattern JC --D 2 --N 1000000 --dtype f64 --no-cpu --no-train --no-pmc --steps 50 --warmup 5 > gpurun_out/r5/d2_jc_prof.json 2>/dev/null || exit 1
echo ALLDONE
