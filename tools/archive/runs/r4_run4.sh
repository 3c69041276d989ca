#!/bin/bash
# round 4, fourth GPU pass: tests, suite, smoke, bench (train share-of-8 leg), D = 2 fp64 single ops,
# config-5 kernel stats at B = 1e5 (fused) and at the 8-rank share
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_round4.py -v --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_round4_d.txt 2>&1 || { echo "round4 tests failed"; exit 1; }
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_gpu_4.txt 2>&1 || { echo "gpu suite failed"; exit 1; }
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke_4.txt 2>&1 || exit 1
$T 600 python bench.py > gpurun_out/r4_bench_4.json 2> gpurun_out/r4_bench_4.err || exit 1
P=gpurun_out/r4_patterns2.jsonl
for pat in S H C K J I CHS SHK; do
  $T 120 python bench.py --pattern $pat --D 2 --N 1000000 --dtype f64 --no-cpu --no-train --no-pmc --steps 10 >> $P 2>>gpurun_out/r4_patterns2.err || exit 1
done
$T 120 python bench.py --pattern C --dtype f64 --N 5000000 --no-cpu --no-train --no-pmc --steps 10 >> $P 2>>gpurun_out/r4_patterns2.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python bench_train.py --steps 100 > gpurun_out/r4_prof_c5.log 2>&1 || exit 1
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5s -o run -- python bench_train.py --steps 100 --emulate-world 8 > gpurun_out/r4_prof_c5s.log 2>&1 || exit 1
echo ALLDONE
