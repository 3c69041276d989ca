#!/bin/bash
# round 4, fifth GPU pass: round-4 tests (fused data-parallel step), suite, smoke, bench, config-5 kernel stats
# (the fused data-parallel step at the 8-rank share), inverse bench after the sinh change
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_round4.py -v --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_round4_e.txt 2>&1 || { echo "round4 tests failed"; exit 1; }
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_gpu_5.txt 2>&1 || { echo "gpu suite failed"; exit 1; }
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke_5.txt 2>&1 || exit 1
$T 600 python bench.py > gpurun_out/r4_bench_5.json 2> gpurun_out/r4_bench_5.err || exit 1
$T 400 python bench.py --inverse --no-train > gpurun_out/r4_bench_inv_5.json 2> gpurun_out/r4_bench_inv_5.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5s2 -o run -- python bench_train.py --steps 100 --emulate-world 8 > gpurun_out/r4_prof_c5s2.log 2>&1 || exit 1
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5b -o run -- python bench_train.py --steps 100 > gpurun_out/r4_prof_c5b.log 2>&1 || exit 1
echo ALLDONE
