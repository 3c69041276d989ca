#!/bin/bash
# round 4, first GPU pass: new tests, the whole GPU suite, smoke, headline bench, inverse bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_round4.py -v --timeout 120 --timeout-method thread > gpurun_out/r4_pytest_round4.txt 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "round4 tests rc=$rc"; exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_gpu_1.txt 2>&1 || { echo "gpu suite failed"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke_1.txt 2>&1 || exit 1
timeout -k 10 500 python bench.py > gpurun_out/r4_bench_1.json 2> gpurun_out/r4_bench_1.err || exit 1
timeout -k 10 400 python bench.py --inverse --no-train > gpurun_out/r4_bench_inv_1.json 2> gpurun_out/r4_bench_inv_1.err || exit 1
echo ALLDONE
