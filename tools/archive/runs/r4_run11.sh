#!/bin/bash
# round 4, eleventh GPU pass: the fp64 forward program's range check as the max of the q high words (|z| < 2^26;
# the product check admitted |z| where asinh64_tab_fin is wrong, tools/asinh64_tab_check.hip), the ulp probe,
# the whole GPU suite, the fp64 forward / inverse bench lines (in-run PMC), the headline bench line
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 120 ./tools/asinh64_tab_check > gpurun_out/r4_asinh64_tab_check_11.txt 2>&1 || { echo "probe failed"; cat gpurun_out/r4_asinh64_tab_check_11.txt; exit 1; }
cat gpurun_out/r4_asinh64_tab_check_11.txt
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_gpu_11.txt 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r4_pytest_gpu_11.txt; exit 1; }
tail -3 gpurun_out/r4_pytest_gpu_11.txt
$T 400 python bench.py --dtype f64 --no-train --no-cpu > gpurun_out/r4_bench_f64_11.json 2> gpurun_out/r4_bench_f64_11.err || exit 1
$T 400 python bench.py --dtype f64 --inverse --no-train --no-cpu > gpurun_out/r4_bench_f64_inv_11.json 2> gpurun_out/r4_bench_f64_inv_11.err || exit 1
$T 600 python bench.py > gpurun_out/r4_bench_11.json 2> gpurun_out/r4_bench_11.err || exit 1
echo ALLDONE
