#!/bin/bash
# round 4, tenth GPU pass (fp64 program: branch-free pair loop with a whole-tile redo, the q product as the
# range check, mov_dpp group sums, three-address y fma; the new compiled fp64 inverse program): table-function
# ulp probe, the whole GPU suite, the fp64 C3 forward and inverse bench lines with in-run PMC, fp64 D = 64 /
# padded D = 24 / 100 lines
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 120 ./tools/asinh64_tab_check > gpurun_out/r4_asinh64_tab_check_10.txt 2>&1 || { echo "probe failed"; cat gpurun_out/r4_asinh64_tab_check_10.txt; exit 1; }
cat gpurun_out/r4_asinh64_tab_check_10.txt
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_gpu_10.txt 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r4_pytest_gpu_10.txt; exit 1; }
tail -3 gpurun_out/r4_pytest_gpu_10.txt
$T 400 python bench.py --dtype f64 --no-train --no-cpu > gpurun_out/r4_bench_f64_10.json 2> gpurun_out/r4_bench_f64_10.err || exit 1
$T 400 python bench.py --dtype f64 --inverse --no-train --no-cpu > gpurun_out/r4_bench_f64_inv_10.json 2> gpurun_out/r4_bench_f64_inv_10.err || exit 1
P=gpurun_out/r4_f64_layouts_10.jsonl
$T 200 python bench.py --dtype f64 --D 64 --N 5000000 --no-train --no-cpu --no-pmc >> $P 2>>gpurun_out/r4_f64_layouts_10.err || exit 1
$T 200 python bench.py --dtype f64 --D 24 --N 10000000 --no-train --no-cpu --no-pmc >> $P 2>>gpurun_out/r4_f64_layouts_10.err || exit 1
$T 200 python bench.py --dtype f64 --D 100 --N 3200000 --no-train --no-cpu --no-pmc >> $P 2>>gpurun_out/r4_f64_layouts_10.err || exit 1
$T 200 python bench.py --dtype f64 --inverse --D 64 --N 5000000 --no-train --no-cpu --no-pmc >> $P 2>>gpurun_out/r4_f64_layouts_10.err || exit 1
$T 200 python bench.py --dtype f64 --inverse --D 100 --N 3200000 --no-train --no-cpu --no-pmc >> $P 2>>gpurun_out/r4_f64_layouts_10.err || exit 1
echo ALLDONE
