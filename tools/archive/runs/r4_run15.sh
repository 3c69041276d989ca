#!/bin/bash
# round 4, fifteenth GPU pass: bench.py with the settle phase (--settle-ms 100 by default): per-launch times in
# launch order after it, the full headline line (in-run PMC, train, CPU baseline), the inverse and fp64 lines,
# and a separate rocprofv3 --kernel-trace --stats run of the default command for profiles/
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 300 python bench.py --steps 40 --warmup 5 --no-train --no-cpu --no-pmc > gpurun_out/r4_bench_order_settled.json 2> gpurun_out/r4_bench_order_settled.err || exit 1
$T 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench_15.json 2> gpurun_out/r4_bench_15.err || exit 1
$T 400 python bench.py --inverse --no-train --no-cpu > gpurun_out/r4_bench_inv_15.json 2> gpurun_out/r4_bench_inv_15.err || exit 1
$T 400 python bench.py --dtype f64 --no-train --no-cpu > gpurun_out/r4_bench_f64_15.json 2> gpurun_out/r4_bench_f64_15.err || exit 1
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_prof15 -o run -- python3 bench.py --steps 20 --warmup 5 --no-train --no-cpu --no-pmc > gpurun_out/r4_prof15.log 2>&1 || exit 1
echo ALLDONE
