#!/bin/bash
# round 4, twelfth GPU pass: per-launch spread of the headline kernel in launch order (two bench lines, 40 launches
# each, no train / cpu / pmc legs) and of the fp64 forward program
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  $T 300 python bench.py --steps 40 --warmup 5 --no-train --no-cpu --no-pmc > gpurun_out/r4_bench_order_$i.json 2> gpurun_out/r4_bench_order_$i.err || exit 1
done
$T 300 python bench.py --steps 40 --warmup 5 --no-train --no-cpu --no-pmc --dtype f64 > gpurun_out/r4_bench_order_f64.json 2> gpurun_out/r4_bench_order_f64.err || exit 1
echo ALLDONE
