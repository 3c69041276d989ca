#!/bin/bash
# round 4, nineteenth GPU pass: the fp64 interpreter's Johnson step with a wave-vote fast path (asinh64_tab_fin,
# plain table log of the segment product): the whole GPU suite and smoke(), the fp64 D = 2 flows with Johnson
# layers, then the final bench line of the session (the driver's command) and the fp64 / inverse lines
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_gpu_19.txt 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r4_pytest_gpu_19.txt; exit 1; }
tail -2 gpurun_out/r4_pytest_gpu_19.txt
$T 300 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/r4_smoke_19.txt 2>&1 || { cat gpurun_out/r4_smoke_19.txt; exit 1; }
tail -2 gpurun_out/r4_smoke_19.txt
P=gpurun_out/r4_patterns19.jsonl
for pat in J JC KJKJ I; do
  $T 120 python bench.py --pattern $pat --D 2 --N 1000000 --dtype f64 --no-cpu --no-train --no-pmc --steps 20 >> $P 2>>gpurun_out/r4_patterns19.err || exit 1
done
$T 120 python bench.py --pattern HJHJ --D 32 --N 5000000 --dtype f64 --no-cpu --no-train --no-pmc --steps 10 >> $P 2>>gpurun_out/r4_patterns19.err || exit 1
$T 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_bench_19.json 2> gpurun_out/r4_bench_19.err || exit 1
$T 400 python bench.py --dtype f64 --no-train --no-cpu > gpurun_out/r4_bench_f64_19.json 2> gpurun_out/r4_bench_f64_19.err || exit 1
$T 400 python bench.py --dtype f64 --inverse --no-train --no-cpu > gpurun_out/r4_bench_f64_inv_19.json 2> gpurun_out/r4_bench_f64_inv_19.err || exit 1
echo ALLDONE
