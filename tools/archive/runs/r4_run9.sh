#!/bin/bash
# round 4, ninth GPU pass (fp64 instruction cuts: degree-6 log1p polynomial, no Goldschmidt h update, the q
# product carried across the pairs of flow_hj64_kernel, z = fma(x, 1/lambda, -xi/lambda)): the whole GPU suite,
# the fp64 C3 bench line with its in-run PMC, and the D = 2 fp64 patterns (config 2 and the Center flows)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_gpu_9.txt 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r4_pytest_gpu_9.txt; exit 1; }
tail -3 gpurun_out/r4_pytest_gpu_9.txt
$T 400 python bench.py --dtype f64 --no-train --no-cpu > gpurun_out/r4_bench_f64_9.json 2> gpurun_out/r4_bench_f64_9.err || exit 1
P=gpurun_out/r4_patterns9.jsonl
for pat in HJ C K I JC KJKJ CHS SHK S; do
  $T 120 python bench.py --pattern $pat --D 2 --N 1000000 --dtype f64 --no-cpu --no-train --no-pmc --steps 20 >> $P 2>>gpurun_out/r4_patterns9.err || exit 1
done
echo ALLDONE
