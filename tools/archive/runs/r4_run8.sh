#!/bin/bash
# round 4, eighth GPU pass (vote-based in-range path): the fp64 Center steps on exp64 / the table log (new wide-range tests, the parity
# files that cover Center / JohnsonInv in fp64), then the D = 2 and D = 32 fp64 pattern timings
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_round4.py -v --timeout 300 --timeout-method thread -k "center" > gpurun_out/r4_pytest_center_8.txt 2>&1 || { echo "center tests failed"; exit 1; }
$T 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_round3.py tests/test_gpu_round4.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_parity_8.txt 2>&1 || { echo "parity tests failed"; exit 1; }
P=gpurun_out/r4_patterns8.jsonl
for pat in C K I JC KJKJ CHS SHK S; do
  $T 120 python bench.py --pattern $pat --D 2 --N 1000000 --dtype f64 --no-cpu --no-train --no-pmc --steps 10 >> $P 2>>gpurun_out/r4_patterns8.err || exit 1
done
for pat in C K I; do
  $T 120 python bench.py --pattern $pat --dtype f64 --N 5000000 --no-cpu --no-train --no-pmc --steps 10 >> $P 2>>gpurun_out/r4_patterns8.err || exit 1
done
echo ALLDONE
