#!/bin/bash
# round 4, sixteenth GPU pass: the whole GPU suite and smoke() on the final library, then settled re-measurements of
# the single transforms / example flows (fp32 D = 32, fp64 D = 2), the C4 shard (D = 64) and the padded layouts
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_gpu_16.txt 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r4_pytest_gpu_16.txt; exit 1; }
tail -2 gpurun_out/r4_pytest_gpu_16.txt
$T 300 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/r4_smoke_16.txt 2>&1 || { cat gpurun_out/r4_smoke_16.txt; exit 1; }
tail -2 gpurun_out/r4_smoke_16.txt
P=gpurun_out/r4_patterns16.jsonl
for pat in S C K I H4 J H4J JC KJKJ CHS SHK; do
  $T 120 python bench.py --pattern $pat --no-cpu --no-train --no-pmc --steps 20 >> $P 2>>gpurun_out/r4_patterns16.err || exit 1
done
for pat in HJ C K I JC KJKJ CHS SHK S; do
  $T 120 python bench.py --pattern $pat --D 2 --N 1000000 --dtype f64 --no-cpu --no-train --no-pmc --steps 20 >> $P 2>>gpurun_out/r4_patterns16.err || exit 1
done
L=gpurun_out/r4_layouts16.jsonl
$T 200 python bench.py --D 64 --N 12500000 --no-cpu --no-train --no-pmc >> $L 2>>gpurun_out/r4_layouts16.err || exit 1
$T 200 python bench.py --D 24 --N 10000000 --no-cpu --no-train --no-pmc >> $L 2>>gpurun_out/r4_layouts16.err || exit 1
$T 200 python bench.py --D 100 --N 3200000 --no-cpu --no-train --no-pmc >> $L 2>>gpurun_out/r4_layouts16.err || exit 1
$T 200 python bench.py --D 128 --N 2500000 --no-cpu --no-train --no-pmc >> $L 2>>gpurun_out/r4_layouts16.err || exit 1
$T 200 python bench.py --pairs 8 --no-cpu --no-train --no-pmc >> $L 2>>gpurun_out/r4_layouts16.err || exit 1
echo ALLDONE
