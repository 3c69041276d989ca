#!/bin/bash
# round 4, third GPU pass: chunked-training and round-4 tests, mailbox A/B (fixed), GPU suite, benches,
# inverse kernel stats, other transforms / example flow shapes
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_round4.py -v --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_round4_c.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "round4 tests rc=$rc"; exit $rc; fi
AB=gpurun_out/r4_mbox_ab2.jsonl
for pass in 1 2; do
  $T 120 python tools/flow_time.py --tag prod >> $AB 2>>gpurun_out/r4_mbox_ab2.err || exit 1
  ENF_HJ_MBOX=1 $T 120 python tools/flow_time.py --tag mbox >> $AB 2>>gpurun_out/r4_mbox_ab2.err || exit 1
  ENF_HJ_MBOX=3 $T 120 python tools/flow_time.py --tag mbox_busy >> $AB 2>>gpurun_out/r4_mbox_ab2.err || exit 1
done
P=gpurun_out/r4_patterns.jsonl
for pat in S C K I H4 H4JH4J JC KJKJ CHS SHK; do
  $T 120 python bench.py --pattern $pat --no-cpu --no-train --no-pmc --steps 10 >> $P 2>>gpurun_out/r4_patterns.err || exit 1
done
for pat in CHS SHK JC KJKJ; do
  $T 120 python bench.py --pattern $pat --D 2 --N 1000000 --dtype f64 --no-cpu --no-train --no-pmc --steps 10 >> $P 2>>gpurun_out/r4_patterns.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_inv -o run -- python bench.py --inverse --no-cpu --no-train --no-pmc --steps 20 > gpurun_out/r4_prof_inv.log 2>&1 || exit 1
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_gpu_3.txt 2>&1 || { echo "gpu suite failed"; exit 1; }
$T 600 python bench.py > gpurun_out/r4_bench_3.json 2> gpurun_out/r4_bench_3.err || exit 1
echo ALLDONE
