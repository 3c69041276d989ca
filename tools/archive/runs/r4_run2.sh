#!/bin/bash
# round 4, second GPU pass: round-4 tests, mailbox A/B (diagnostics library), GPU suite, smoke, benches
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_round4.py -v --timeout 120 --timeout-method thread > gpurun_out/r4_pytest_round4_b.txt 2>&1 || { echo "round4 tests failed"; exit 1; }
AB=gpurun_out/r4_mbox_ab.jsonl
for pass in 1 2; do
  $T 120 python tools/flow_time.py --tag prod >> $AB 2>>gpurun_out/r4_mbox_ab.err || exit 1
  ENF_HJ_MBOX=1 $T 120 python tools/flow_time.py --tag mbox >> $AB 2>>gpurun_out/r4_mbox_ab.err || exit 1
  ENF_HJ_MBOX=2 $T 120 python tools/flow_time.py --tag mbox_nowait >> $AB 2>>gpurun_out/r4_mbox_ab.err || exit 1
done
$T 120 python tools/flow_time.py --tag prod_ragged --N 10000003 >> $AB 2>>gpurun_out/r4_mbox_ab.err || exit 1
ENF_HJ_MBOX=1 $T 120 python tools/flow_time.py --tag mbox_ragged --N 10000003 >> $AB 2>>gpurun_out/r4_mbox_ab.err || exit 1
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_gpu_2.txt 2>&1 || { echo "gpu suite failed"; exit 1; }
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke_2.txt 2>&1 || exit 1
$T 500 python bench.py > gpurun_out/r4_bench_2.json 2> gpurun_out/r4_bench_2.err || exit 1
$T 400 python bench.py --inverse --no-train > gpurun_out/r4_bench_inv_2.json 2> gpurun_out/r4_bench_inv_2.err || exit 1
echo ALLDONE
