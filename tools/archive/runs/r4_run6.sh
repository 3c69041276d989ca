#!/bin/bash
# round 4, sixth GPU pass: fp64 C3 program instruction mix (in-run PMC incl. the fp64 classes) and the
# register-cap A/B of flow_hj64_kernel on the diagnostics library
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 400 python bench.py --dtype f64 --no-train --no-cpu > gpurun_out/r4_bench_f64_6.json 2> gpurun_out/r4_bench_f64_6.err || exit 1
for occ in 1 4; do
  ENF_HJ64_OCC=$occ $T 200 python tools/flow_time.py --dtype f64 --tag occ$occ >> gpurun_out/r4_f64_ab_6.jsonl 2>> gpurun_out/r4_f64_ab_6.err || exit 1
done
echo ALLDONE
