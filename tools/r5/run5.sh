#!/bin/bash
# round 5, fifth GPU pass: config-5 kernels under graph replay (rocprofv3), and the small-argument launch probe
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof5_share8_graph -o c5 -- python3 bench_train.py --steps 200 --warmup 20 --emulate-world 8 > gpurun_out/r5/c5_share8_graph_prof.json 2>/dev/null || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof5_B1e5_graph -o c5 -- python3 bench_train.py --steps 200 --warmup 20 > gpurun_out/r5/c5_B1e5_graph_prof.json 2>/dev/null || exit 1
for dbg in 1 3; do
  ENF_RED_DBG=$dbg $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof5_reddbg${dbg}_graph -o c5 -- python3 bench_train.py --diag --steps 200 --warmup 20 --emulate-world 8 > gpurun_out/r5/reddbg${dbg}_graph.json 2>/dev/null || exit 1
  ENF_RED_DBG=$dbg $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof5_reddbg${dbg}_eager -o c5 -- python3 bench_train.py --diag --steps 100 --warmup 10 --emulate-world 8 --graph 0 > /dev/null 2>&1 || exit 1
done
echo PROBES_DONE
# D <= 2: the per-wave prologue (product) against the block prologue (ENF_SMALL_PW=0, diagnostics library),
# kernel durations under rocprofv3 (cold legs last), then the D <= 2 GPU parity tests
for pw in 1 0; do
  for pat in JC SHK S J; do
    ENF_SMALL_PW=$pw $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof5_pw${pw}_$pat -o d2 -- python3 tools/flow_time.py --pattern $pat --D 2 --N 1000000 --dtype f64 --steps 200 --tag pw${pw}_$pat >> gpurun_out/r5/pw_ab.jsonl 2>/dev/null || exit 1
  done
done
echo PW_DONE
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_round4.py -k "fp64_center or D or d2 or small or center" > gpurun_out/r5/pytest_run5.txt 2>&1 || { tail -30 gpurun_out/r5/pytest_run5.txt; exit 1; }
tail -2 gpurun_out/r5/pytest_run5.txt
echo ALLDONE
