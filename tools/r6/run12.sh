#!/bin/bash
# round 6, GPU pass 12: (1) the data-parallel step's row-payload threshold (rows path only while <= 64 KiB) and the
# finite-loss asserts of the finite-difference tests; (2) config 5's 8-rank share (one-rank emulation) on the product
# path it now takes, and the reference examples after the zygote loss moved into the step prologue
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_round5.py tests/test_gpu_round3.py \
  tests/test_gpu_round4.py tests/test_gpu_train.py tests/test_gpu_round6.py > gpurun_out/r6/pytest_run12.txt 2>&1 || { tail -30 gpurun_out/r6/pytest_run12.txt; exit 1; }
tail -1 gpurun_out/r6/pytest_run12.txt
$T 200 python bench_train.py --steps 100 --emulate-world 8 > gpurun_out/r6/c5_share8_v2.json 2> gpurun_out/r6/c5.err || { tail -5 gpurun_out/r6/c5.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r6/c5_share8_v2.json').read().strip().splitlines()[-1]); print('share8', d['ms_per_step']*1e3, 'us')"
for ex in 1d 2d; do
  $T 300 python bench_train.py --example $ex > gpurun_out/r6/example_${ex}_v2.json 2> gpurun_out/r6/ex.err || { tail -5 gpurun_out/r6/ex.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r6/example_${ex}_v2.json').read().strip().splitlines()[-1]); print('$ex', d.get('us_per_step'), d.get('parity'))"
done
