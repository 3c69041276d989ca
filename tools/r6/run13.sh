#!/bin/bash
# round 6, GPU pass 13: the zygote offset read from the LDS records (fp64 in-range forms) -- its tests and the
# reference examples' step times
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_round6.py tests/test_gpu_train.py \
  tests/test_gpu_train_semantics.py tests/test_gpu_round5.py > gpurun_out/r6/pytest_run13.txt 2>&1 || { tail -30 gpurun_out/r6/pytest_run13.txt; exit 1; }
tail -1 gpurun_out/r6/pytest_run13.txt
for ex in 1d 2d; do
  $T 300 python bench_train.py --example $ex > gpurun_out/r6/example_${ex}_v3.json 2> gpurun_out/r6/ex.err || { tail -5 gpurun_out/r6/ex.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r6/example_${ex}_v3.json').read().strip().splitlines()[-1]); print('$ex', d.get('us_per_step'), d['parity']['history_max_rel_diff_vs_oracle'])"
done
