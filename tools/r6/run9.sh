#!/bin/bash
# round 6, GPU pass 9: the data-parallel rows path (enf_whitening_step_dp without the reduction launch): the training
# tests, then the config-5 legs of the bench (B = 1e5 fused step, the 8-rank share with its per-phase breakdown) and
# a kernel trace of the share step
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_round5.py tests/test_gpu_round4.py \
  tests/test_gpu_train.py tests/test_gpu_round6.py tests/test_gpu_train_semantics.py > gpurun_out/r6/pytest_run9.txt 2>&1 || { tail -30 gpurun_out/r6/pytest_run9.txt; exit 1; }
tail -1 gpurun_out/r6/pytest_run9.txt
$T 300 python bench_train.py --steps 100 --emulate-world 8 --breakdown > gpurun_out/r6/c5_share8_v1.json 2> gpurun_out/r6/c5_share8_v1.err || { tail -5 gpurun_out/r6/c5_share8_v1.err; exit 1; }
$T 300 python bench_train.py --steps 100 --breakdown > gpurun_out/r6/c5_B1e5_v1.json 2> gpurun_out/r6/c5_B1e5_v1.err || { tail -5 gpurun_out/r6/c5_B1e5_v1.err; exit 1; }
python3 -c "
import json
for f in ('gpurun_out/r6/c5_share8_v1.json','gpurun_out/r6/c5_B1e5_v1.json'):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d.get('ms_per_step'), d.get('step'), json.dumps(d.get('phases'))[:300])
"
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof9 -o s -- python3 bench_train.py --steps 100 --emulate-world 8 > /dev/null 2>&1 || exit 1
echo ALLDONE
