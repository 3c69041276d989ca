#!/bin/bash
# round 4, twentieth GPU pass: the driver's bench command with the stdout guard (exactly one line on stdout)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_bench_20.json 2> gpurun_out/r4_bench_20.err || exit 1
wc -l gpurun_out/r4_bench_20.json
python -c "import json; d=json.load(open('gpurun_out/r4_bench_20.json')); print(d['value'], d['roofline']['frac'], d['train'].get('value'))"
echo ALLDONE
