#!/bin/bash
# Training path: GPU tests, config-5 bench, rocprofv3 kernel stats of the bench.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/train_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/train_tests.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench_train.py ${TRAIN_ARGS:-} > gpurun_out/train.json 2> gpurun_out/train.err || { tail -5 gpurun_out/train.err; exit 1; }
cat gpurun_out/train.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/proftrain -o run -- python bench_train.py --steps 50 ${TRAIN_ARGS:-} > /dev/null 2> gpurun_out/proftrain.err || { tail -5 gpurun_out/proftrain.err; exit 1; }
cut -c1-160 gpurun_out/proftrain/run_kernel_stats.csv | head -8
