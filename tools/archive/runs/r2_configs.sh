#!/bin/bash
# Every BASELINE.json config measured on one MI355X (the round's evidence): C1 on the host cores
# (tools/c1_cpu_bench.py), C2-C4 through bench.py (inputs resident in HBM, HIP-event kernel time),
# C5 through bench_train.py. One JSON line per run into gpurun_out/r02_configs.jsonl.
set -u
OUT=gpurun_out/r02_configs.jsonl
: > $OUT
run() { timeout -k 10 300 "$@" 2> gpurun_out/r02_configs.err | grep '^{' >> $OUT; rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "failed rc=$rc: $*"; tail -5 gpurun_out/r02_configs.err; exit $rc; }; }
run python tools/c1_cpu_bench.py
run python bench.py --no-cpu --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 50 --warmup 5
run python bench.py --no-cpu --D 2 --N 1000000 --pairs 1 --dtype f32 --steps 50 --warmup 5
run python bench.py --no-cpu
run python bench.py --no-cpu --dtype f64 --steps 5 --warmup 2
run python bench.py --no-cpu --D 64 --N 12500000 --steps 10 --warmup 2
run python bench_train.py
cat $OUT | cut -c1-400
