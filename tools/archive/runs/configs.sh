#!/bin/bash
# The other SURVEY §8(d) configs on one GPU: C2 (J∘H, D=2, N=1e6, fp64), C4 per-GPU shard
# (D=64, N=1.25e7), C3 fp64 and the 8x(J∘H) variant; one JSON line each.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { timeout -k 5 180 python bench.py --no-cpu "$@" 2>/dev/null || { echo "failed: $*"; exit 1; }; }
{
run --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 200
run --D 64 --N 12500000 --pairs 4 --steps 20
run --D 32 --N 10000000 --pairs 4 --dtype f64 --steps 10
run --D 32 --N 10000000 --pairs 8 --steps 20
} | tee gpurun_out/configs.jsonl
