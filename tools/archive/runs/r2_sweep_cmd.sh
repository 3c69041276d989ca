set -u
mkdir -p gpurun_out
for p in 1 2 4 8; do
  for v in "acc:ENF_DEBUG_MODE=2" "fast:ENF_DEBUG_MODE=2 ENF_HJ_ASINH=0" "accmem:ENF_NONE=0" "fastmem:ENF_HJ_ASINH=0"; do
    tag=${v%%:*}; kv=${v#*:}
    env $kv timeout -k 10 120 python tools/flow_time.py --pairs $p --tag ${tag}_p$p >> gpurun_out/r2c_sweep.jsonl 2>> gpurun_out/r2c_sweep.err || exit $?
  done
done
cat gpurun_out/r2c_sweep.jsonl | python -c "import sys,json; [print(d['tag'], round(d['kernel_ms'],4)) for d in map(json.loads, sys.stdin)]"
LIST=1 TAG=acc_compute VAR="ENF_DEBUG_MODE=2" bash tools/pmc_flow.sh
