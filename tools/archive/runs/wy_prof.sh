#!/bin/bash
# Dense-Householder kernel evidence: throughput lines (tools/wy_bench.py, both paths), JohnsonSU
# throughput (tools/jsu_bench.py), rocprofv3 kernel stats and FETCH_SIZE / WRITE_SIZE passes of the
# D=32 k=32 fp32 flow (tools/wy_one.py).
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/wy
mkdir -p $OUT
timeout -k 10 300 python tools/wy_bench.py > $OUT/wy_mfma.jsonl 2> $OUT/wy_mfma.err || { tail -5 $OUT/wy_mfma.err; exit 1; }
ENF_WY_MIN_K=100000 timeout -k 10 300 python tools/wy_bench.py > $OUT/wy_interp.jsonl 2> $OUT/wy_interp.err || { tail -5 $OUT/wy_interp.err; exit 1; }
timeout -k 10 300 python tools/jsu_bench.py > $OUT/jsu.jsonl 2> $OUT/jsu.err || { tail -5 $OUT/jsu.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python tools/wy_one.py 32 32 f32 10000000 10 > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof64 -o run -- python tools/wy_one.py 64 64 f32 12500000 10 > $OUT/prof64.log 2>&1 || { tail -5 $OUT/prof64.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profjsu -o run -- python tools/jsu_bench.py > $OUT/profjsu.log 2>&1 || { tail -5 $OUT/profjsu.log; exit 1; }
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/pmc/p$i -o run -- python tools/wy_one.py 32 32 f32 10000000 3 > $OUT/pmc$i.log 2>&1 || { echo "pmc $grp failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
cat $OUT/wy_mfma.jsonl $OUT/wy_interp.jsonl $OUT/jsu.jsonl | cut -c1-220
cut -c1-150 $OUT/prof/run_kernel_stats.csv | head -4
cut -c1-150 $OUT/prof64/run_kernel_stats.csv | head -4
cut -c1-150 $OUT/profjsu/run_kernel_stats.csv | head -6
python tools/pmc_summary.py flow_wy $OUT/pmc
