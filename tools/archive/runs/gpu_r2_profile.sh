#!/bin/bash
# Round-2 evidence run: the GPU test suite, the bench (with the CPU baseline), the rocprofv3 kernel
# trace of the bench, and the PMC passes of the headline kernel. Stops at a crash / timeout.
set -u
OUT=gpurun_out
V=${V:-v1}
mkdir -p $OUT
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r02_pytest_gpu_$V.txt 2>&1
  rc=$?; tail -4 $OUT/r02_pytest_gpu_$V.txt; ok $rc || { echo "pytest crashed rc=$rc"; exit $rc; }
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
echo "== bench"
timeout -k 10 600 python bench.py > $OUT/r02_bench_$V.json 2> $OUT/r02_bench_$V.err
rc=$?; cat $OUT/r02_bench_$V.json; [ $rc -eq 0 ] || { tail -5 $OUT/r02_bench_$V.err; exit $rc; }
echo "== rocprofv3 kernel trace"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$V -o run -- python bench.py --no-cpu --no-train --no-pmc --steps 20 > $OUT/r02_prof_bench_$V.json 2> $OUT/r02_prof_$V.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/r02_prof_$V.err; exit $rc; }
find $OUT/prof_$V -name '*kernel_stats.csv' -exec cp {} $OUT/r02_kernel_stats_$V.csv \;
cat $OUT/r02_kernel_stats_$V.csv | head -5
fi
echo "== PMC"
# one counter group per pass: FETCH_SIZE (3 TCC) and WRITE_SIZE (2 TCC) cannot share a pass
PMC_PASSES=("FETCH_SIZE SQ_WAVES" "WRITE_SIZE"
        "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
        "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR")
i=0
for grp in "${PMC_PASSES[@]}"; do
  i=$((i+1))
  mkdir -p $OUT/pmc_$V; timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/pmc_$V/p$i -o run -- python bench.py --no-cpu --no-train --no-pmc --steps 3 --warmup 1 > $OUT/pmc_$V/p$i.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "pmc pass $i ($grp) failed rc=$rc"; tail -5 $OUT/pmc_$V/p$i.log; exit $rc; }
  echo "pass $i ok"
done
python tools/pmc_summary.py flow_hj $OUT/pmc_$V D=32 N=10000000 dtype=f32 pairs=4 kernel="enf::flow_hj_kernel<32,8,2,1,4,0,1>" git=${GIT:-unknown} > $OUT/r02_pmc_bench_$V.json
cat $OUT/r02_pmc_bench_$V.json | head -40
