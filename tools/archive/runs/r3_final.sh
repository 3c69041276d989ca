#!/bin/bash
# Round-3 evidence run (final state): GPU suite (-x, unserialised), smoke, bench (with the CPU baseline and the
# config-5 train object), rocprofv3 kernel stats of the bench, the PMC passes of the headline kernel, the compiled
# programs against the interpreter on the padded layouts, C2 kernel times. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/fin
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/r03_pytest_gpu_final.txt 2>&1
rc=$?; tail -3 $OUT/r03_pytest_gpu_final.txt; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r03_smoke_final.txt 2>&1
rc=$?; tail -2 $OUT/r03_smoke_final.txt; [ $rc -eq 0 ] || exit $rc
echo "== bench"
timeout -k 10 600 python bench.py > $OUT/r03_bench_final.json 2> $OUT/r03_bench_final.err
rc=$?; cut -c1-400 $OUT/r03_bench_final.json; [ $rc -eq 0 ] || { tail -5 $OUT/r03_bench_final.err; exit $rc; }
echo "== rocprofv3 kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu --no-train --no-pmc --steps 20 > $OUT/r03_prof_bench_final.json 2> $OUT/r03_prof_final.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/r03_prof_final.err; exit $rc; }
cp $OUT/prof/run_kernel_stats.csv $OUT/r03_kernel_stats_final.csv
head -3 $OUT/r03_kernel_stats_final.csv | cut -c1-200
echo "== PMC"
PMC_PASSES=("FETCH_SIZE SQ_WAVES" "WRITE_SIZE"
        "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
        "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR")
i=0
for grp in "${PMC_PASSES[@]}"; do
  i=$((i+1))
  mkdir -p $OUT/pmc; timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/pmc/p$i -o run -- python bench.py --no-cpu --no-train --no-pmc --steps 3 --warmup 1 > $OUT/pmc/p$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pmc pass $i ($grp) failed rc=$rc"; tail -5 $OUT/pmc/p$i.log; exit $rc; }
  echo "pass $i ok"
done
python tools/pmc_summary.py flow_hj_kernel $OUT/pmc D=32 N=10000000 dtype=f32 pairs=4 kernel="enf::flow_hj_kernel<32,8,2,1,4,0,1,0,false>" git=${GIT:-unknown} > $OUT/r03_pmc_bench.json
head -30 $OUT/r03_pmc_bench.json
echo "== compiled programs vs interpreter (padded layouts, D = 128)"
for d in "f32 24 13333333" "f32 100 3200000" "f32 128 2500000" "f64 24 6666666" "f64 100 1600000" "f64 128 1250000"; do
  set -- $d
  timeout -k 10 120 python tools/flow_time.py --product --dtype $1 --D $2 --N $3 --tag compiled_$1_D$2 >> $OUT/r03_padded_vs_interp.jsonl 2>> $OUT/flow.err || { tail -3 $OUT/flow.err; exit 1; }
  ENF_NO_SPECIALIZE=1 timeout -k 10 120 python tools/flow_time.py --dtype $1 --D $2 --N $3 --tag interp_$1_D$2 >> $OUT/r03_padded_vs_interp.jsonl 2>> $OUT/flow.err || { tail -3 $OUT/flow.err; exit 1; }
done
python - <<PY
import json
for l in open("$OUT/r03_padded_vs_interp.jsonl"):
    r = json.loads(l); print(f"{r['tag']:18s} {r['kernel_ms']:.4f} ms  {r['samples_per_s']:.3e}/s  frac {r['hbm_frac']:.3f}")
PY
echo "== C2"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2 -o run -- python tools/flow_time.py --product --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 50 > $OUT/c2.log 2>&1 || { tail -3 $OUT/c2.log; exit 1; }
cp $OUT/c2/run_kernel_stats.csv $OUT/r03_c2_kernel_stats_final.csv
grep flow_ $OUT/r03_c2_kernel_stats_final.csv | cut -c1-160
