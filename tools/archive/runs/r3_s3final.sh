#!/bin/bash
# Round-3 last-session final evidence (kernel with the wave-priority schedule): GPU suite (-x, unserialised), smoke,
# bench (in-run PMC), rocprofv3 kernel stats of the bench command, the PMC passes as a committed summary (the
# fallback for multi-rank runs), compiled programs on the padded layouts. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/s3f
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.txt; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
rc=$?; tail -1 $OUT/smoke.txt; [ $rc -eq 0 ] || exit $rc
echo "== bench"
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']
print('value %.4g frac %.4f kernel_ms %.4f rocprof %s traffic %s' % (d['value'], r['frac'], r['kernel_ms'], r['rocprof_kernel_stats'] and r['rocprof_kernel_stats']['average_ms'], r['traffic']))
print('train', d['train'].get('value'))"
echo "== rocprofv3 kernel stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu --no-train --no-pmc --steps 20 > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/prof.err; exit $rc; }
cp $OUT/prof/run_kernel_stats.csv $OUT/kernel_stats.csv; grep flow_hj $OUT/kernel_stats.csv | cut -c1-200
echo "== PMC"
PMC_PASSES=("FETCH_SIZE SQ_WAVES" "WRITE_SIZE"
        "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
        "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR")
i=0
for grp in "${PMC_PASSES[@]}"; do
  i=$((i+1))
  mkdir -p $OUT/pmc; timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/pmc/p$i -o run -- python bench.py --no-cpu --no-train --no-pmc --steps 3 --warmup 1 > $OUT/pmc/p$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pmc pass $i failed rc=$rc"; tail -5 $OUT/pmc/p$i.log; exit $rc; }
done
python tools/pmc_summary.py flow_hj_kernel $OUT/pmc D=32 N=10000000 dtype=f32 pairs=4 kernel="enf::flow_hj_kernel<32,8,2,1,4,0,1,0,false>" git=${GIT:-unknown} > $OUT/pmc_bench.json
grep -E "hbm_bytes_per_launch|SQ_INSTS_VALU\"|effective_clock" $OUT/pmc_bench.json
echo "== compiled programs, padded layouts"
for d in "f32 24 13333333" "f32 100 3200000" "f32 128 2500000" "f32 64 5000000"; do
  set -- $d
  timeout -k 10 120 python tools/flow_time.py --product --dtype $1 --D $2 --N $3 --tag compiled_$1_D$2 >> $OUT/padded.jsonl 2>> $OUT/flow.err || { tail -3 $OUT/flow.err; exit 1; }
done
python3 -c "
import json
for l in open('$OUT/padded.jsonl'):
    r=json.loads(l); print(r['tag'], '%.4f ms' % r['kernel_ms'], '%.3e/s' % r['samples_per_s'], 'frac %.3f' % r['hbm_frac'])"
