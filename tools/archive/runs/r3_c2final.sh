set -u
mkdir -p gpurun_out/c2final
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c2final/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/c2final/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/c2final/pytest_gpu.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c2final/prof -o run -- python tools/flow_time.py --product --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 500 > gpurun_out/c2final/flow_time.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c2final/prof_cold -o run -- python tools/flow_time.py --product --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 300 --flush-mb 512 > gpurun_out/c2final/flow_time_cold.log 2>&1 || exit 1
python3 -c "
import csv
for d in ('prof', 'prof_cold'):
    for r in csv.DictReader(open('gpurun_out/c2final/%s/run_kernel_stats.csv' % d)):
        if 'flow_' in r['Name']: print(d, r['Name'][:60], r['Calls'], 'avg_us %.2f' % (float(r['AverageNs']) / 1e3), 'min_us %.2f' % (float(r['MinNs']) / 1e3))
"
