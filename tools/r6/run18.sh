#!/bin/bash
# round 6, GPU pass 18 (final build): the whole GPU suite, smoke, the default bench line (in-run PMC, CPU baseline,
# config-5 train object and the reference examples) and a kernel-trace summary of the same command
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/pytest_run18_full.txt 2>&1 || { tail -30 gpurun_out/r6/pytest_run18_full.txt; exit 1; }
tail -1 gpurun_out/r6/pytest_run18_full.txt
$T 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/smoke_run18.txt 2>&1 || { cat gpurun_out/r6/smoke_run18.txt; exit 1; }
tail -1 gpurun_out/r6/smoke_run18.txt
$T 500 python bench.py > gpurun_out/r6/bench_v2.json 2> gpurun_out/r6/bench_v2.err || { tail -20 gpurun_out/r6/bench_v2.err; exit 1; }
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof18 -o b -- python3 bench.py --no-cpu --no-train --no-pmc > /dev/null 2>&1 || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r6/bench_v2.json')); r=d['roofline']
print('value', d['value'], 'frac', r['frac'], 'kernel_ms', r['kernel_ms'], 'traffic', r['traffic'], 'copy', r['frac_of_copy_ceiling'])
print('valu', json.dumps(d.get('valu'))[:400])
t=d.get('train') or {}
print('train', json.dumps({k: t[k] for k in t if k in ('value','ms_per_step')}))
s8=t.get('rank_share_of_8') or {}
print('share8', s8.get('ms_per_step'))
ex=t.get('reference_examples') or {}
for k,v in ex.items(): print('example', k, v.get('us_per_step'), v.get('parity'))
"
echo ALLDONE
