#!/bin/bash
# Config 2 memory floor: the compiled D = 2 kernel with loads and stores but no Johnson arithmetic
# (ENF_D2_DBG=3) and the product kernel with and without nontemporal loads / stores (ENF_D2_NT), and a torch device copy of X's 16 MB and
# a 40 MB read+write elementwise op for scale. gpurun_out/c2floor/.
set -u
OUT=gpurun_out/c2floor
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # tag, env [flow_time args]
  local tag=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python tools/flow_time.py --D 2 --N 1000000 --pairs 1 --dtype f64 --steps 200 "$@" > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$tag/run_kernel_stats.csv')):
    if 'flow_' in r['Name']: print('$tag', r['Name'][:60], r['Calls'], 'avg_us %.2f' % (float(r['AverageNs']) / 1e3), 'min_us %.2f' % (float(r['MinNs']) / 1e3), flush=True)
"
}
if [ "${ONLY_COLD:-0}" = 1 ]; then
  for rep in 1 2 3; do for nt in 3 2; do run cold_nt${nt}_r$rep ENF_D2_NT=$nt --flush-mb 512 || exit 1; done; done
  exit 0
fi
for rep in 1 2; do
  for nt in 3 0 1 2; do run product_nt${nt}_r$rep ENF_D2_NT=$nt || exit 1; done
  for nt in 3 0; do run memonly_nt${nt}_r$rep "ENF_D2_DBG=3 ENF_D2_NT=$nt" || exit 1; done
  for nt in 3 2 0; do run cold_nt${nt}_r$rep ENF_D2_NT=$nt --flush-mb 512 || exit 1; done
done
grep -h -o '"tag".*"out_sha1": "[0-9a-f]*"' $OUT/product_nt*_r1.log $OUT/cold_nt*_r1.log | sed 's/"D".*"out_sha1"/ sha1/'
cat > $OUT/c2copy.py <<'PY'
import torch
x = torch.randn(2_000_000, dtype=torch.float64, device="cuda")
y = torch.empty_like(x)
z = torch.empty(1_000_000, dtype=torch.float64, device="cuda")
for _ in range(200):
    y.copy_(x)
for _ in range(200):
    torch.mul(x, 2.0, out=y)
torch.cuda.synchronize()
PY
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/copy -o run -- python $OUT/c2copy.py > $OUT/copy.log 2>&1 || { echo "copy fail"; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/copy/run_kernel_stats.csv')):
    print('copy', r['Name'][:70], r['Calls'], 'avg_us %.2f' % (float(r['AverageNs']) / 1e3), 'min_us %.2f' % (float(r['MinNs']) / 1e3))
"
