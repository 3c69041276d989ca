#!/bin/bash
# (1) pin probe on the staging ring (no host registration), heap-only allocations; (2) wave-specialised
# headline kernel A/B (ENF_HJ_SPEC=0/1, diagnostics library, bitwise output fingerprints), D = 32 and 64;
# (3) GPU suite once; (4) ingest throughput of the staging ring.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s2d
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_VM_FAULT_MESSAGE=1
MALLOC_MMAP_THRESHOLD_=2000000000 timeout -k 10 400 python -u tools/pin_overlap_probe.py --iters 60 > $O/probe.txt 2>&1
rc=$?; tail -2 $O/probe.txt; [ $rc -eq 0 ] || { echo "probe rc=$rc"; exit $rc; }
for rep in 1 2 3; do
  for v in 0 1; do
    ENF_HJ_SPEC=$v timeout -k 10 120 python tools/flow_time.py --tag spec$v > /dev/null 2>> $O/ab.err && \
    ENF_HJ_SPEC=$v timeout -k 10 120 python tools/flow_time.py --tag spec$v >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab failed"; tail -5 $O/ab.err; exit 1; }
  done
done
for v in 0 1; do
  ENF_HJ_SPEC=$v timeout -k 10 120 python tools/flow_time.py --D 64 --N 5000000 --tag d64spec$v >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab64 failed"; tail -5 $O/ab.err; exit 1; }
done
python - <<PY
import json
for l in open("$O/ab.jsonl"):
    r = json.loads(l); print(f"{r['tag']:10s} D{r['D']} {r['kernel_ms']:.4f} ms frac {r['hbm_frac']:.3f} sha {r['out_sha1']}")
PY
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -4 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ingest_bench.py > $O/ingest.jsonl 2>&1; rc=$?; cat $O/ingest.jsonl; exit $rc
