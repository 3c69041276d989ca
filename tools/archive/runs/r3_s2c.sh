#!/bin/bash
# pin-overlap hypothesis (tools/pin_overlap_probe.py): (1) round 2's per-array registration (diagnostics library,
# ENF_PIN_LEGACY=1) with heap-only allocations; stops here if it faults. (2) the product's disjoint page-aligned
# registration, same traffic. (3) the GPU suite once, unserialised.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s2c
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_VM_FAULT_MESSAGE=1
timeout -k 5 60 ./tools/microbench23 > $O/mb23.txt 2>&1 || exit 1
cat $O/mb23.txt
MALLOC_MMAP_THRESHOLD_=2000000000 timeout -k 10 300 python -u tools/pin_overlap_probe.py --legacy --iters 30 > $O/probe_legacy.txt 2>&1
rc=$?; tail -4 $O/probe_legacy.txt; grep -c " ok" $O/probe_legacy.txt
[ $rc -eq 0 ] || { echo "legacy probe rc=$rc"; exit $rc; }
MALLOC_MMAP_THRESHOLD_=2000000000 timeout -k 10 300 python -u tools/pin_overlap_probe.py --iters 30 > $O/probe_new.txt 2>&1
rc=$?; tail -2 $O/probe_new.txt
[ $rc -eq 0 ] || { echo "new probe rc=$rc"; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -4 $O/pytest_gpu.txt
exit $rc
