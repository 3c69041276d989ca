#!/bin/bash
# Round-3, third session: the freshly rebuilt tree on MI355X -- GPU suite (-x, unserialised), smoke, bench.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/s3a
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.txt; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
rc=$?; tail -2 $OUT/smoke.txt; [ $rc -eq 0 ] || exit $rc
echo "== bench"
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cut -c1-600 $OUT/bench.json; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
