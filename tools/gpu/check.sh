#!/bin/bash
# Smoke, the GPU suite and one default bench run of the current tree.
# Usage (from the repo root, on the GPU box): TAG=name bash tools/gpu/check.sh
set -o pipefail
OUT=gpurun_out/${TAG:-check}
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 900 python bench.py $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-800 $OUT/bench.json
exit $rc
