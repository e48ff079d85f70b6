#!/bin/bash
# Round 2: new parity tests (config 1, processors, empty-row LSE) + the full bench line.
set -o pipefail
OUT=gpurun_out/r02_a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_module.py tests/test_gpu_forward.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > $OUT/bench_cog.json 2> $OUT/bench_cog.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench_cog.json
