#!/bin/bash
# multi-level path: its GPU parity tests, then the forward regression tests
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_multilevel.py -x -q -p no:cacheprovider > gpurun_out/pytest_ml.log 2>&1
rc=$?
echo "ml pytest rc=$rc"; tail -30 gpurun_out/pytest_ml.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 600 python -m pytest tests/test_gpu_forward.py -x -q -p no:cacheprovider > gpurun_out/pytest_fwd.log 2>&1
  echo "fwd pytest rc=$?"; tail -5 gpurun_out/pytest_fwd.log
fi
