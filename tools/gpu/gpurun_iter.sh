#!/bin/bash
# iteration loop: gpu parity tests (fail fast) then per-kernel timing
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 400 python tools/kbench.py ${KB_ARGS} 2>&1 | grep -v amdgpu.ids
fi
