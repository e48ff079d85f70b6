#!/bin/bash
# determinism diagnostic + GPU suite + A/B timing of library variants: AB="base new" bash tools/gpu/gpurun_ab.sh
mkdir -p gpurun_out
timeout -k 10 200 python tools/diag_first.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python tools/ab.py ${AB} 2>&1 | grep -v amdgpu.ids
