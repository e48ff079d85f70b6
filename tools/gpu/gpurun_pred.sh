#!/bin/bash
# predictor change: module/forward GPU parity tests (fail fast), then A/B of the predictor
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab.py ${AB:-pw4 pvm pw4 pvm} --what pred 2>&1 | grep -v amdgpu.ids
