#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/overlap_ab.py --opt gather_kv 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python tools/ab.py old new old new 2>&1 | grep -v amdgpu.ids
