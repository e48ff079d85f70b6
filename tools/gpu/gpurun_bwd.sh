#!/bin/bash
# backward bring-up: backward parity tests first (fail fast), then the whole GPU suite, then timing
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_backward.py -x -q -p no:cacheprovider > gpurun_out/pytest_bwd.log 2>&1
rc=$?
echo "bwd pytest rc=$rc"; tail -30 gpurun_out/pytest_bwd.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "all gpu pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/kbench.py --bwd 2>&1 | grep -v amdgpu.ids
