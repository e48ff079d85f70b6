#!/bin/bash
# Fused level mask: multilevel GPU tests, the multi-level call A/B (fused vs its own launch), then
# predictor A/B of the contiguous-copy K stream variants.
set -o pipefail
OUT=gpurun_out/r03_lv
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_multilevel.py tests/test_gpu_module.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 400 python tools/ab.py cur@lvsep cur cur@lvsep cur --what mlcall --variant cog > $OUT/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab.py base g0 g0b4 base g0 g0b4 --what pred --variant both > $OUT/ab_g0.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_g0.log; exit $rc
