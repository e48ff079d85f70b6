#!/bin/bash
# Philox draws in the sampling launch: the GPU suite, then the per-call A/B against torch.rand draws.
set -o pipefail
OUT=gpurun_out/r03_philox
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 600 python tools/ab.py cur@torchrand cur cur@torchrand cur --what call --variant both > $OUT/ab_call.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_call.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/traffic_probe.py --out $OUT/traffic.json
