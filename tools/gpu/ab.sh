#!/bin/bash
# A/B timing of prebuilt library variants (tools/build_variant.sh) in one process:
#   AB="base new" AB_ARGS="--what attn --variant cog" bash tools/gpu/ab.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab.py ${AB} ${AB_ARGS} 2>&1 | grep -v amdgpu.ids
