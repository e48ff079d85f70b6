#!/bin/bash
# Build the current sources into video-blade_amd/vblade/variants/lib_<TAG>.so (A/B timing, tools/ab.py)
set -e
TAG=${1:?tag}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=/tmp/vb_variant_$TAG
rm -rf $B
mkdir -p $B "$ROOT/video-blade_amd/vblade/variants"
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$ROOT/include -I$ROOT/video-blade_amd/csrc ${VB_EXTRA_FLAGS}"
pids=()
for f in "$ROOT"/video-blade_amd/csrc/*.hip "$ROOT"/video-blade_amd/csrc/*.cpp; do
  extra=""; case "$f" in *vb_attn_fwd.hip|*vb_attn_fwd_m16.hip) extra="-fno-slp-vectorize -fno-honor-nans ${VB_FWD_FLAGS--mllvm -amdgpu-sched-strategy=iterative-ilp}";; *vb_predict.hip) extra="-fno-honor-nans ${VB_PRED_FLAGS}";; *vb_attn_bwd.hip) extra="${VB_BWD_FLAGS--mllvm -amdgpu-sched-strategy=iterative-ilp}";; *vb_attn_bwd_kv.hip) extra="-fno-slp-vectorize ${VB_KV_FLAGS}";; esac
  /opt/rocm/bin/hipcc $FL $extra -c "$f" -o $B/$(basename $f).o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "compile failed"; exit 1; }; done
/opt/rocm/bin/hipcc -shared -fPIC -Wl,--no-undefined --offload-arch=gfx950 $B/*.o -o "$ROOT/video-blade_amd/vblade/variants/lib_$TAG.so"
echo "built variants/lib_$TAG.so"
