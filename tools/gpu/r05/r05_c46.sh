# Gathered K/V cost: the per-tile kv_rows-entry DMA skipped after the first 4 tiles (noidx, timing
# only: stale entries) vs the real gather path (cur)
set -o pipefail
O=gpurun_out/r05_c46
mkdir -p $O
for lib in cur noidx cur noidx; do
  if [ $lib = cur ]; then L=video-blade_amd/vblade/libvblade_hip.so; else L=video-blade_amd/vblade/variants/lib_$lib.so; fi
  VBLADE_LIB=$L timeout -k 10 300 python -u tools/diag/gather_cost.py cog > $O/cog_$lib.log 2>&1 || exit $?
  echo "== $lib"; grep -h "attn" $O/cog_$lib.log
done
