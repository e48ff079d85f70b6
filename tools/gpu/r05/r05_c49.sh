# Gathered K/V: no entry/row stages past the last kept tile (nopast, timing only: the last tile's
# counts over-release) vs the committed path (cur)
set -o pipefail
O=gpurun_out/r05_c49
mkdir -p $O
for lib in cur nopast cur nopast; do
  if [ $lib = cur ]; then L=video-blade_amd/vblade/libvblade_hip.so; else L=video-blade_amd/vblade/variants/lib_$lib.so; fi
  VBLADE_LIB=$L timeout -k 10 300 python -u tools/diag/gather_cost.py cog > $O/cog_$lib.log 2>&1 || exit $?
  echo "== $lib"; grep -h "attn" $O/cog_$lib.log
done
