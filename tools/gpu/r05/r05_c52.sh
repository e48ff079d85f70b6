# Gathered K/V: the row voffset multiply-add from the compiler (__umul24) instead of inline asm (cmad)
set -o pipefail
O=gpurun_out/r05_c52
mkdir -p $O
for lib in cur cmad cur cmad; do
  if [ $lib = cur ]; then L=video-blade_amd/vblade/libvblade_hip.so; else L=video-blade_amd/vblade/variants/lib_$lib.so; fi
  VBLADE_LIB=$L timeout -k 10 300 python -u tools/diag/gather_cost.py cog > $O/cog_$lib.log 2>&1 || exit $?
  echo "== $lib"; grep -h "attn\|identical" $O/cog_$lib.log
done
