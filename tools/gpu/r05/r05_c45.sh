# Gathered K/V: kv_rows entries read at the end of the previous body (VB_EARLY_ENT64=1, in-tree; early128
# adds D=128) vs read between the barrier and the row DMAs (noearly). Parity first.
set -o pipefail
O=gpurun_out/r05_c45
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_module.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head -8; exit $rc; }
for lib in noearly cur early128 noearly cur; do
  if [ $lib = cur ]; then L=video-blade_amd/vblade/libvblade_hip.so; else L=video-blade_amd/vblade/variants/lib_$lib.so; fi
  VBLADE_LIB=$L timeout -k 10 300 python -u tools/diag/gather_cost.py cog > $O/cog_$lib.log 2>&1 || exit $?
  VBLADE_LIB=$L timeout -k 10 300 python -u tools/diag/gather_cost.py wan > $O/wan_$lib.log 2>&1 || exit $?
  echo "== $lib"; grep -h "attn" $O/cog_$lib.log $O/wan_$lib.log
done
