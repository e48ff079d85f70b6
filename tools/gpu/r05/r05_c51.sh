# Gathered K/V: the first two tiles' kv_rows entries fetched before the kept-block list is built
# (cur, VB_GATHER_EARLY=1) vs the committed prologue (gbase). Parity first; then the module call
# with gather_kv on/off on the new library.
set -o pipefail
O=gpurun_out/r05_c51
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_module.py tests/test_gpu_fullsize.py tests/test_gpu_config1.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head -8; exit $rc; }
for lib in gbase cur gbase cur; do
  if [ $lib = cur ]; then L=video-blade_amd/vblade/libvblade_hip.so; else L=video-blade_amd/vblade/variants/lib_$lib.so; fi
  VBLADE_LIB=$L timeout -k 10 300 python -u tools/diag/gather_cost.py cog > $O/cog_$lib.log 2>&1 || exit $?
  VBLADE_LIB=$L timeout -k 10 300 python -u tools/diag/gather_cost.py wan > $O/wan_$lib.log 2>&1 || exit $?
  echo "== $lib"; grep -h "attn" $O/cog_$lib.log $O/wan_$lib.log
done
timeout -k 10 300 python -u tools/diag/overlap_ab.py --opt gather_kv > $O/gather_call.log 2>&1 || exit $?
grep -h median $O/gather_call.log
