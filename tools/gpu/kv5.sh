mkdir -p gpurun_out/kv5
VB_BWD_KV64=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kv5/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/kv5/pytest.log; [ $rc -eq 0 ] || exit $rc
AB="kvold kvnew kv64" AB_ARGS="--what bwd --variant cog" bash tools/gpu/ab.sh > gpurun_out/kv5/ab_cog.log 2>&1 || exit 1
tail -6 gpurun_out/kv5/ab_cog.log
AB="kvold kvnew nodma" AB_ARGS="--what bwd --variant wan" bash tools/gpu/ab.sh > gpurun_out/kv5/ab_wan.log 2>&1 || exit 1
tail -6 gpurun_out/kv5/ab_wan.log
