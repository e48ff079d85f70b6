#!/bin/bash
# Backward pipeline kernels: parity with every new kernel on, A/B against the previous kernels, traces.
set -o pipefail
O=gpurun_out/${TAG:-bwd_ab}
mkdir -p $O
export TMPDIR=/tmp
VB_BWD_KV64=1 VB_BWD_DQ128=1 VB_BWD_DQ64=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for var in cog wan; do
  AB="kvold cur all" AB_ARGS="--what bwd --variant $var" bash tools/gpu/ab.sh > $O/ab_$var.log 2>&1 || exit 1
  tail -6 $O/ab_$var.log
done
for var in cog wan; do
  VB_BWD_KV64=1 VB_BWD_DQ128=1 VB_BWD_DQ64=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$var -o run --output-format csv -- python3 tools/kbench.py --only-bwd --variant $var > $O/kbench_$var.log 2>&1 || exit 1
  python3 tools/kstats.py $O/prof_$var | grep -E "vb::bwd|vb::pool_grad" | head -8
done
