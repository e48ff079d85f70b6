set -o pipefail
O=gpurun_out/r05_c27
mkdir -p $O
timeout -k 10 500 python tools/diag/bwd_parity_err.py > $O/bwd_err.log 2>&1
rc=$?; cat $O/bwd_err.log | grep -v amdgpu.ids; exit $rc
