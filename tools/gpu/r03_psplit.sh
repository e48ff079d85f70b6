set -o pipefail
OUT=gpurun_out/r03_psplit; mkdir -p $OUT
timeout -k 10 300 python tools/pred_split.py pdiag 0,1,2,4,5,6 > $OUT/split.log 2>&1; rc=$?; grep -v amdgpu $OUT/split.log; exit $rc
