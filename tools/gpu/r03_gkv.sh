set -o pipefail
OUT=gpurun_out/r03_gkv; mkdir -p $OUT
timeout -k 10 300 python tools/overlap_ab.py --opt gather_kv > $OUT/gkv.log 2>&1; rc=$?; grep -v amdgpu $OUT/gkv.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/gkv_prof.py > $OUT/prof.log 2>&1; rc=$?; echo "prof rc=$rc"
python3 tools/kstats.py $OUT/prof | grep -E "mask_pred|sample_rows|attn_fwd|pool_kv"
