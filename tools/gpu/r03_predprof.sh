# Kernel-trace summaries of the predictor launch for library variants: TAGS="base inl" bash tools/gpu/r03_predprof.sh
set -o pipefail
OUT=gpurun_out/${OUTTAG:-predprof}; mkdir -p $OUT
export TMPDIR=/tmp
for tag in ${TAGS:-base inl}; do for var in cog wan; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/$tag-$var -o run --output-format csv -- python3 tools/pred_prof.py $tag $var both > $OUT/$tag-$var.log 2>&1
  rc=$?; echo "$tag $var rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/kstats.py $OUT/$tag-$var | grep -E "mask_pred|sample_rows|attn_fwd|pool_kv" 
done; done
