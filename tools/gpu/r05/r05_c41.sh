# Kernel-level split of gather_kv on vs off (attention kernel with gathered K/V rows vs Gilbert copies;
# predictor launch with and without the copies' writes)
set -o pipefail
O=gpurun_out/r05_c41
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/diag/overlap_ab.py --opt gather_kv > $O/gather.log 2>&1 || exit $?
grep -h median $O/gather.log
