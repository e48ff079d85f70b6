# Predictor epilogue share (diagnostic build, score-only launch): full / no energy rule / no epilogue
set -o pipefail
O=gpurun_out/r05_c42
mkdir -p $O
timeout -k 10 300 python -u tools/ab.py diag diag@env:VB_DEBUG_PRED=8 diag@env:VB_DEBUG_PRED=1 --what pred --variant both --rounds 20 > $O/ab.log 2>&1 || exit $?
grep -h median $O/ab.log
