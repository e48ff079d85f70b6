set -o pipefail
O=gpurun_out/r05_c20
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multilevel.py -x -q --timeout 120 --timeout-method thread > $O/pytest_ml.log 2>&1 && \
timeout -k 10 300 python tools/ab.py mldq0 mlkv0 cur mldq0 mlkv0 cur --what mlbwd --variant cog > $O/mlbwd.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mlbwd -o run --output-format csv -- python3 tools/ab.py cur --what mlbwd --variant cog --rounds 5 > $O/mlbwd_prof.log 2>&1 && \
python3 tools/kstats.py $O/prof_mlbwd > $O/mlbwd_kstats.txt 2>&1
rc=$?; tail -n 3 $O/pytest_ml.log; grep -h -E "median|identical|diff" $O/mlbwd.log; head -8 $O/mlbwd_kstats.txt; exit $rc
