set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multilevel.py tests/test_gpu_module.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mlrand_pytest.log 2>&1
tail -1 gpurun_out/mlrand_pytest.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/mlrand_prof -o run -- python bench.py --steps 10 --warmup 3 > gpurun_out/mlrand_bench.log 2>&1
python - <<'PY'
import sqlite3, glob
db = glob.glob('gpurun_out/mlrand_prof/**/*.db', recursive=True) + glob.glob('gpurun_out/mlrand_prof/*.db')
c = sqlite3.connect(db[0])
for r in c.execute("select name,total_calls,average from top_kernels where name like '%topk%' or name like '%sample_rows%'"): print(r)
PY
