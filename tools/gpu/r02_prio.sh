set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/prio_pytest.log 2>&1
tail -1 gpurun_out/prio_pytest.log
timeout -k 10 400 python tools/ab.py x0 x1 --variant both --what call > gpurun_out/prio_call.log 2>&1
grep median gpurun_out/prio_call.log
timeout -k 10 400 python bench.py > gpurun_out/prio_bench.json 2> gpurun_out/prio_bench.err
python -c "import json; d=json.loads(open('gpurun_out/prio_bench.json').read().strip().splitlines()[-1]); print(d['value'], [(p['variant'], p['ms_per_call'], p['speedup_vs_dense_sdpa']) for p in d['points']])"
