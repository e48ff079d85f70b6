set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/topk_pytest.log 2>&1
tail -3 gpurun_out/topk_pytest.log
timeout -k 10 300 python tools/ab.py t0 t1 --variant both --what call > gpurun_out/topk_ab.log 2>&1
cat gpurun_out/topk_ab.log | tail -12
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/topk_prof -o run -- python bench.py --steps 20 --warmup 5 > gpurun_out/topk_bench.log 2>&1
tail -1 gpurun_out/topk_bench.log
