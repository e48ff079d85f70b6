# Round-2 end-of-session check: smoke, the GPU suite, one default bench run
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/end2_smoke.log 2>&1
tail -1 gpurun_out/end2_smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/end2_pytest.log 2>&1
tail -1 gpurun_out/end2_pytest.log
timeout -k 10 400 python bench.py > gpurun_out/end2_bench.json 2> gpurun_out/end2_bench.err
tail -c 300 gpurun_out/end2_bench.json
