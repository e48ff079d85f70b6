set -o pipefail
O=gpurun_out/r05_c32
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; tail -n 3 $O/pytest_gpu.log; tail -n 2 $O/smoke.log; exit $rc
