# Final binary: the default bench line (sanity against r05_final3)
set -o pipefail
O=gpurun_out/r05_c53
mkdir -p $O
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench.err; exit $rc; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_call'],d['speedup_vs_dense_sdpa'],d['roofline']['avg_launch_ms'],d['roofline']['frac'],[(b['variant'],b['avg_ms']) for b in d['backward']])"
