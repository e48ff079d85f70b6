#!/bin/bash
# Is the D=128 dK/dV pipeline waiting on memory? A/B against a build without DMA after the
# prologue (wrong results, timing only), and L2 hit/miss + fetch counters of the backward.
set -o pipefail
O=gpurun_out/${TAG:-bwd_l2}
mkdir -p $O
export TMPDIR=/tmp
AB="cur nodma" AB_ARGS="--what bwd --variant wan" bash tools/gpu/ab.sh > $O/ab_wan.log 2>&1 || exit 1
tail -3 $O/ab_wan.log
for c in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  n=$(echo $c | cut -d" " -f1)
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$n -o run -- python3 tools/kbench.py --only-bwd --variant wan > $O/pmc_$n.log 2>&1 || { echo "pmc $n failed"; tail -3 $O/pmc_$n.log; }
done
python3 - <<PY
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob("$O/pmc_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "bwd_" in r["Kernel_Name"]:
            acc[(r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k, len(v), "%.4g" % (sum(v) / len(v)))
PY
