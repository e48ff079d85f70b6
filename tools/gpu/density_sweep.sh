set -o pipefail
mkdir -p gpurun_out/sweep
for d in 0.7 0.5 0.3; do
  timeout -k 10 300 python bench.py --density $d --no-cpu-baseline --no-pmc > gpurun_out/sweep/cog_d$d.json 2> gpurun_out/sweep/cog_d$d.err || exit 1
  echo "cog $d: $(cut -c1-200 gpurun_out/sweep/cog_d$d.json)"
done
for d in 0.5 0.3; do
  timeout -k 10 300 python bench.py --variant wan --density $d --no-cpu-baseline --no-pmc > gpurun_out/sweep/wan_d$d.json 2> gpurun_out/sweep/wan_d$d.err || exit 1
  echo "wan $d done"
done
