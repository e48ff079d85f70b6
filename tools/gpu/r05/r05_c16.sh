set -o pipefail
O=gpurun_out/r05_c16
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mlbwd -o run --output-format csv -- python3 tools/ab.py cur --what mlbwd --variant cog --rounds 5 > $O/mlbwd.log 2>&1 && \
python3 tools/kstats.py $O/prof_mlbwd > $O/mlbwd_kstats.txt 2>&1 && \
PMC_VARIANT=cog bash tools/gpu/pmc.sh > $O/pmc_fwd_cog.txt 2>&1
rc=$?; cat $O/mlbwd_kstats.txt | head -30; tail -40 $O/pmc_fwd_cog.txt; exit $rc
