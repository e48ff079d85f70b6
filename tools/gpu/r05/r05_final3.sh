# Round-5 final measurement after the pipelined pool/pyramid passes (and Wan's pooling workgroups
# after its score workgroups): A/B against the tree before them, then the full measurement.
set -o pipefail
mkdir -p gpurun_out/r05_final3
timeout -k 10 400 python -u tools/ab.py pbase cur --what call --variant both --rounds 25 > gpurun_out/r05_final3/ab_call.log 2>&1 || exit $?
grep -h median gpurun_out/r05_final3/ab_call.log
TAG=r05_final3 bash tools/gpu/measure.sh
