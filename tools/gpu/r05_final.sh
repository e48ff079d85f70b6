# Round-5 final measurement of the committed tree: GPU suite, smoke, bench line, kernel traces of
# the bench variants and the backward, training steps (tools/gpu/measure.sh), then the forward PMC.
set -o pipefail
TAG=r05_final bash tools/gpu/measure.sh && \
PMC_VARIANT=cog bash tools/gpu/pmc.sh > gpurun_out/r05_final/pmc_fwd_cog.txt 2>&1
