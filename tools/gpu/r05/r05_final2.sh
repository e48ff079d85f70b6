# Round-5 final measurement after the 2-wave multi-level pyramid items (training steps unchanged: r05_final)
set -o pipefail
TAG=r05_final2 NO_TRAIN=1 bash tools/gpu/measure.sh
