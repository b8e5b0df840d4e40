set -o pipefail
bash tools/gpu_pmc.sh r03_g1 20 || exit 1
PMC_SCRIPT=tools/cross_one.py bash tools/gpu_pmc.sh r03_cross_g1 20 edit 4096 40 || exit 1
PMC_SCRIPT=tools/cross_one.py bash tools/gpu_pmc.sh r03_cross_g2 20 edit+store 1024 80 || exit 1
PMC_SCRIPT=tools/cross_one.py bash tools/gpu_pmc.sh r03_cross_g3 20 edit+store 256 160 || exit 1
