set -o pipefail
bash tools/gpu_suite.sh r3c5 && bash tools/gpu_perf_groups.sh r3c5
