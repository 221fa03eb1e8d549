set -o pipefail
bash scripts/r3_gpu_suite.sh r3_suite_a && bash scripts/r3_trace_routed.sh r3_trace_a
