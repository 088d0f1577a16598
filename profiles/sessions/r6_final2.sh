set -o pipefail
# closing run on the final kernels: smoke, the GPU suite, forward and training bench lines, then the
# round-6 profiles re-collected (profiles/collect.sh)
bash profiles/sessions/r6_final.sh || exit 1
bash profiles/collect.sh r06
