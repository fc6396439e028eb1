set -o pipefail
# per-kernel counters (ResNet-50 and GPT-2) at the current head + one steady step's per-dispatch bytes (ResNet)
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash scripts/gpu_pmc_steady.sh || exit 1
