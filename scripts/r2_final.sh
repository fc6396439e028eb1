# full GPU suite + smoke + benches + steady-state profiles (current tree)
set -o pipefail
bash scripts/r2_verify.sh || exit 1
bash scripts/r2_prof_both.sh || exit 1
