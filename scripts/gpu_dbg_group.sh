#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for g in 2 0; do
  echo "== DPE_GPT2_WGRAD_GROUP=$g"
  DPE_GPT2_WGRAD_GROUP=$g timeout -k 10 120 python scripts/debug_wgrad_group.py || exit 1
done
