#!/bin/bash
# Round 6, the final build (six programs per wave): rocprofv3 kernel trace +
# PMC passes of the bench workload.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/profile.sh r06c
