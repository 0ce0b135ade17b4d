#!/bin/bash
# Round 6: rocprofv3 kernel trace + PMC passes of the product core (glibc_seq4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/profile.sh ${1:-r06a}
