#!/bin/bash
# PMC passes over scripts/prof_decode.py (diagnostic).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/pmc_passes.sh gpurun_out/pmc scripts/prof_decode.py "$@"
python scripts/pmc_summary.py gpurun_out/pmc
