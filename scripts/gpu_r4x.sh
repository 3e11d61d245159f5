#!/bin/bash
# Round 4: the MLP chain check (gpu_r4o.sh), then the final pass part 1 (gpu_r4z.sh); stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
bash scripts/gpu_r4o.sh && bash scripts/gpu_r4z.sh
