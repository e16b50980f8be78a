#!/bin/bash
# Round 4: profiles and PMC passes again with --no-paced (kernel-level statistics of the default
# schedule only), then the bench lines (PART=1) so they pick up this code's PMC summaries.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
T=${1:-r4}
PART=2 bash tools/gpu_round.sh $T
