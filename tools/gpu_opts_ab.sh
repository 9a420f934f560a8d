#!/bin/bash
# Per-unit code-generation options re-checked on the current source: each unit's variants against
# the in-tree build on that unit's own workload (tools/ab_env.sh, interleaved on one box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-opts}
TAG=${TAG}_W REPS=2 VARIANTS="base|| w_npr_ilp|build/ab/w_npr_ilp.so| w_npr_trk|build/ab/w_npr_trk.so|" CASES="W:--config W;W2:--config W --ebn0 2" bash tools/ab_env.sh | tail -7 || exit 1
TAG=${TAG}_R REPS=2 VARIANTS="base|| m_none|build/ab/m_none.so| m_trk_npr|build/ab/m_trk_npr.so|" CASES="R:--config R" bash tools/ab_env.sh | tail -4 || exit 1
TAG=${TAG}_A REPS=2 VARIANTS="base|| a_npr|build/ab/a_npr.so| a_npr_ilp_trk|build/ab/a_npr_ilp_trk.so|" CASES="A:--config A;A45:--config A --ebn0 4.5" bash tools/ab_env.sh | tail -7 || exit 1
