#!/bin/bash
# the walk-priority and far-child prefetch knobs (A/B in one build), then the evidence session
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_env_matrix.sh r04g "dragon bunny helmet sky_dragon bunny16" 2 "-" "PT_WALK_PREFETCH=1" "PT_WALK_PRIO=1" || exit $?
bash tools/gpu_evidence.sh r04g
