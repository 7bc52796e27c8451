#!/bin/bash
# r02 (last session) end check on the GPU box: full GPU suite, smoke(), the
# default bench line, then rocprof kernel stats of the bench and PMC traffic passes.
set -u
bash scripts/check_r02c.sh final3 || exit $?
bash scripts/gpu_profile_r02.sh final3_prof
