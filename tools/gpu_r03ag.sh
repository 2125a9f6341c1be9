#!/bin/bash
# Round 3 ag: rocprofv3 kernel statistics + PMC passes (tools/profile_round.sh) of the
# bench workload on the current build, SCL-LUT and FastSCL-LUT.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 bash tools/profile_round.sh r03ag_scl --kind SCL-LUT > $O/r03ag_prof_scl.log 2>&1 || exit $?
timeout -k 10 550 bash tools/profile_round.sh r03ag_fscl --kind FastSCL-LUT > $O/r03ag_prof_fscl.log 2>&1 || exit $?
echo "profiles done"
