#!/bin/bash
# round 4: fresh PMC traffic of the Detect head after the paired line loads
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04am}; mkdir -p $O
bash scripts/pmc_run.sh $O/pmc head > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
tail -2 $O/pmc.log
