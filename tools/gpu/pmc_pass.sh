#!/bin/bash
# One rocprofv3 PMC pass per invocation (counters of one block group only), written under
# gpurun_out/<name>/.  Usage (on the GPU box):
#   bash tools/gpu/pmc_pass.sh <name> "<counters>" "<kernel regex>" <program args...>
set -o pipefail
name=$1; counters=$2; regex=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -s KILL 200 rocprofv3 --pmc $counters --kernel-include-regex "$regex" --output-format csv \
  -d "gpurun_out/$name" -o run -- "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "pmc $name rc=$rc"
exit $rc
