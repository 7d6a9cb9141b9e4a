#!/bin/bash
# Surrogate-fit stamp probe over tuning settings (diagnostic; tools/wlm_probe built with
# -DXPG_WLM_STAMPS).  Usage: bash scripts/probe_sweep.sh S R batch "ENV=.. ENV=.." ...
mkdir -p gpurun_out
S=$1; R=$2; B=$3; shift 3
for cfg in "$@"; do
  echo "=== $cfg"
  env $cfg timeout -k 5 60 ./tools/wlm_probe $S $R $B | tail -9 || exit $?
done
