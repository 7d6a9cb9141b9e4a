#!/bin/bash
# A/B of two stamp-probe binaries, alternating, same box (diagnostic).
# Usage: bash scripts/probe_ab.sh binA binB S R batch rounds
A=$1; B=$2; S=$3; R=$4; BT=$5; N=${6:-3}
for i in $(seq $N); do
  for b in $A $B; do
    echo "=== $b"
    timeout -k 5 60 $b $S $R $BT | grep "fit chain" | tail -1 || exit $?
  done
done
