#!/bin/bash
# usage: scripts/exp_lib_ab.sh REPS LIB_A LIB_B [scale]   (interleaved, one process per run)
reps=$1; a=$2; b=$3; scale=${4:-26}
for i in $(seq $reps); do
  for l in $a $b; do timeout -k 10 200 scripts/probes/lib_ab $l $scale 20 || exit 1; done
done
