#!/bin/bash
# Sparse-exchange packs on the comm stream (PR_PACKCOMM=1) against the compute stream (0): round
# time of a p-rank group on one GPU, interleaved.  usage: scripts/exp_packcomm.sh TAG SCALE REPS p...
tag=$1; scale=$2; reps=$3; shift 3
export GPU_MAX_HW_QUEUES=24
out=gpurun_out/packcomm_$tag.txt
for p in "$@"; do
  for i in $(seq $reps); do
    for v in 0 1; do
      line=$(PR_PACKCOMM=$v timeout -k 10 300 python3 scripts/group_split.py $scale $p 2>gpurun_out/packcomm_err.log | tail -1) || { echo "failed p=$p v=$v"; tail -5 gpurun_out/packcomm_err.log; exit 1; }
      echo "rep $i | PR_PACKCOMM=$v | $line" | tee -a "$out"
    done
  done
done
