#!/bin/bash
# Overlapped exchange in a rank group on ONE GPU: round time of the p-rank group at R-MAT scale
# SCALE with an injected delay before every chunk's copies (PR_XDELAY_US, standing in for the
# transfer time device copies do not have), uncut schedule (PR_XOVERLAP=0) against the cut one.
# usage: scripts/exp_overlap.sh TAG SCALE p "delay_us ..."
tag=$1; scale=$2; p=$3; delays=$4
out=gpurun_out/overlap_$tag.txt
for d in $delays; do
  for ov in 0 1; do
    line=$(PR_XDELAY_US=$d PR_XOVERLAP=$ov timeout -k 10 300 python3 scripts/group_split.py $scale $p 2>gpurun_out/overlap_err.log | tail -1) || { echo "failed d=$d ov=$ov"; tail -5 gpurun_out/overlap_err.log; exit 1; }
    echo "delay ${d} us/chunk | overlap $ov | $line" | tee -a "$out"
  done
done
