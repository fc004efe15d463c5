#!/bin/bash
# Stream-launch diagnosis at the current defaults: kernel trace, PR_DBG ablations (1 no piece
# stores, 2 no L2 gathers, 3 neither), per-phase stamps, SQ counter passes.
# usage (GPU box, repo root): scripts/diag.sh TAG ["VAR=value ..."]
tag=$1; v=$2
mkdir -p gpurun_out
scripts/kt.sh ${tag} $v || exit $?
scripts/exp.sh "$v PR_DBG=0" "$v PR_DBG=1" "$v PR_DBG=2" "$v PR_DBG=3" "$v PR_DBG=0" || exit $?
scripts/stamps.sh ${tag} "$v" > /dev/null || exit $?
grep -h "stamps\] slice\|phase 20\|phase  0\|phase 19" gpurun_out/stamps_${tag}.txt
scripts/pmc_stream.sh ${tag} $v || exit $?
