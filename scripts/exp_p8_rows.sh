#!/bin/bash
# Per-rank kernel times of a p-rank group on one GPU under row-launch variants (rows per block,
# chunks of the exchange).  usage: scripts/exp_p8_rows.sh TAG P "ENV=.. ENV=.." ...
tag=$1; p=$2; shift 2
i=0
for v in "$@"; do
  i=$((i + 1))
  echo "== ${v:-defaults}"
  env $v scripts/group_kt.sh ${tag}_$i $p || exit 1
done
