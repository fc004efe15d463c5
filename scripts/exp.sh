#!/bin/bash
# timing experiments: kernel ms of the stream + row launches under env knobs
for cfg in "PR_X=0" "PR_DBG=1" "PR_DBG=2" "PR_DBG=3" "PR_DBG=4" "PR_DBG=6" "PR_DBG=7"; do
  r=$(env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2) || exit $?
  echo "$cfg : $(echo "$r" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'GTEPS', d['roofline']['kernel_ms'], 'ms')")"
done
