#!/bin/bash
# timing experiments: kernel ms of the stream + row launches under env knobs (args: configs)
for cfg in "$@"; do
  r=$(env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2) || exit $?
  echo "$cfg : $(echo "$r" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'GTEPS', d['roofline']['kernel_ms'], 'ms')")"
done
