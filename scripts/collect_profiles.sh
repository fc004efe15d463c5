#!/bin/bash
# Round profile artefacts for the bench workload (run on the GPU box from the repo root):
#   rocprofv3 --kernel-trace --stats of the bench command, then separate PMC passes for the
#   HBM traffic of the SpMV kernels.  usage: scripts/collect_profiles.sh TAG [bench args]
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
pass() { # name, rocprof args...
  local name=$1; shift
  timeout -s KILL 180 rocprofv3 "$@" -d $out/$name -o run --output-format csv -- python3 bench.py --no-cpu-baseline "${BA[@]}" > $out/$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"; tail -n 1 $out/$name.log
  [ $rc -eq 0 ] || exit $rc
}
BA=("$@")
[ -n "$SKIP_KT" ] || pass kt --kernel-trace --stats   # (SKIP_KT: the caller has taken the trace already)
pass rd --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-include-regex spmv
pass wr --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-include-regex spmv
pass fetch --pmc FETCH_SIZE --kernel-include-regex spmv
pass write --pmc WRITE_SIZE --kernel-include-regex spmv
pass l2 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex spmv
