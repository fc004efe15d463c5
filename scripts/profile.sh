#!/bin/bash
# rocprofv3 passes over a short bench run (each PMC pass its own run; no trace domains
# combined with --pmc).  usage: scripts/profile.sh TAG [bench args...]
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { # name, rocprof args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" -d $out/$name -o run --output-format csv -- python3 bench.py --no-cpu-baseline "${BENCH_ARGS[@]}" > $out/$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"; tail -n 2 $out/$name.log
  case $rc in 0) ;; *) exit $rc ;; esac
}
BENCH_ARGS=("$@")
run kt --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run tcc --pmc TCC_HIT_sum TCC_MISS_sum
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
