#!/bin/bash
# Register use and scratch spills of the SpMV kernels in the built engine object (CPU only).
# usage: scripts/kernel_regs.sh
set -e
cd "$(dirname "$0")/../page-rank-and-tfidf-using-apache-spark_amd/_build"
tmp=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objdump --offloading engine.o > /dev/null
mv engine.o.0.hipv4-amdgcn-amd-amdhsa--gfx950 "$tmp/engine.co"
rm -f engine.o.0.host-x86_64-unknown-linux-gnu-
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$tmp/engine.co" \
  | grep -E "^ +\.name:|\.vgpr_count|vgpr_spill|\.sgpr_count|private_segment_fixed" | paste - - - - - \
  | grep -E "spmv_(stream|rows|dpull)" | sed 's/ \+/ /g' | cut -c1-220
rm -rf "$tmp"
