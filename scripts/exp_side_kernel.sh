#!/bin/bash
# scripts/probes/side_kernel_probe under 32 / 31 / 30 / 28 stream-launch compute units per XCD
for c in 32 31 30 28; do
  PR_STREAM_CUS=$c timeout -k 10 200 scripts/probes/side_kernel_probe 26 || exit 1
done
