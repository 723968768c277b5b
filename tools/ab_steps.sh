#!/bin/bash
# Interleaved same-box A/B of one environment switch on the headline bench:
#   gpurun -- bash tools/ab_steps.sh ACCELERATE_FSDP_WGRAD_XT 0
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
VAR=$1; OFF=$2
for i in 1 2; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/ab_default_$i.log 2>&1 || exit 1
  env "$VAR=$OFF" timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/ab_switched_$i.log 2>&1 || exit 1
done
