#!/bin/bash
# Bench pass: small-model bench, then the 8B headline bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python bench.py --model llama-small --seq 4096 --steps 5 --warmup 2 --verbose > gpurun_out/bench_small.log 2>&1; rc=$?
echo "bench_small rc=$rc"; tail -8 gpurun_out/bench_small.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps ${STEPS:-5} --warmup 2 --verbose > gpurun_out/bench_8b.log 2>&1; rc=$?
echo "bench_8b rc=$rc"; tail -8 gpurun_out/bench_8b.log
exit $rc
