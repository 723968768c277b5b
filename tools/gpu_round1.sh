#!/bin/bash
# First GPU pass: kernel numerics, smoke, small-model bench, 8B bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ok() { rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -rf > gpurun_out/kernels.log 2>&1; rc=$?
echo "kernels rc=$rc"; tail -30 gpurun_out/kernels.log
ok $rc || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 400 python bench.py --model llama-small --seq 4096 --steps 5 --warmup 2 --verbose > gpurun_out/bench_small.log 2>&1; rc=$?
echo "bench_small rc=$rc"; tail -8 gpurun_out/bench_small.log
ok $rc || exit $rc
timeout -k 10 900 python bench.py --steps 5 --warmup 2 --verbose > gpurun_out/bench_8b.log 2>&1; rc=$?
echo "bench_8b rc=$rc"; tail -8 gpurun_out/bench_8b.log
exit $rc
