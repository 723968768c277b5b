#!/bin/bash
# Iteration pass: full GPU test suite, attention microbench, 8B bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_attn.py > gpurun_out/bench_attn.log 2>&1; rc=$?
echo "attn bench rc=$rc"; tail -1 gpurun_out/bench_attn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS} > gpurun_out/bench_8b.log 2>&1; rc=$?
echo "bench_8b rc=$rc"; tail -1 gpurun_out/bench_8b.log
exit $rc
