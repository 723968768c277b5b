#!/bin/bash
# Round-1 pass E: fp8 GEMM v2 (4-wave, 2 static stages) correctness + microbench + fp8 8B step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -k fp8 -x > gpurun_out/fp8_tests_e.log 2>&1; rc=$?
echo "fp8 tests rc=$rc"; tail -3 gpurun_out/fp8_tests_e.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/bench_gemm_v2b.log 2>&1; rc=$?
echo "gemm v2b rc=$rc"; cut -c1-220 gpurun_out/bench_gemm_v2b.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --precision fp8 > gpurun_out/bench_8b_fp8_e.log 2>&1; rc=$?
echo "bench fp8 rc=$rc"; tail -1 gpurun_out/bench_8b_fp8_e.log
exit $rc
