#!/bin/bash
# Round-1 pass D: TunableOp A/B, fp8 GEMM v2 tests + microbench, kernel profile of the tuned 8B step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof_d
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python tools/ab_tunable.py > gpurun_out/ab_tunable.log 2>&1; rc=$?
echo "ab rc=$rc"; cat gpurun_out/ab_tunable.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -k fp8 -x > gpurun_out/fp8_tests.log 2>&1; rc=$?
echo "fp8 tests rc=$rc"; tail -3 gpurun_out/fp8_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/bench_gemm_v2.log 2>&1; rc=$?
echo "gemm v2 rc=$rc"; cat gpurun_out/bench_gemm_v2.log
[ $rc -eq 0 ] || exit $rc
ACCELERATE_FP8_GEMM_V1=1 timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/bench_gemm_v1.log 2>&1; rc=$?
echo "gemm v1 rc=$rc"; cat gpurun_out/bench_gemm_v1.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_d -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_d_bench.log 2>&1; rc=$?
echo "prof rc=$rc"; tail -1 gpurun_out/prof_d_bench.log
exit $rc
