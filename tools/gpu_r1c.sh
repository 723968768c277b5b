#!/bin/bash
# Round-1 pass C: hipBLASLt per-shape search for the 8B step, re-measure with the table, fp8 kernel profile.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof_fp8
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1200 python bench.py --steps 2 --warmup 2 --gemm-tuning tune --gemm-table gpurun_out/tunableop_gfx950.csv --verbose > gpurun_out/bench_tune.log 2>&1; rc=$?
echo "tune rc=$rc"; tail -2 gpurun_out/bench_tune.log; ls -la gpurun_out/tunableop_gfx950.csv
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --gemm-tuning auto --gemm-table gpurun_out/tunableop_gfx950.csv > gpurun_out/bench_tuned.log 2>&1; rc=$?
echo "tuned bench rc=$rc"; tail -1 gpurun_out/bench_tuned.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fp8 -o run -- python3 bench.py --steps 2 --warmup 1 --precision fp8 --gemm-tuning off > gpurun_out/prof_fp8_bench.log 2>&1; rc=$?
echo "prof fp8 rc=$rc"; tail -1 gpurun_out/prof_fp8_bench.log
exit $rc
