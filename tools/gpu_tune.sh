#!/bin/bash
# hipBLASLt per-shape search (progress per shape), then a bench with the resulting table.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=0
timeout -k 10 1500 python tools/tune_gemms.py --model llama3-8b --tokens 8192 --out gpurun_out/tunableop_gfx950.csv --seed-table accelerate_hpc_test_amd/ops/tuned/tunableop_gfx950.csv; rc=$?
echo "tune rc=$rc"
python tools/tune_gemms.py --merge gpurun_out/tunableop_gfx950.csv accelerate_hpc_test_amd/ops/tuned/tunableop_gfx950.csv
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --gemm-tuning auto --gemm-table gpurun_out/tunableop_gfx950.csv > gpurun_out/bench_tuned.log 2>&1; rc=$?
echo "tuned bench rc=$rc"; tail -1 gpurun_out/bench_tuned.log
exit $rc
