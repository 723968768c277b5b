#!/bin/bash
# Round-1 pass F: fp8 GEMM 8-wave A/B, Mixtral-8x7B (4-layer slice) FSDP bf16 vs fp8, Llama-3-70B big-model dispatch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ACCELERATE_FP8_GEMM_WAVES=8 timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/bench_gemm_w8.log 2>&1; rc=$?
echo "gemm w8 rc=$rc"; cut -c1-60,150-220 gpurun_out/bench_gemm_w8.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --model mixtral-8x7b-4l --steps 3 --warmup 2 --precision bf16 > gpurun_out/bench_mixtral_bf16.log 2>&1; rc=$?
echo "mixtral bf16 rc=$rc"; tail -1 gpurun_out/bench_mixtral_bf16.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --model mixtral-8x7b-4l --steps 3 --warmup 2 --precision fp8 > gpurun_out/bench_mixtral_fp8.log 2>&1; rc=$?
echo "mixtral fp8 rc=$rc"; tail -1 gpurun_out/bench_mixtral_fp8.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/bench_big_model.py --model llama3-70b --tokens 2048 --iters 3 > gpurun_out/bench_70b_gpu.log 2>&1; rc=$?
echo "70b all-gpu rc=$rc"; tail -1 gpurun_out/bench_70b_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/bench_big_model.py --model llama3-70b --gpu-mem 100GiB --tokens 2048 --iters 3 > gpurun_out/bench_70b_offload.log 2>&1; rc=$?
echo "70b offload rc=$rc"; tail -1 gpurun_out/bench_70b_offload.log
exit $rc
