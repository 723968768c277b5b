#!/bin/bash
# Round-1 pass G: fp8 grouped-expert test, Mixtral-8x7B (4-layer slice) fp8, Llama-3-8B DDP bf16 (1 GPU), 70B dispatch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
run bench_8b_fusedwgrad 600 python bench.py --steps 5 --warmup 2
run test_moe_fp8 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "moe or fp8"
run bench_mixtral_fp8 600 python bench.py --model mixtral-8x7b-4l --steps 3 --warmup 2 --precision fp8
run bench_8b_ddp 600 python bench.py --parallel ddp --steps 5 --warmup 2
run bench_70b_gpu 900 python tools/bench_big_model.py --model llama3-70b --tokens 2048 --iters 3
run bench_70b_offload 900 python tools/bench_big_model.py --model llama3-70b --gpu-mem 100GiB --tokens 2048 --iters 3
