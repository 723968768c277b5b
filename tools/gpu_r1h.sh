#!/bin/bash
# Round-1 pass H: 8B FSDP with fp32-direct fused wgrad, Mixtral fp8 (256-row expert padding) + kernel profile, 70B dispatch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-700
  [ $rc -eq 0 ] || exit $rc
}
run bench_8b_direct 600 python bench.py --steps 5 --warmup 2
run bench_mixtral_fp8_pad256 600 python bench.py --model mixtral-8x7b-4l --steps 3 --warmup 2 --precision fp8
export TMPDIR=/tmp
run prof_mixtral_fp8 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mixtral_fp8 -o run -- python3 bench.py --model mixtral-8x7b-4l --steps 2 --warmup 1 --precision fp8
run bench_70b_gpu 900 python tools/bench_big_model.py --model llama3-70b --tokens 2048 --iters 3
run bench_70b_offload 900 python tools/bench_big_model.py --model llama3-70b --gpu-mem 100GiB --tokens 2048 --iters 3
