#!/bin/bash
# Named GPU steps for `gpurun`: each runs under its own time limit, logs to gpurun_out/<step>.log, and the first
# failing step ends the call (no retries, nothing more on the GPU after a fault or a timeout).
#
#   gpurun --timeout 1200 -- bash tools/gpu_steps.sh tests smoke bench8b prof8b
#
# Extra bench flags for the bench*/prof* steps: BENCH_ARGS="--prefetch 2" bash tools/gpu_steps.sh bench8b
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name (limit ${t}s)"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-900
  [ $rc -eq 0 ] || exit $rc
}
prof() {  # name timeout bench-args...   (PROF_EXTRA: more rocprofv3 trace flags, e.g. --memory-copy-trace)
  local name=$1 t=$2; shift 2
  rm -rf "gpurun_out/$name"
  run "$name" "$t" rocprofv3 --kernel-trace $PROF_EXTRA --stats --output-format csv -d "gpurun_out/$name" -o run -- python3 "$@"
  python3 tools/prof_summary.py "gpurun_out/$name" > "gpurun_out/$name.md" && head -40 "gpurun_out/$name.md"
  python3 tools/prof_overlap.py "gpurun_out/$name" --pattern "${OVERLAP_PATTERN:-nccl|rccl}" > "gpurun_out/${name}_overlap.md" && cat "gpurun_out/${name}_overlap.md"
  find "gpurun_out/$name" -name '*kernel_trace.csv' -size +20M -delete  # keep the pull under the 64 MiB cap
}
for step in "$@"; do
  case $step in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench20) run bench20 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_fp8) run bench20_fp8 600 python bench.py --gpus 1 --steps 20 --warmup 5 --precision fp8 ;;
    bench20_mxfp8) run bench20_mxfp8 600 python bench.py --gpus 1 --steps 20 --warmup 5 --precision mxfp8 ;;
    bench20_adambf16) run bench20_adambf16 600 python bench.py --gpus 1 --steps 20 --warmup 5 --adam-states bf16 ;;
    bench20_asm) ACCELERATE_ASM_BF16_GEMM=1 run bench20_asm 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_abmn) ACCELERATE_ASM_WGRAD_ABMN=1 run bench20_abmn 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_abmn_b) ACCELERATE_ASM_WGRAD_ABMN=1 run bench20_abmn_b 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_dgamn) ACCELERATE_ASM_DGRAD_AMN=1 run bench20_dgamn 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_dgamn_b) ACCELERATE_ASM_DGRAD_AMN=1 run bench20_dgamn_b 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_dgbl) ACCELERATE_ASM_DGRAD_AMN=0 run bench20_dgbl 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_dgbl_b) ACCELERATE_ASM_DGRAD_AMN=0 run bench20_dgbl_b 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_noamn) ACCELERATE_ASM_WGRAD_AMN=0 run bench20_noamn 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_b) run bench20_b 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_noamn_b) ACCELERATE_ASM_WGRAD_AMN=0 run bench20_noamn_b 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    newtests) run newtests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_async_checkpoint.py -k "upcast or layerwise or amn or grouped or moe or async or native_writer" ;;
    mr_sp) run mr_sp 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multirank.py -k "tp" ;;
    bench20_asmw) ACCELERATE_ASM_BF16_GEMM=wgrad run bench20_asmw 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_dyt) ACCELERATE_WGRAD_DYT=1 run bench20_dyt 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    prof8b_dyt) ACCELERATE_WGRAD_DYT=1 prof prof8b_dyt 600 bench.py --steps 3 --warmup 2 $BENCH_ARGS ;;
    prof8b_asmw) ACCELERATE_ASM_BF16_GEMM=wgrad prof prof8b_asmw 600 bench.py --steps 3 --warmup 2 $BENCH_ARGS ;;
    bench20_fp8bl) ACCELERATE_FP8_GEMM=blaslt run bench20_fp8bl 600 python bench.py --gpus 1 --steps 20 --warmup 5 --precision fp8 ;;
    bench20_fp8hip) ACCELERATE_FP8_GEMM=hip run bench20_fp8hip 600 python bench.py --gpus 1 --steps 20 --warmup 5 --precision fp8 ;;
    bench8b) run bench8b 600 python bench.py --steps 5 --warmup 2 $BENCH_ARGS ;;
    bench8b_nodgradwt) ACCELERATE_DGRAD_WT=0 run bench8b_nodgradwt 600 python bench.py --steps 5 --warmup 2 $BENCH_ARGS ;;
    transpose) run transpose 300 python tools/bench_transpose.py && ACCELERATE_TRANSPOSE128=0 run transpose_old 300 python tools/bench_transpose.py ;;
    ktest) run ktest 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "${KTEST:-transpose}" ;;
    tune_step1) run tune_step 900 python bench.py --gemm-tuning tune --gemm-table gpurun_out/tunableop_step.csv --steps 1 --warmup 2 && \
               cp accelerate_hpc_test_amd/ops/tuned/tunableop_gfx950.csv gpurun_out/tunableop_merged.csv && \
               python tools/tune_gemms.py --merge gpurun_out/tunableop_merged.csv gpurun_out/tunableop_step.csv && \
               run bench_tuned 600 python bench.py --gpus 1 --steps 20 --warmup 5 --gemm-table gpurun_out/tunableop_merged.csv && \
               run bench_untuned 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    tune_step) run tune_step 900 python bench.py --gemm-tuning tune --gemm-table gpurun_out/tunableop_step.csv --steps 1 --warmup 2 && \
               run tune_step_sharded 900 python bench.py --gemm-tuning tune --gemm-table gpurun_out/tunableop_step_sharded.csv --steps 1 --warmup 2 --fsdp-force-sharded && \
               cp accelerate_hpc_test_amd/ops/tuned/tunableop_gfx950.csv gpurun_out/tunableop_merged.csv && \
               python tools/tune_gemms.py --merge gpurun_out/tunableop_merged.csv gpurun_out/tunableop_step.csv gpurun_out/tunableop_step_sharded.csv && \
               run bench_tuned 600 python bench.py --steps 5 --warmup 2 --gemm-table gpurun_out/tunableop_merged.csv && \
               run bench_untuned 600 python bench.py --steps 5 --warmup 2 ;;
    wgrad_layout) run wgrad_layout 300 python tools/bench_wgrad_layout.py ;;
    wgrad_wide) ACCELERATE_BLASLT_CANDIDATES=${CANDIDATES:-256} run wgrad_wide 300 python tools/bench_wgrad_layout.py ;;
    bench20_wide) ACCELERATE_BLASLT_CANDIDATES=${CANDIDATES:-256} run bench20_wide 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench8b_noblaslt) ACCELERATE_BLASLT_WGRAD=0 run bench8b_noblaslt 600 python bench.py --steps 5 --warmup 2 $BENCH_ARGS ;;
    bench8b_blaslt) ACCELERATE_BLASLT_WGRAD=1 run bench8b_blaslt 600 python bench.py --steps 5 --warmup 2 $BENCH_ARGS ;;
    bench8b_nooverlap) run bench8b_nooverlap 600 python bench.py --steps 5 --warmup 2 --optimizer-overlap off $BENCH_ARGS ;;
    bench8b_sharded) run bench8b_sharded 600 python bench.py --steps 5 --warmup 2 --fsdp-force-sharded $BENCH_ARGS ;;
    prof8b_sharded) OVERLAP_PATTERN="nccl|rccl|copyBuffer" PROF_EXTRA=--memory-copy-trace prof prof8b_sharded 600 bench.py --steps 3 --warmup 2 --fsdp-force-sharded $BENCH_ARGS ;;
    bench8b_offload) run bench8b_offload 900 python bench.py --steps 2 --warmup 1 --fsdp-cpu-offload --verbose $BENCH_ARGS ;;
    long32k) run long32k 900 python bench.py --seq 32768 --steps 2 --warmup 1 --activation-checkpointing --verbose $BENCH_ARGS ;;
    long64k) run long64k 900 python bench.py --seq 65536 --steps 2 --warmup 1 --activation-checkpointing --verbose $BENCH_ARGS ;;
    bench8b_fp8) run bench8b_fp8 600 python bench.py --steps 5 --warmup 2 --precision fp8 $BENCH_ARGS ;;
    mxprobe) run mxprobe 300 python tools/debug/mx_blaslt_probe.py ;;
    bench8b_mxfp8) run bench8b_mxfp8 600 python bench.py --steps 5 --warmup 2 --precision mxfp8 $BENCH_ARGS ;;
    bench8b_ddp) run bench8b_ddp 600 python bench.py --parallel ddp --steps 5 --warmup 2 $BENCH_ARGS ;;
    bench8b_ddp_forced) run bench8b_ddp_forced 600 python bench.py --parallel ddp --ddp-force --steps 5 --warmup 2 $BENCH_ARGS ;;
    prof_ddp_forced) prof prof_ddp_forced 600 bench.py --parallel ddp --ddp-force --steps 3 --warmup 2 $BENCH_ARGS ;;
    prof_ddp) prof prof_ddp 600 bench.py --parallel ddp --steps 3 --warmup 2 $BENCH_ARGS ;;
    prof_mixtral8l_bf16) prof prof_mixtral8l_bf16 600 bench.py --model mixtral-8x7b-8l --steps 2 --warmup 1 ;;
    mix8_bf16_grid0) ACCELERATE_FP8ASM_GRID=0 run mix8_bf16_grid0 600 python bench.py --model mixtral-8x7b-8l --steps 5 --warmup 2 --verbose $BENCH_ARGS ;;
    mix8_fp8_grid0) ACCELERATE_FP8ASM_GRID=0 run mix8_fp8_grid0 600 python bench.py --model mixtral-8x7b-8l --steps 5 --warmup 2 --precision fp8 --verbose $BENCH_ARGS ;;
    bench20_fp8_grid0) ACCELERATE_FP8ASM_GRID=0 run bench20_fp8_grid0 600 python bench.py --gpus 1 --steps 20 --warmup 5 --precision fp8 ;;
    prof8b_sharded_grid0) ACCELERATE_FP8ASM_GRID=0 OVERLAP_PATTERN="nccl|rccl|copyBuffer" PROF_EXTRA=--memory-copy-trace prof prof8b_sharded_grid0 600 bench.py --steps 3 --warmup 2 --fsdp-force-sharded $BENCH_ARGS ;;
    mix8_bf16) run mix8_bf16 600 python bench.py --model mixtral-8x7b-8l --steps 5 --warmup 2 --verbose $BENCH_ARGS ;;
    mix8_fp8) run mix8_fp8 600 python bench.py --model mixtral-8x7b-8l --steps 5 --warmup 2 --precision fp8 --verbose $BENCH_ARGS ;;
    mix8_bf16_asmall) ACCELERATE_MOE_ASM_BF16=fwd,wgrad,dgrad run mix8_bf16_asmall 600 python bench.py --model mixtral-8x7b-8l --steps 5 --warmup 2 --verbose $BENCH_ARGS ;;
    mix8_bf16_asmnone) ACCELERATE_MOE_ASM_BF16=none run mix8_bf16_asmnone 600 python bench.py --model mixtral-8x7b-8l --steps 5 --warmup 2 --verbose $BENCH_ARGS ;;
    mix8_bf16_asmfwd) ACCELERATE_MOE_ASM_BF16=fwd run mix8_bf16_asmfwd 600 python bench.py --model mixtral-8x7b-8l --steps 5 --warmup 2 --verbose $BENCH_ARGS ;;
    mix8_bf16_nonn) ACCELERATE_MOE_DGRAD_NN=0 run mix8_bf16_nonn 600 python bench.py --model mixtral-8x7b-8l --steps 5 --warmup 2 --verbose $BENCH_ARGS ;;
    mix8_fp8_noroute) ACCELERATE_MOE_ROUTE_HIP=0 run mix8_fp8_noroute 600 python bench.py --model mixtral-8x7b-8l --steps 5 --warmup 2 --precision fp8 --verbose $BENCH_ARGS ;;
    mix8_fp8_nocastt) ACCELERATE_MOE_FP8_CAST_T=0 run mix8_fp8_nocastt 600 python bench.py --model mixtral-8x7b-8l --steps 5 --warmup 2 --precision fp8 --verbose $BENCH_ARGS ;;
    mix8_fp8_blaslt) ACCELERATE_MOE_FP8_BLASLT=1 run mix8_fp8_blaslt 600 python bench.py --model mixtral-8x7b-8l --steps 5 --warmup 2 --precision fp8 --verbose $BENCH_ARGS ;;
    moegemm) run moegemm 300 python tools/bench_moe_gemm.py ;;
    prof_mix8_fp8) prof prof_mix8_fp8 600 bench.py --model mixtral-8x7b-8l --steps 2 --warmup 2 --precision fp8 ;;
    prof_mix8_fp8_blaslt) ACCELERATE_MOE_FP8_BLASLT=1 prof prof_mix8_fp8_blaslt 600 bench.py --model mixtral-8x7b-8l --steps 2 --warmup 2 --precision fp8 ;;
    mixtral_bf16) run mixtral_bf16 600 python bench.py --model mixtral-8x7b-4l --steps 3 --warmup 2 $BENCH_ARGS ;;
    mixtral_fp8) run mixtral_fp8 600 python bench.py --model mixtral-8x7b-4l --steps 3 --warmup 2 --precision fp8 $BENCH_ARGS ;;
    prof8b) prof prof8b 600 bench.py --steps 3 --warmup 2 $BENCH_ARGS ;;
    prof8b_fp8) prof prof8b_fp8 600 bench.py --steps 3 --warmup 2 --precision fp8 $BENCH_ARGS ;;
    prof_mixtral_fp8) prof prof_mixtral_fp8 600 bench.py --model mixtral-8x7b-4l --steps 2 --warmup 1 --precision fp8 ;;
    prof_mixtral_bf16) prof prof_mixtral_bf16 600 bench.py --model mixtral-8x7b-4l --steps 2 --warmup 1 ;;
    moetests) run moetests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "grouped or moe or transpose" ;;
    attn) run attn 300 python tools/bench_attn.py --no-sdpa ;;
    attn_fwd4) run ktest_fwd4 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fwd_w4" && \
               ACCELERATE_ATTN_FWD_W4=1 run ktest_attn_fwd4 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention or context_parallel" && \
               run attn_fwd4 300 python tools/bench_attn.py --no-sdpa --fwd-variants 0,1 --rounds 3 ;;
    attn_w4) run ktest_attn 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention or context_parallel" && \
             run attn_w4 300 python tools/bench_attn.py --no-sdpa && ACCELERATE_ATTN_DKDV=8 run attn_w8 300 python tools/bench_attn.py --no-sdpa && \
             ACCELERATE_ATTN_DKDV_SCHED=1 run attn_w4s1 300 python tools/bench_attn.py --no-sdpa ;;
    attn_dkdv) run ktest_attn 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention or context_parallel" && \
               ACCELERATE_ATTN_DQ_W4=1 ACCELERATE_ATTN_DKDV_SCHED=${KTEST_SCHED:-2} run ktest_attn_s2 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention or context_parallel" && \
               run attn_dkdv 300 python tools/bench_attn.py --no-sdpa --dkdv-variants ${DKDV_VARIANTS:-8:8:0,8:4:0,8:4:2,8:4:3,4:4:0,4:4:2} ;;
    attn_dq128) run attn_dq64 300 python tools/bench_attn.py --no-sdpa --dkdv-variants 8:8:0,8:4:6 && \
                ACCELERATE_ATTN_DQ_KEYS=128 run attn_dq128 300 python tools/bench_attn.py --no-sdpa --dkdv-variants 8:8:0,8:4:6 ;;
    attn_var) for v in ${ATTN_VARIANTS:-0 2 3}; do ACCELERATE_ATTN_DKDV_SCHED=$v run ktest_attn_s$v 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention or context_parallel" && \
              ACCELERATE_ATTN_DKDV_SCHED=$v run attn_s$v 300 python tools/bench_attn.py --no-sdpa || exit 1; done ;;
    prof_attn) prof prof_attn 300 tools/bench_attn.py --no-sdpa --iters 5 && \
               ACCELERATE_ATTN_DKDV_SCHED=1 prof prof_attn_s1 300 tools/bench_attn.py --no-sdpa --iters 5 ;;
    attn_k128) ACCELERATE_ATTN_FWD_KEYS=128 run attn_k128 300 python tools/bench_attn.py --no-sdpa ;;
    ktest_k128) ACCELERATE_ATTN_FWD_KEYS=128 run ktest_k128 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention or context_parallel" ;;
    ktest_dq128) ACCELERATE_ATTN_DQ_KEYS=128 run ktest_dq128 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention or context_parallel" ;;
    attn_dq128) ACCELERATE_ATTN_DQ_KEYS=128 run attn_dq128 300 python tools/bench_attn.py --no-sdpa ;;
    bench20_dq128) ACCELERATE_ATTN_DQ_KEYS=128 run bench20_dq128 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_fwd4) ACCELERATE_ATTN_FWD_W4=1 run bench20_fwd4 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_fwd4_b) ACCELERATE_ATTN_FWD_W4=1 run bench20_fwd4_b 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_adamg) ACCELERATE_ADAM_NT=1 run bench20_adamg 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_adamnt) ACCELERATE_ADAM_NT=2 run bench20_adamnt 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    adam_tests) ACCELERATE_ADAM_NT=2 run adam_tests_nt 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "adam" && \
                ACCELERATE_ADAM_NT=1 run adam_tests_g 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "adam" ;;
    bench20_sharded_rsp0) ACCELERATE_FSDP_RS_PRIORITY=0 run bench20_sharded_rsp0 600 python bench.py --gpus 1 --steps 20 --warmup 5 --fsdp-force-sharded ;;
    split_tests) run split_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "amn" ;;
    bench20_nosplit) ACCELERATE_ASM_SPLIT_TAIL=0 run bench20_nosplit 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_nosplit_b) ACCELERATE_ASM_SPLIT_TAIL=0 run bench20_nosplit_b 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_grid0) ACCELERATE_FP8ASM_GRID=0 run bench20_grid0 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_sharded_grid0) ACCELERATE_FP8ASM_GRID=0 run bench20_sharded_grid0 600 python bench.py --gpus 1 --steps 20 --warmup 5 --fsdp-force-sharded ;;
    bench20_sharded_dgbl) ACCELERATE_ASM_DGRAD_AMN=0 run bench20_sharded_dgbl 600 python bench.py --gpus 1 --steps 20 --warmup 5 --fsdp-force-sharded ;;
    bench20_sharded) run bench20_sharded 600 python bench.py --gpus 1 --steps 20 --warmup 5 --fsdp-force-sharded ;;
    bench20_sharded_nors) run bench20_sharded_nors 600 python bench.py --gpus 1 --steps 20 --warmup 5 --fsdp-force-sharded --reshard-after-forward off ;;
    bench20_ovl) run bench20_ovl 600 python bench.py --gpus 1 --steps 20 --warmup 5 --optimizer-overlap on ;;
    bench20_fp8_ovl) run bench20_fp8_ovl 600 python bench.py --gpus 1 --steps 20 --warmup 5 --precision fp8 --optimizer-overlap on ;;
    bench20_fp8_amaxoff) ACCELERATE_FP8_AMAX_IN_ADAM=0 run bench20_fp8_amaxoff 600 python bench.py --gpus 1 --steps 20 --warmup 5 --precision fp8 ;;
    bench20_fp8_pret) ACCELERATE_FP8_PRETRANSPOSE=1 run bench20_fp8_pret 600 python bench.py --gpus 1 --steps 20 --warmup 5 --precision fp8 ;;
    bench20_dgradbl) ACCELERATE_DGRAD_BLASLT=1 run bench20_dgradbl 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20_k128) ACCELERATE_ATTN_FWD_KEYS=128 run bench20_k128 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    attn_long) run attn_long 300 python tools/bench_attn.py --S 32768 --iters 3 ;;
    pmc_attn) run pmc_attn 200 bash tools/pmc_attn.sh ;;
    pmc_attn_var) run pmc_attn_var 200 bash tools/pmc_attn.sh --no-sdpa --dkdv-variants 8:4:2,4:4:2 --rounds 1 ;;
    gemm) run gemm 300 python tools/bench_gemm.py ;;
    asmdiag) run asmdiag 120 python tools/debug/fp8asm_diag.py ;;
    gemm_grp) run gemm_grp 400 python tools/bench_gemm.py --variants ${GEMM_VARIANTS:-bl,18,18g1,18g2,18g8,18g16} --no-bf16 --no-scaled-mm --rounds 3 ;;
    gprobe) run gprobe 300 python tools/bench_gemm_probe.py ;;
    g8test) run g8test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm8" ;;
    trprobe) run trprobe 60 tools/microbench/tr_probe ;;
    f8mn) run ktest_f8mn 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fp8_asm_amn" ;;
    f8tests) run f8tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fp8" ;;
    bench20_fp8_nomn) ACCELERATE_FP8_MN=0 run bench20_fp8_nomn 600 python bench.py --gpus 1 --steps 20 --warmup 5 --precision fp8 ;;
    f8tests_spread) ACCELERATE_FP8ASM_SPREAD=1 run f8tests_spread 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fp8" ;;
    bench20_fp8_spread) ACCELERATE_FP8ASM_SPREAD=1 run bench20_fp8_spread 600 python bench.py --gpus 1 --steps 20 --warmup 5 --precision fp8 ;;
    gemm_fp8_spread) ACCELERATE_FP8ASM_SPREAD=1 run gemm_fp8_spread 400 python tools/bench_gemm.py --variants bl,18 --no-bf16 --no-scaled-mm --rounds 3 --check ;;
    bench20_fp8_b) run bench20_fp8_b 600 python bench.py --gpus 1 --steps 20 --warmup 5 --precision fp8 ;;
    amn) run ktest_amn 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "bf16_asm" && \
         run gemm_amn 400 python tools/bench_gemm_amn.py ;;
    gemm_bf16) run ktest_bf16asm 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "bf16_asm" && \
               run gemm_bf16 400 python tools/bench_gemm_bf16.py ;;
    ktest_moe_asm) run ktest_moe_asm 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "grouped or moe or expert" ;;
    ckpt8b) run ckpt8b 900 python tools/ckpt_roundtrip.py ;;
    asmprobe) run asmprobe 120 python tools/debug/fp8asm_probe.py ;;
    mr_tp) run mr_tp 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multirank.py -k "tp" ;;
    gemm_asm) run ktest_asm 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fp8_gemm_v4" && \
              run gemm_asm 400 python tools/bench_gemm.py --variants ${GEMM_VARIANTS:-bl,18,17} --no-bf16 --no-scaled-mm --rounds 3 --check ;;
    pmc_gemm) run pmc_gemm 400 bash tools/pmc_gemm.sh --variants ${GEMM_VARIANTS:-bl,4,8,7} --shapes o,down --iters 2 --rounds 1 --no-bf16 --no-scaled-mm ;;
    dgrad) run dgrad 300 python tools/bench_dgrad.py ;;
    bench8b_dgradbl) ACCELERATE_DGRAD_BLASLT=1 run bench8b_dgradbl 600 python bench.py --steps 5 --warmup 2 $BENCH_ARGS ;;
    mfma_peak) run mfma_peak 60 tools/microbench/mfma_peak ;;
    probe) run probe 60 bash -c 'df -h . /tmp /dev/shm; free -g; nproc; mount | grep -E " /tmp | /dev/shm | / " || true' ;;
    gemm_v4) run ktest_v4 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fp8_gemm_v4 or fp8_gemm_v3 or fp8_gemm_exact" && \
             run gemm_v4 400 python tools/bench_gemm.py --variants ${GEMM_VARIANTS:-bl,4,6,7} --no-bf16 --no-scaled-mm --rounds 3 ;;
    gen_gptj) run gen_gptj 600 python tools/bench_generate.py --model gpt-j-6b ;;
    gen_neox) run gen_neox 600 python tools/bench_generate.py --model gpt-neox-20b --keep-ckpt ;;
    gen_neox_offload) run gen_neox_offload 600 python tools/bench_generate.py --model gpt-neox-20b --gpu-mem 20GiB ;;
    gen_opt30b_offload) run gen_opt30b_offload 900 python tools/bench_generate.py --model opt-30b --gpu-mem 46GiB ;;
    gen_neox_disk) run gen_neox_disk 900 python tools/bench_generate.py --model gpt-neox-20b --gpu-mem 14GiB --cpu-mem 10GiB --disk-offload ;;
    gen_llama70b) run gen_llama70b 900 python tools/bench_generate.py --model llama3-70b --dtype bf16 ;;
    gen70_disk) CK=/dev/shm/acc_ckpt_llama3_70b_bf16; trap 'rm -rf /dev/shm/acc_ckpt_llama3_70b_bf16' EXIT
                run gen70_resident 900 python tools/bench_generate.py --model llama3-70b --dtype bf16 --ckpt-dir $CK && \
                run gen70_offload 900 python tools/bench_generate.py --model llama3-70b --dtype bf16 --ckpt-dir $CK --gpu-mem 100GiB ;;
    big70b) run big70b 900 python tools/bench_big_model.py --model llama3-70b --tokens 2048 --iters 3 ;;
    big70b_offload) run big70b_offload 900 python tools/bench_big_model.py --model llama3-70b --gpu-mem 100GiB --tokens 2048 --iters 3 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
