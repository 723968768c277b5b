#!/bin/bash
# rocprofv3 hardware-counter passes (one pass per block budget: <= 8 SQ, 2 GRBM) over the attention and GEMM
# microbenchmarks: MFMA busy cycles vs SQ busy cycles (matrix-core utilisation), LDS instructions / bank conflicts /
# LDS-array activity (the LDS staging of every hand-written kernel). Summaries: tools/prof_summary.py --pmc.
#   gpurun --timeout 900 -- bash tools/pmc_steps.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
CTR="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1
echo "list rc=$?"
pass() {  # name cmd...
  local name=$1; shift
  rm -rf "gpurun_out/pmc/$name"
  timeout -s KILL 180 rocprofv3 --pmc $CTR --output-format csv -d "gpurun_out/pmc/$name" -o run -- "$@" > "gpurun_out/pmc/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -2 "gpurun_out/pmc/$name.log" | cut -c1-300; return $rc
}
pass attn python3 tools/bench_attn.py --iters 2 && pass gemm python3 tools/bench_gemm.py --iters 2
