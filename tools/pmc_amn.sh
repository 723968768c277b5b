#!/bin/bash
# Hardware counters of the MN-major bf16 asm GEMMs (weight / data gradients, tools/bench_gemm_amn.py) against the
# hipBLASLt kernels the same script runs: stall anatomy (8 SQ) and LDS / clock (5 SQ + 1 GRBM), one rocprofv3 --pmc
# pass each.
#   gpurun -- bash tools/pmc_amn.sh [bench_gemm_amn args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
ARGS=${@:---shapes qkv,gate_up,down --iters 2 --rounds 1}
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
rm -rf gpurun_out/pmc/amn_stall gpurun_out/pmc/amn_lds
timeout -s KILL 150 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmc/amn_stall -o run -- python3 tools/bench_gemm_amn.py $ARGS > gpurun_out/pmc/amn_stall.log 2>&1
rc=$?; echo "pmc1 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmc/amn_lds -o run -- python3 tools/bench_gemm_amn.py $ARGS > gpurun_out/pmc/amn_lds.log 2>&1
rc=$?; echo "pmc2 rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py --stall gpurun_out/pmc/amn_stall > gpurun_out/pmc/amn_stall.md
python3 tools/pmc_summary.py gpurun_out/pmc/amn_lds > gpurun_out/pmc/amn_lds.md
cat gpurun_out/pmc/amn_stall.md gpurun_out/pmc/amn_lds.md
