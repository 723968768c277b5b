#!/bin/bash
# Stall anatomy of the attention kernels (pass 1, <= 8 SQ counters) and their L2 locality (pass 2, 3 TCC):
#   gpurun -- bash tools/pmc_attn.sh [bench_attn args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
CTR="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"
rm -rf gpurun_out/pmc/attn_stall
timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d gpurun_out/pmc/attn_stall -o run -- python3 tools/bench_attn.py --iters 2 "$@" > gpurun_out/pmc/attn_stall.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 gpurun_out/pmc/attn_stall.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py --stall gpurun_out/pmc/attn_stall
# pass 2: L2 locality of the K/V (Q/dO) streams: TCC hit rate and fabric read requests (3 TCC + 2 SQ + 1 GRBM)
CTR2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
rm -rf gpurun_out/pmc/attn_cache
timeout -s KILL 120 rocprofv3 --pmc $CTR2 --output-format csv -d gpurun_out/pmc/attn_cache -o run -- python3 tools/bench_attn.py --iters 2 "$@" > gpurun_out/pmc/attn_cache.log 2>&1
rc=$?; echo "pmc2 rc=$rc"; tail -3 gpurun_out/pmc/attn_cache.log | cut -c1-300
[ $rc -eq 0 ] && python3 tools/pmc_summary.py --cache gpurun_out/pmc/attn_cache
exit $rc
