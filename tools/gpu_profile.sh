#!/bin/bash
# Kernel-level profile of the 8B FSDP bf16 step (rocprofv3 kernel trace + stats).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 2 ${BENCH_ARGS} > gpurun_out/prof_bench.log 2>&1; rc=$?
echo "prof rc=$rc"; tail -3 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
