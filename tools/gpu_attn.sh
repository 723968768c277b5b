#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -rf -k "flash or extension" --co -q > gpurun_out/kernels_attn.log 2>&1; rc=$?
echo "attn tests rc=$rc"; tail -5 gpurun_out/kernels_attn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_attn.py > gpurun_out/bench_attn.log 2>&1; rc=$?
echo "attn bench rc=$rc"; tail -3 gpurun_out/bench_attn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_8b.log 2>&1; rc=$?
echo "bench_8b rc=$rc"; tail -2 gpurun_out/bench_8b.log
exit $rc
