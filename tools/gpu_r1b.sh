#!/bin/bash
# Round-1 pass B: fp8 8B bench, kernel profile of the bf16 step, `accelerate-amd test` on one GPU.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof_b
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --precision fp8 > gpurun_out/bench_8b_fp8.log 2>&1; rc=$?
echo "bench fp8 rc=$rc"; tail -2 gpurun_out/bench_8b_fp8.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m accelerate_hpc_test_amd.commands.accelerate_cli test > gpurun_out/accel_test.log 2>&1; rc=$?
echo "accelerate test rc=$rc"; tail -3 gpurun_out/accel_test.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_b_bench.log 2>&1; rc=$?
echo "prof rc=$rc"; tail -1 gpurun_out/prof_b_bench.log
exit $rc
