#!/bin/bash
# One node, 8 MI355X, one process per GPU (RCCL over xGMI).
#SBATCH --job-name=multigpu
#SBATCH --nodes=1
#SBATCH --ntasks-per-node=1
#SBATCH --gres=gpu:8
#SBATCH --cpus-per-task=128
#SBATCH --output=%x-%j.out
set -e
export HSA_ENABLE_IPC_MODE_LEGACY=0   # dmabuf IPC for RCCL peer buffers
export SCRIPT=${SCRIPT:-examples/complete_nlp_example.py}
export SCRIPT_ARGS=${SCRIPT_ARGS:-"--mixed_precision bf16 --output_dir ${PWD}/out --with_tracking"}
accelerate-amd launch --num_processes 8 --mixed_precision bf16 $SCRIPT $SCRIPT_ARGS
