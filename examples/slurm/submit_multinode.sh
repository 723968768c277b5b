#!/bin/bash
# N nodes x 8 MI355X: srun starts one launcher per node; each launcher starts 8 ranks (torchrun, c10d rendezvous on
# the first node).
#SBATCH --job-name=multinode
#SBATCH --nodes=2
#SBATCH --ntasks-per-node=1
#SBATCH --gres=gpu:8
#SBATCH --cpus-per-task=128
#SBATCH --output=%x-%j.out
set -e
export HSA_ENABLE_IPC_MODE_LEGACY=0
GPUS_PER_NODE=8
head_node_ip=$(scontrol show hostnames "$SLURM_JOB_NODELIST" | head -n 1)
export SCRIPT=${SCRIPT:-examples/complete_nlp_example.py}
export SCRIPT_ARGS=${SCRIPT_ARGS:-"--mixed_precision bf16 --output_dir ${PWD}/out"}
export LAUNCHER="accelerate-amd launch \
    --num_processes $((SLURM_NNODES * GPUS_PER_NODE)) \
    --num_machines $SLURM_NNODES \
    --rdzv_backend c10d \
    --main_process_ip $head_node_ip \
    --main_process_port 29500"
# \$SLURM_NODEID is expanded on each node by the inner shell
srun bash -c "$LAUNCHER --machine_rank \$SLURM_NODEID $SCRIPT $SCRIPT_ARGS"
