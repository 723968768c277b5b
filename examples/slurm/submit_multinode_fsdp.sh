#!/bin/bash
# FSDP2 across N nodes x 8 MI355X with the config in fsdp_config.yaml (bench.py = the Llama-3-8B headline step).
#SBATCH --job-name=multinode-fsdp
#SBATCH --nodes=2
#SBATCH --ntasks-per-node=1
#SBATCH --gres=gpu:8
#SBATCH --cpus-per-task=128
#SBATCH --output=%x-%j.out
set -e
export HSA_ENABLE_IPC_MODE_LEGACY=0
GPUS_PER_NODE=8
head_node_ip=$(scontrol show hostnames "$SLURM_JOB_NODELIST" | head -n 1)
export LAUNCHER="accelerate-amd launch --config_file examples/slurm/fsdp_config.yaml \
    --num_processes $((SLURM_NNODES * GPUS_PER_NODE)) --num_machines $SLURM_NNODES \
    --rdzv_backend c10d --main_process_ip $head_node_ip --main_process_port 29500"
srun bash -c "$LAUNCHER --machine_rank \$SLURM_NODEID bench.py --gpus $((SLURM_NNODES * GPUS_PER_NODE)) --steps 20 --warmup 5"
