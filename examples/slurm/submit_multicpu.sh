#!/bin/bash
# CPU-only data parallel over gloo: N nodes, one process per node.
#SBATCH --job-name=multicpu
#SBATCH --nodes=2
#SBATCH --ntasks-per-node=1
#SBATCH --cpus-per-task=64
#SBATCH --output=%x-%j.out
set -e
head_node_ip=$(scontrol show hostnames "$SLURM_JOB_NODELIST" | head -n 1)
export LAUNCHER="accelerate-amd launch --cpu --num_processes $SLURM_NNODES --num_machines $SLURM_NNODES \
    --rdzv_backend c10d --main_process_ip $head_node_ip --main_process_port 29500"
srun bash -c "$LAUNCHER --machine_rank \$SLURM_NODEID examples/nlp_example.py --cpu"
