"""Pipeline-parallel inference of BERT (parity: reference examples/inference/pippy/bert.py, which splits
bert-base-uncased at its middle encoder layer). `prepare_pippy` cuts the encoder stack over the processes.

    accelerate-amd launch --cpu --num_processes 2 examples/inference/pippy/bert.py --cpu
"""

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _hf_common import run  # noqa: E402


def build(full: bool):
    import transformers as tf

    cfg = tf.BertConfig() if full else tf.BertConfig(vocab_size=128, hidden_size=64, num_hidden_layers=4,
                                                      num_attention_heads=4, intermediate_size=96,
                                                      max_position_embeddings=64)
    ids = torch.randint(1, cfg.vocab_size, (4, 16 if not full else 128), generator=torch.Generator().manual_seed(1))
    return tf.BertForMaskedLM(cfg), {"input_ids": ids, "attention_mask": torch.ones_like(ids)}


if __name__ == "__main__":
    run(build)
