"""Pipeline-parallel inference of GPT-2 for sequence classification (parity: reference
examples/inference/pippy/gpt2.py, `GPT2ForSequenceClassification`).

    accelerate-amd launch --cpu --num_processes 2 examples/inference/pippy/gpt2.py --cpu
"""

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _hf_common import run  # noqa: E402


def build(full: bool):
    import transformers as tf

    cfg = tf.GPT2Config(pad_token_id=0) if full else tf.GPT2Config(vocab_size=128, n_embd=64, n_layer=4, n_head=4,
                                                                    n_positions=64, num_labels=3, pad_token_id=0)
    ids = torch.randint(1, cfg.vocab_size, (4, 16 if not full else 128), generator=torch.Generator().manual_seed(1))
    return tf.GPT2ForSequenceClassification(cfg), {"input_ids": ids}


if __name__ == "__main__":
    run(build)
