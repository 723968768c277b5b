"""Pipeline-parallel inference of T5 (parity: reference examples/inference/pippy/t5.py, `T5ForConditionalGeneration`
split between the encoder and the decoder). Both block lists (encoder.block, decoder.block) are staged, the shared
embedding is replicated on every stage.

    accelerate-amd launch --cpu --num_processes 2 examples/inference/pippy/t5.py --cpu
"""

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _hf_common import run  # noqa: E402


def build(full: bool):
    import transformers as tf

    cfg = (tf.T5Config(decoder_start_token_id=0) if full else
           tf.T5Config(vocab_size=128, d_model=64, d_ff=96, d_kv=16, num_layers=2, num_decoder_layers=2, num_heads=4,
                       decoder_start_token_id=0, pad_token_id=0))
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(1, cfg.vocab_size, (4, 16 if not full else 128), generator=g)
    dec = torch.randint(1, cfg.vocab_size, (4, 8), generator=g)
    return tf.T5ForConditionalGeneration(cfg), {"input_ids": ids, "decoder_input_ids": dec}


if __name__ == "__main__":
    run(build)
