"""Data-parallel batched generation: the prompt list is split across processes with `split_between_processes`,
each rank generates greedily for its share, and the results are gathered on the main process (parity: reference
examples/inference/distributed/phi2.py — same split / pad / gather pattern, a random-init Llama instead of a
downloaded checkpoint).

    accelerate-amd launch --num_processes 8 examples/inference/distributed/llama_generation.py
    accelerate-amd launch --cpu --num_processes 2 examples/inference/distributed/llama_generation.py --cpu
"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))

from accelerate_hpc_test_amd import PartialState  # noqa: E402
from accelerate_hpc_test_amd.models.llama import LlamaConfig, LlamaForCausalLM  # noqa: E402
from accelerate_hpc_test_amd.utils import gather_object, set_seed  # noqa: E402


@torch.no_grad()
def greedy(model, ids, new_tokens):
    for _ in range(new_tokens):
        nxt = model(ids).logits[:, -1].argmax(-1, keepdim=True)
        ids = torch.cat([ids, nxt], dim=1)
    return ids


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--n_prompts", type=int, default=10)
    p.add_argument("--new_tokens", type=int, default=8)
    args = p.parse_args(argv)
    state = PartialState(cpu=args.cpu)
    cfg = LlamaConfig(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256)
    set_seed(0)
    model = LlamaForCausalLM(cfg)
    model.init_weights()
    model.eval().to(state.device)
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, cfg.vocab_size, (int(torch.randint(4, 12, (1,), generator=g)),), generator=g).tolist()
               for _ in range(args.n_prompts)]
    # each rank gets a contiguous share (the last ones may be padded with a repeat of the final prompt)
    with state.split_between_processes(list(enumerate(prompts)), apply_padding=True) as mine:
        done = []
        for idx, prompt in mine:
            ids = torch.tensor([prompt], device=state.device)
            done.append((idx, greedy(model, ids, args.new_tokens)[0, len(prompt):].tolist()))
    results = gather_object(done)
    by_idx = None
    if state.is_main_process:
        by_idx = dict(results)  # padding duplicates collapse onto their index
        assert sorted(by_idx) == list(range(args.n_prompts)), sorted(by_idx)
        for i in range(min(3, args.n_prompts)):
            print(f"prompt {i}: {prompts[i]} -> {by_idx[i]}")
        print(f"generated {args.n_prompts} completions on {state.num_processes} process(es)")
    # tear the group down on every rank together: a rank that exits while its peer is still inside a gloo call
    # can abort in the transport's destructor
    state.wait_for_everyone()
    state.destroy_process_group()
    return by_idx


if __name__ == "__main__":
    main()
