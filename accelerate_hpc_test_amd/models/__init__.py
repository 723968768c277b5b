"""Reference model families built on the MI355X kernels (random-init, synthetic-data benchmarks)."""

from .llama import LLAMA_PRESETS, LlamaConfig, LlamaForCausalLM, build_llama
from .mixtral import MIXTRAL_PRESETS, MixtralConfig, MixtralForCausalLM, build_mixtral

# name -> zero-arg constructor (used by `accelerate-amd estimate-memory` and the benches)
MODEL_PRESETS = {}
for _n, _c in LLAMA_PRESETS.items():
    MODEL_PRESETS[_n] = (lambda c=_c: LlamaForCausalLM(c))
for _n, _c in MIXTRAL_PRESETS.items():
    MODEL_PRESETS[_n] = (lambda c=_c: MixtralForCausalLM(c))
