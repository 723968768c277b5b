// Host AdamW for FSDP CPU offload (the optimizer step of offloaded fp32 master shards runs on the host CPUs).
//
// One OpenMP-parallel, vectorised pass over (param, grad, exp_avg, exp_avg_sq) fp32 shard ranges — torch.optim.AdamW
// / Adam semantics, bit-compatible state layout — that also writes the bf16 copy of the updated parameters into a
// pinned staging buffer. The FSDP engine then uploads 2 bytes per parameter (instead of the 4-byte master) with one
// non-blocking H2D copy per unit into the bf16 all-gather source on the GPU. The loop is compiled for AVX-512, AVX2
// and baseline x86-64 (`target_clones`), picked at load time for the host it runs on.
#include <torch/extension.h>

#include "host_kernels.h"

using acc_host::Hyper;
using acc_host::adam_range;

// In-place AdamW/Adam step over contiguous fp32 CPU tensors; `shadow` (bf16, same numel) receives the updated params.
void cpu_adam_step(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, c10::optional<torch::Tensor> shadow,
                   double lr, double beta1, double beta2, double eps, double wd, double bc1, double bc2_sqrt, bool adamw) {
  for (const auto* t : {&p, &g, &m, &v}) {
    TORCH_CHECK(t->device().is_cpu() && t->scalar_type() == at::kFloat && t->is_contiguous(),
                "cpu_adam_step: contiguous fp32 CPU tensors required");
    TORCH_CHECK(t->numel() == p.numel(), "cpu_adam_step: size mismatch");
  }
  uint16_t* sh = nullptr;
  if (shadow.has_value() && shadow->defined()) {
    TORCH_CHECK(shadow->device().is_cpu() && shadow->scalar_type() == at::kBFloat16 && shadow->is_contiguous() &&
                    shadow->numel() == p.numel(),
                "cpu_adam_step: shadow must be a contiguous bf16 CPU tensor of the same size");
    sh = reinterpret_cast<uint16_t*>(shadow->data_ptr());
  }
  Hyper h{(float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd, (float)bc1, (float)bc2_sqrt, adamw};
  pybind11::gil_scoped_release nogil;
  adam_range(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), sh, p.numel(), h);
}
