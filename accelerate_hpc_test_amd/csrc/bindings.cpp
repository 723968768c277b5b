// Python bindings of the accelerate_hpc_test_amd native extension (`accelerate_hpc_test_amd._C`).
// Kernels live in csrc/kernels/*.hip (gfx950), the host runtime pieces in csrc/runtime/*.cpp.
#include <torch/extension.h>

// device-side check words of the debug build (one per kernel file; release builds return 0), see kernels/common.h
int64_t acc_dbg_take_flash_attn();
int64_t acc_dbg_take_fp8();
int64_t acc_dbg_take_fp8_asm();
int64_t acc_dbg_take_grouped_gemm();
int64_t acc_dbg_take_norm_act();
int64_t acc_dbg_take_xent_optim();
int64_t acc_dbg_take_small_allreduce();
int64_t acc_dbg_take_comm_pack();
int64_t acc_dbg_take_moe_route();
int64_t acc_dbg_take_cast();
bool debug_selftest(torch::Tensor out, int64_t overshoot);

// (check id << 32 | source line) of the first failed device check since the last call, 0 if none; clears it.
static int64_t debug_status() {
  int64_t first = 0;
  for (auto fn : {acc_dbg_take_flash_attn, acc_dbg_take_fp8, acc_dbg_take_fp8_asm, acc_dbg_take_grouped_gemm, acc_dbg_take_norm_act,
                  acc_dbg_take_xent_optim, acc_dbg_take_small_allreduce, acc_dbg_take_comm_pack,
                  acc_dbg_take_moe_route, acc_dbg_take_cast}) {
    const int64_t w = fn();
    if (first == 0) first = w;
  }
  return first;
}

// norm_act.hip
std::vector<torch::Tensor> rmsnorm_fwd(torch::Tensor x, c10::optional<torch::Tensor> residual, torch::Tensor w, double eps,
                                       c10::optional<torch::Tensor> amax);
std::vector<torch::Tensor> rmsnorm_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor w, torch::Tensor rstd,
                                       c10::optional<torch::Tensor> dres, c10::optional<torch::Tensor> amax,
                                       c10::optional<torch::Tensor> dw_out, bool accumulate);
torch::Tensor swiglu_fwd(torch::Tensor gu, c10::optional<torch::Tensor> amax);
torch::Tensor transpose_bf16(torch::Tensor x);
torch::Tensor swiglu_bwd(torch::Tensor gu, torch::Tensor dh, c10::optional<torch::Tensor> amax);
void rope_inplace(torch::Tensor qkv, torch::Tensor cos, torch::Tensor sin, c10::optional<torch::Tensor> pos,
                  int64_t n_rot_heads, int64_t n_heads_total, int64_t head_dim, double sign);
torch::Tensor rope_out(torch::Tensor src, torch::Tensor cos, torch::Tensor sin, c10::optional<torch::Tensor> pos,
                       int64_t n_rot_heads, int64_t n_heads_total, int64_t head_dim, double sign);
// xent_optim.hip
std::vector<torch::Tensor> xent_fwd(torch::Tensor logits, torch::Tensor labels, int64_t ignore_index);
void xent_bwd(torch::Tensor logits, torch::Tensor labels, torch::Tensor lse, torch::Tensor scale, torch::Tensor out,
              int64_t ignore_index);
void adam_multi_tensor(torch::Tensor meta, torch::Tensor block_prefix, int64_t nblocks, int64_t pdtype, int64_t gdtype,
                       int64_t sdtype, double lr, double beta1, double beta2, double eps, double wd, double bc1,
                       double bc2_sqrt, bool adamw, c10::optional<torch::Tensor> grad_scale);
int64_t multi_tensor_chunk();
void sqnorm_multi_tensor(torch::Tensor meta, torch::Tensor block_prefix, int64_t nblocks, int64_t gdtype, torch::Tensor out,
                         bool accumulate);
void unscale_multi_tensor(torch::Tensor meta, torch::Tensor block_prefix, int64_t nblocks, int64_t gdtype, torch::Tensor inv_scale,
                          torch::Tensor found_inf);
void clip_multi_tensor(torch::Tensor meta, torch::Tensor block_prefix, int64_t nblocks, int64_t gdtype, torch::Tensor total_sq,
                       double max_norm);
// flash_attn.hip
std::vector<torch::Tensor> flash_attn_fwd(torch::Tensor q, torch::Tensor k, torch::Tensor v, double softmax_scale, bool causal);
void flash_attn_bwd(torch::Tensor dout, torch::Tensor q, torch::Tensor k, torch::Tensor v, torch::Tensor o,
                    torch::Tensor lse, torch::Tensor dq, torch::Tensor dk, torch::Tensor dv, double softmax_scale,
                    bool causal);
// fp8.hip
torch::Tensor fp8_amax(torch::Tensor x, c10::optional<torch::Tensor> out);
std::vector<torch::Tensor> fp8_cast(torch::Tensor x, torch::Tensor t, double qmax, bool from_amax, bool e5m2, bool transpose);
void fp8_cast_into(torch::Tensor x, torch::Tensor t, double qmax, bool from_amax, bool e5m2, torch::Tensor y,
                   c10::optional<torch::Tensor> yt);
void fp8_cast_batched_into(torch::Tensor x, torch::Tensor amax, double qmax, torch::Tensor y, torch::Tensor yt);
void moe_scatter_rows(torch::Tensor src, torch::Tensor pos, c10::optional<torch::Tensor> w, torch::Tensor dst,
                      c10::optional<torch::Tensor> y, c10::optional<torch::Tensor> dotw, int64_t K);
torch::Tensor moe_gather_rows(torch::Tensor src, torch::Tensor pos, c10::optional<torch::Tensor> w, int64_t T, int64_t K);
torch::Tensor fp8_gemm(torch::Tensor a, torch::Tensor b, torch::Tensor a_scale_inv, torch::Tensor b_scale_inv,
                       double smul, bool a_e5m2, bool b_e5m2, c10::optional<torch::Tensor> bias, bool out_fp32,
                       c10::optional<torch::Tensor> out, bool accumulate);
void fp8_segment_amax(torch::Tensor x, torch::Tensor lo, torch::Tensor hi, torch::Tensor out, int64_t max_len);
void fp8_segment_cast(torch::Tensor x, torch::Tensor lo, torch::Tensor hi, torch::Tensor amax, double qmax, torch::Tensor y,
                      int64_t max_len);
torch::Tensor u8_transpose(torch::Tensor x);
std::vector<torch::Tensor> mx_quant(torch::Tensor x, bool e5m2, bool colwise);
torch::Tensor mx_gemm(torch::Tensor a, torch::Tensor b, torch::Tensor sa, torch::Tensor sb, double smul,
                      c10::optional<torch::Tensor> bias, bool out_fp32, c10::optional<torch::Tensor> out_opt, bool accumulate);
void fp8_gemm_select(int64_t variant, int64_t group_m);
torch::Tensor fp8asm_dma_probe(torch::Tensor a, torch::Tensor b);
bool bf16_gemm_asm(torch::Tensor a, torch::Tensor b, c10::optional<torch::Tensor> bias, torch::Tensor out, bool accumulate);
bool bf16_gemm_asm_amn(torch::Tensor a_t, torch::Tensor b, torch::Tensor out, bool accumulate, bool trans_out, bool b_mn);
bool bf16_gemm_asm_probe(torch::Tensor a, torch::Tensor b, torch::Tensor out, int64_t probe);
bool fp8_gemm_asm_amn(torch::Tensor a_t, torch::Tensor b, c10::optional<torch::Tensor> sa, c10::optional<torch::Tensor> sb,
                      double smul, torch::Tensor out, bool accumulate, bool b_mn);
// cast.hip
bool upcast_multi(std::vector<torch::Tensor> srcs, std::vector<torch::Tensor> dsts);
bool grouped_gemm_asm(torch::Tensor a, torch::Tensor b, torch::Tensor out, std::vector<int64_t> bounds, int64_t mode,
                      c10::optional<torch::Tensor> sa, c10::optional<torch::Tensor> sb, double smul, bool accumulate);
// grouped_gemm.hip
void grouped_gemm(torch::Tensor a, torch::Tensor b, torch::Tensor out, torch::Tensor seg, int64_t mode, torch::Tensor sa,
                  torch::Tensor sb, double smul, bool accumulate);
torch::Tensor batched_transpose(torch::Tensor x);
void attn_debug_mode(int64_t mode);
void attn_dkdv_config(int64_t waves, int64_t sched, int64_t dq_waves);
void attn_fwd_config(int64_t w4);
void attn_trace(torch::Tensor buf);
// small_allreduce.hip
std::tuple<int64_t, pybind11::bytes> sar_create(int64_t rank, int64_t world, int64_t max_bytes);
void sar_open(int64_t id, std::vector<std::string> handles);
void sar_link_local(std::vector<int64_t> ids);
void sar_allreduce(int64_t id, torch::Tensor in, torch::Tensor out, int64_t op, double timeout_ms);
int64_t sar_status(int64_t id);
void sar_allreduce_local_group(std::vector<int64_t> ids, std::vector<torch::Tensor> ins, std::vector<torch::Tensor> outs,
                               int64_t op, double timeout_ms);
void sar_destroy(int64_t id);
// comm_pack.hip
void grad_shard_update(torch::Tensor dst, torch::Tensor src, double scale, bool accumulate);
// runtime/*.cpp
void register_runtime(pybind11::module& m);
void register_d2h_writer(pybind11::module& m);
void cpu_adam_step(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, c10::optional<torch::Tensor> shadow,
                   double lr, double beta1, double beta2, double eps, double wd, double bc1, double bc2_sqrt, bool adamw);
bool blaslt_wgrad_f32(torch::Tensor dy, torch::Tensor x, torch::Tensor out, bool accumulate, bool x_t, bool dy_t);
bool blaslt_dgrad_bf16(torch::Tensor dy, torch::Tensor w, torch::Tensor out);
std::vector<std::tuple<int64_t, int64_t, int64_t, int64_t, double>> blaslt_wgrad_plans();
bool blaslt_fp8_gemm(torch::Tensor a, torch::Tensor b, torch::Tensor sa, torch::Tensor sb, double alpha, torch::Tensor out,
                     bool accumulate, bool dynamic);
std::vector<int64_t> blaslt_fp8_dynamic_stats();
bool blaslt_mx_gemm(torch::Tensor a, torch::Tensor b, torch::Tensor sa, torch::Tensor sb, torch::Tensor out, bool accumulate);
std::vector<std::tuple<int64_t, int64_t, int64_t, int64_t, double>> blaslt_fp8_plans();

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X (gfx950) native kernels and runtime for accelerate_hpc_test_amd";
  m.def("rmsnorm_fwd", &rmsnorm_fwd, pybind11::arg("x"), pybind11::arg("residual"), pybind11::arg("w"), pybind11::arg("eps"),
        pybind11::arg("amax") = pybind11::none());
  m.def("rmsnorm_bwd", &rmsnorm_bwd, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("rstd"),
        pybind11::arg("dres"), pybind11::arg("amax") = pybind11::none(), pybind11::arg("dw_out") = pybind11::none(),
        pybind11::arg("accumulate") = false);
  m.def("swiglu_fwd", &swiglu_fwd, pybind11::arg("gu"), pybind11::arg("amax") = pybind11::none());
  m.def("transpose_bf16", &transpose_bf16);
  m.def("swiglu_bwd", &swiglu_bwd, pybind11::arg("gu"), pybind11::arg("dh"), pybind11::arg("amax") = pybind11::none());
  m.def("rope_inplace", &rope_inplace);
  m.def("rope_out", &rope_out);
  m.def("xent_fwd", &xent_fwd);
  m.def("xent_bwd", &xent_bwd);
  m.def("adam_multi_tensor", &adam_multi_tensor);
  m.def("multi_tensor_chunk", &multi_tensor_chunk);
  m.def("sqnorm_multi_tensor", &sqnorm_multi_tensor);
  m.def("clip_multi_tensor", &clip_multi_tensor);
  m.def("unscale_multi_tensor", &unscale_multi_tensor);
  m.def("flash_attn_fwd", &flash_attn_fwd);
  m.def("flash_attn_bwd", &flash_attn_bwd);
  m.def("fp8_amax", &fp8_amax);
  m.def("fp8_cast", &fp8_cast);
  m.def("fp8_cast_into", &fp8_cast_into);
  m.def("fp8_cast_batched_into", &fp8_cast_batched_into);
  m.def("moe_scatter_rows", &moe_scatter_rows);
  m.def("moe_gather_rows", &moe_gather_rows);
  m.def("fp8_gemm", &fp8_gemm, pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("a_scale_inv"), pybind11::arg("b_scale_inv"),
        pybind11::arg("smul"), pybind11::arg("a_e5m2"), pybind11::arg("b_e5m2"), pybind11::arg("bias"), pybind11::arg("out_fp32"),
        pybind11::arg("out") = pybind11::none(), pybind11::arg("accumulate") = false);
  m.def("grad_shard_update", &grad_shard_update);
  m.def("fp8_segment_amax", &fp8_segment_amax);
  m.def("fp8_segment_cast", &fp8_segment_cast);
  m.def("u8_transpose", &u8_transpose);
  m.def("mx_quant", &mx_quant, pybind11::arg("x"), pybind11::arg("e5m2") = false, pybind11::arg("colwise") = true);
  m.def("mx_gemm", &mx_gemm, pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("sa"), pybind11::arg("sb"),
        pybind11::arg("smul") = 1.0, pybind11::arg("bias") = pybind11::none(), pybind11::arg("out_fp32") = false,
        pybind11::arg("out") = pybind11::none(), pybind11::arg("accumulate") = false);
  m.def("grouped_gemm", &grouped_gemm);
  m.def("batched_transpose", &batched_transpose);
  m.def("attn_debug_mode", &attn_debug_mode);
  m.def("attn_dkdv_config", &attn_dkdv_config);
  m.def("attn_fwd_config", &attn_fwd_config);
  m.def("attn_trace", &attn_trace);
  m.def("sar_create", &sar_create);
  m.def("sar_open", &sar_open);
  m.def("sar_link_local", &sar_link_local);
  m.def("sar_allreduce", &sar_allreduce);
  m.def("sar_status", &sar_status);
  m.def("sar_allreduce_local_group", &sar_allreduce_local_group);
  m.def("sar_destroy", &sar_destroy);
  m.def("bf16_gemm_asm", &bf16_gemm_asm, pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("bias"), pybind11::arg("out"),
        pybind11::arg("accumulate") = false, "bf16 out (=|+=) a . b^T (+ bias) on the asm-scheduled GEMM; false = shape not tiled");
  m.def("bf16_gemm_asm_amn", &bf16_gemm_asm_amn, pybind11::arg("a_t"), pybind11::arg("b"), pybind11::arg("out"),
        pybind11::arg("accumulate") = false, pybind11::arg("trans_out") = false, pybind11::arg("b_mn") = false,
        "out (=|+=) a_t^T . b^T (or its transpose) with a_t [K, M] M-contiguous (b_mn: b [K, N] N-contiguous, "
        "transposed store), on the asm GEMM; false = shape not tiled");
  m.def("fp8_gemm_asm_amn", &fp8_gemm_asm_amn, pybind11::arg("a_t"), pybind11::arg("b"), pybind11::arg("sa"),
        pybind11::arg("sb"), pybind11::arg("smul") = 1.0, pybind11::arg("out"), pybind11::arg("accumulate") = false,
        pybind11::arg("b_mn") = false,
        "out (=|+=) (a_t^T . b^T)^T * sa * sb * smul, fp8 a_t [K, M] M-contiguous (b_mn: b [K, N]); false = not tiled");
  m.def("bf16_gemm_asm_probe", &bf16_gemm_asm_probe, "timing probe of the bf16 asm loop (1 no DMA, 2 no reads, 3 MFMA only)");
  m.def("upcast_multi", &upcast_multi, pybind11::arg("srcs"), pybind11::arg("dsts"),
        "dsts[i] = srcs[i] upcast (fp8 / fp16 / bf16 / fp32 -> bf16 / fp16 / fp32) in one launch; false = not handled");
  m.def("grouped_gemm_asm", &grouped_gemm_asm, pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("out"),
        pybind11::arg("bounds"), pybind11::arg("mode"), pybind11::arg("sa") = pybind11::none(),
        pybind11::arg("sb") = pybind11::none(), pybind11::arg("smul") = 1.0, pybind11::arg("accumulate") = false,
        "MoE grouped GEMM on the asm kernel with a host segment table; false = not tiled (nothing launched)");
  m.def("fp8asm_dma_probe", &fp8asm_dma_probe, "debug: LDS image after the asm GEMM's first-tile DMA");
  m.def("fp8_gemm_select", &fp8_gemm_select, pybind11::arg("variant"), pybind11::arg("group_m") = 0);
  register_runtime(m);
  register_d2h_writer(m);
  m.def("blaslt_dgrad_bf16", &blaslt_dgrad_bf16, pybind11::arg("dy"), pybind11::arg("w"), pybind11::arg("out"),
        "dx = dy . W (bf16, both row-major: the NN layout) on a searched hipBLASLt algorithm; False if none");
  m.def("blaslt_wgrad_f32", &blaslt_wgrad_f32, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("out"), pybind11::arg("accumulate"),
        pybind11::arg("x_t") = false, pybind11::arg("dy_t") = false);
  m.def("cpu_adam_step", &cpu_adam_step);
  m.def("blaslt_wgrad_plans", &blaslt_wgrad_plans);
  m.def("blaslt_fp8_gemm", &blaslt_fp8_gemm, "per-tensor-scaled fp8 GEMM on hipBLASLt (C = alpha sa sb A B^T)",
        pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("sa"), pybind11::arg("sb"), pybind11::arg("alpha"),
        pybind11::arg("out"), pybind11::arg("accumulate"), pybind11::arg("dynamic") = false);
  m.def("blaslt_fp8_dynamic_stats", &blaslt_fp8_dynamic_stats);
  m.def("blaslt_mx_gemm", &blaslt_mx_gemm, "MXFP8 GEMM on hipBLASLt (VEC32_UE8M0 block scales)");
  m.def("blaslt_fp8_plans", &blaslt_fp8_plans);
  m.def("debug_status", &debug_status, "first failed device bounds check (id << 32 | line), 0 if none; clears it");
  m.def("debug_selftest", &debug_selftest);
#ifdef ACC_DEBUG_BOUNDS
  m.attr("debug_build") = true;
#else
  m.attr("debug_build") = false;
#endif
}
