// PyTorch bindings for the distriflow_amd gfx950 kernels (module distriflow_amd._C).
//
// Every entry point validates shapes/dtypes/devices on the host BEFORE launching (a bad launch
// on a shared MI355X node can reset all GPUs), then launches on PyTorch's current HIP stream so
// the calls compose with torch.cuda graph capture and RCCL collectives on the same stream.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>
#include <hip/hip_runtime_api.h>

#include "kernels.h"
#include "native_runtime.h"


namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_hip(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "distriflow_amd kernel '", what, "' failed: ", hipGetErrorString(e));
}

void need(const torch::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

template <typename T>
const T* cptr(const c10::optional<torch::Tensor>& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<const T*>(t->data_ptr()) : nullptr;
}

// geometry: [SH, SW, SC, OH, OW, KH, KW, stride, pad]
// Conv geometry [SH, SW, SC, OH, OW, KH, KW, stride, pad(, stride_w, pad_w)] (the launch's source / output
// dims: for the data gradient the source is dY and the output dX).  stride / pad are the row stride and the
// top padding; the output size may imply more padding at the bottom / right than at the top / left (Keras
// 'same' with an odd total).  Anything but one stride, one symmetric padding and a square kernel is
// 'irregular': the specialised kernels refuse it and the generic implicit GEMM runs.
template <typename A>
void set_conv_geom(A& a, const std::vector<int64_t>& geom, int mode) {
  TORCH_CHECK(geom.size() == 9 || geom.size() == 11, "geometry must have 9 or 11 ints");
  int g[11];
  for (size_t i = 0; i < geom.size(); ++i) g[i] = (int)geom[i];
  if (geom.size() == 9) g[9] = g[7], g[10] = g[8];
  a.SH = g[0]; a.SW = g[1]; a.SC = g[2]; a.OH = g[3]; a.OW = g[4]; a.KH = g[5]; a.KW = g[6];
  a.stride = g[7]; a.pad = g[8]; a.stride_w = g[9]; a.pad_w = g[10];
  a.irregular = 0;
  if (mode == dfa::MODE_DIRECT) return;
  TORCH_CHECK(a.stride >= 1 && a.stride_w >= 1 && a.pad >= 0 && a.pad_w >= 0 && a.KH >= 1 && a.KW >= 1,
              "conv geometry: stride >= 1, pad >= 0");
  const bool fwd = mode == dfa::MODE_FWD;
  const int ih = fwd ? a.SH : a.OH, iw = fwd ? a.SW : a.OW, oh = fwd ? a.OH : a.SH, ow = fwd ? a.OW : a.SW;
  a.irregular = a.KH != a.KW || a.stride_w != a.stride || a.pad_w != a.pad ||
                oh != (ih + 2 * a.pad - a.KH) / a.stride + 1 || ow != (iw + 2 * a.pad - a.KW) / a.stride + 1;
}

dfa::DropSpec drop_from(double p, int64_t seed, const c10::optional<torch::Tensor>& step, int64_t step_add) {
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout p must be in [0,1)");
  const long long* sp = nullptr;
  if (step.has_value() && step->defined()) {
    need(*step, at::kLong, "dropout step");
    sp = reinterpret_cast<const long long*>(step->data_ptr());
  }
  return dfa::make_drop((float)p, (unsigned long long)seed, sp, (int)step_add);
}

void igemm_fwd_py(torch::Tensor src, torch::Tensor w, c10::optional<torch::Tensor> bias,
                  c10::optional<torch::Tensor> mask, torch::Tensor out, int64_t M, int64_t N, int64_t K, int64_t Kpad,
                  int64_t lda, int64_t ldc, std::vector<int64_t> geom, int64_t mode, bool relu, double alpha,
                  c10::optional<torch::Tensor> res, c10::optional<torch::Tensor> resmask, double drop_p,
                  int64_t drop_seed, c10::optional<torch::Tensor> drop_step, c10::optional<torch::Tensor> pool_code,
                  int64_t drop_step_add, c10::optional<torch::Tensor> bn_ws, c10::optional<torch::Tensor> bn_ticket,
                  int64_t bn_mode, std::vector<torch::Tensor> bn_vecs, c10::optional<torch::Tensor> bn_x,
                  double bn_momentum, double bn_eps, double bn_gscale, c10::optional<torch::Tensor> bacc,
                  int64_t bacc_mode, std::vector<torch::Tensor> bacc_in, c10::optional<torch::Tensor> bacc2,
                  std::vector<torch::Tensor> bacc2_in) {
  need(src, at::kBFloat16, "src");
  need(w, at::kBFloat16, "w");
  TORCH_CHECK(out.is_cuda() && out.is_contiguous(), "out must be a contiguous GPU tensor");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat, "out must be bf16 or fp32");
  TORCH_CHECK(Kpad % 32 == 0 && Kpad >= K, "Kpad must be a multiple of 32 and >= K");
  TORCH_CHECK(w.numel() >= ((N + 15) / 16 * 16) * Kpad, "weight buffer smaller than [Npad16][Kpad]");
  const bool pooled = pool_code.has_value() && pool_code->defined();
  if (pooled) {
    TORCH_CHECK(mode == 1 && M % 4 == 0 && ldc == N, "pooled conv: forward conv, M % 4 == 0, ldc == N");
    TORCH_CHECK(pool_code->is_cuda() && pool_code->is_contiguous() && pool_code->scalar_type() == at::kByte &&
                    pool_code->numel() >= M / 4 * N,
                "pool_code must be a uint8 GPU tensor of [M/4][N]");
    TORCH_CHECK(out.numel() >= M / 4 * N, "pooled out too small for [M/4][N]");
  } else {
    TORCH_CHECK(out.numel() >= (M - 1) * ldc + N, "out too small for [M][ldc]");
  }
  TORCH_CHECK(ldc >= N, "ldc < N");
  dfa::IGemmArgs a{};
  set_conv_geom(a, geom, (int)mode);
  if (mode == 0) {
    TORCH_CHECK(src.numel() >= (M - 1) * lda + K, "src too small for [M][lda]");
  } else {
    TORCH_CHECK(a.OH > 0 && a.OW > 0 && M % (a.OH * a.OW) == 0, "M must be B*OH*OW");
    const int64_t Bn = M / (a.OH * a.OW);
    TORCH_CHECK(src.numel() >= Bn * a.SH * a.SW * a.SC, "src too small for the conv geometry");
    TORCH_CHECK(K == (int64_t)a.KH * a.KW * a.SC, "K must be KH*KW*C");
    TORCH_CHECK(a.KH < 128 && a.KW < 128 && a.SC < 65536, "conv geometry out of range");
  }
  if (bias.has_value() && bias->defined()) {
    need(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() >= N, "bias too small");
  }
  if (mask.has_value() && mask->defined()) {
    need(*mask, at::kBFloat16, "mask");
    TORCH_CHECK(mask->numel() >= (M - 1) * ldc + N, "mask too small");
  }
  for (auto* t : {&res, &resmask}) {
    if (t->has_value() && (*t)->defined()) {
      need(**t, at::kBFloat16, "residual");
      TORCH_CHECK((*t)->numel() >= (M - 1) * ldc + N, "residual too small");
    }
  }
  TORCH_CHECK(!(resmask.has_value() && resmask->defined()) || (res.has_value() && res->defined()),
              "resmask without res");
  a.src = reinterpret_cast<const dfa::bf16*>(src.data_ptr());
  a.w = reinterpret_cast<const dfa::bf16*>(w.data_ptr());
  a.bias = cptr<float>(bias);
  a.mask = cptr<dfa::bf16>(mask);
  a.res = cptr<dfa::bf16>(res);
  a.resmask = cptr<dfa::bf16>(resmask);
  a.out = out.data_ptr();
  a.M = (int)M; a.N = (int)N; a.K = (int)K; a.Kpad = (int)Kpad; a.lda = (int)lda; a.ldc = (int)ldc;
  a.relu = relu ? 1 : 0;
  a.out_f32 = out.scalar_type() == at::kFloat ? 1 : 0;
  a.alpha = (float)alpha;
  a.drop = drop_from(drop_p, drop_seed, drop_step, drop_step_add);
  if (pooled) {
    a.pool_code = pool_code->data_ptr<uint8_t>();
    TORCH_CHECK(dfa::igemm64_pool_supported(a), "pooled conv: unsupported geometry / alignment");
  }
  if (bn_ws.has_value() && bn_ws->defined()) {
    // BatchNorm statistics finalised inside this launch (kernels.h BnEpi)
    need(*bn_ws, at::kFloat, "bn_ws");
    TORCH_CHECK(bn_ticket.has_value() && bn_ticket->defined(), "bn_ws needs bn_ticket");
    need(*bn_ticket, at::kInt, "bn_ticket");
    int ntn = 0;
    const int ntm = dfa::igemm64_bn_layout(a, (int)mode, &ntn);
    TORCH_CHECK(ntm > 0, "bn: this conv launch cannot finalise BatchNorm statistics");
    const int ngrp = (ntm + 15) / 16;
    TORCH_CHECK(bn_ws->numel() >= (int64_t)(ntm + ngrp) * 2 * N, "bn_ws too small");
    TORCH_CHECK(bn_ticket->numel() >= (int64_t)ntn * (1 + ngrp), "bn_ticket too small");
    TORCH_CHECK(out.scalar_type() == at::kBFloat16, "bn: bf16 output");
    dfa::BnEpi& e = a.bn;
    e.part = bn_ws->data_ptr<float>();
    e.ticket = reinterpret_cast<unsigned*>(bn_ticket->data_ptr<int>());
    e.ntm = ntm;
    e.ngrp = ngrp;
    e.mode = (int)bn_mode;
    e.momentum = (float)bn_momentum;
    e.eps = (float)bn_eps;
    e.gscale = (float)bn_gscale;
    for (auto& v : bn_vecs) {
      need(v, at::kFloat, "bn vector");
      TORCH_CHECK(v.numel() >= N, "bn vector smaller than N");
    }
    if (bn_mode == 0) {
      TORCH_CHECK(bn_vecs.size() == 4, "bn mode 0: [mean, invstd, run_mean, run_var]");
      e.mean_out = bn_vecs[0].data_ptr<float>();
      e.invstd_out = bn_vecs[1].data_ptr<float>();
      e.run_mean = bn_vecs[2].data_ptr<float>();
      e.run_var = bn_vecs[3].data_ptr<float>();
    } else {
      TORCH_CHECK(bn_mode == 1 && bn_vecs.size() == 6, "bn mode 1: [mean, invstd, gamma, dgamma, dbeta, coef]");
      TORCH_CHECK(bn_x.has_value() && bn_x->defined(), "bn mode 1 needs the BN input");
      need(*bn_x, at::kBFloat16, "bn_x");
      TORCH_CHECK(bn_x->numel() >= (M - 1) * ldc + N, "bn_x too small");
      TORCH_CHECK(bn_vecs[5].numel() >= 3 * N, "bn coef must hold [3][N]");
      e.x = reinterpret_cast<const dfa::bf16*>(bn_x->data_ptr());
      e.mean = bn_vecs[0].data_ptr<float>();
      e.invstd = bn_vecs[1].data_ptr<float>();
      e.gamma = bn_vecs[2].data_ptr<float>();
      e.dgamma = bn_vecs[3].data_ptr<float>();
      e.dbeta = bn_vecs[4].data_ptr<float>();
      e.coef = bn_vecs[5].data_ptr<float>();
    }
  }
  if (bacc.has_value() && bacc->defined()) {
    // BatchNorm sums accumulated by the epilogue (kernels.h BnAcc): acc [nrep][2][N] fp64; mode 1 inputs
    // [x, mean, invstd] of the BatchNorm (and of a second one sharing the gradient)
    need(*bacc, at::kDouble, "bacc");
    TORCH_CHECK(bacc->numel() % (2 * N) == 0, "bacc must be [nrep][2][N]");
    dfa::BnAcc& e = a.bacc;
    e.acc = bacc->data_ptr<double>();
    e.nrep = (int)(bacc->numel() / (2 * N));
    e.mode = (int)bacc_mode;
    TORCH_CHECK(bacc_mode == 0 || bacc_mode == 1, "bacc_mode 0 (forward) or 1 (backward)");
    auto inputs = [&](const std::vector<torch::Tensor>& v, const dfa::bf16** x, const float** mu, const float** is) {
      TORCH_CHECK(v.size() == 3, "bacc mode 1 inputs: [x, mean, invstd]");
      need(v[0], at::kBFloat16, "bacc x");
      TORCH_CHECK(v[0].numel() >= (M - 1) * ldc + N, "bacc x too small");
      need(v[1], at::kFloat, "bacc mean");
      need(v[2], at::kFloat, "bacc invstd");
      TORCH_CHECK(v[1].numel() >= N && v[2].numel() >= N, "bacc mean / invstd smaller than N");
      *x = reinterpret_cast<const dfa::bf16*>(v[0].data_ptr());
      *mu = v[1].data_ptr<float>();
      *is = v[2].data_ptr<float>();
    };
    if (bacc_mode == 1) inputs(bacc_in, &e.x, &e.mean, &e.invstd);
    if (bacc2.has_value() && bacc2->defined()) {
      TORCH_CHECK(bacc_mode == 1, "a second BatchNorm's sums: backward only");
      need(*bacc2, at::kDouble, "bacc2");
      TORCH_CHECK(bacc2->numel() == bacc->numel(), "bacc2 must match bacc");
      e.acc2 = bacc2->data_ptr<double>();
      inputs(bacc2_in, &e.x2, &e.mean2, &e.invstd2);
    }
    TORCH_CHECK(dfa::igemm_bacc_ok(a, (int)mode), "bacc: this launch cannot accumulate BatchNorm sums");
  }
  TORCH_CHECK(!a.drop.on || (ldc == N && !a.out_f32), "folded dropout needs a dense bf16 output (ldc == N)");
  // split-K partials for the under-filled (small-M, long-K) shapes: PyTorch's caching allocator is
  // stream ordered and graph-capture aware, so the scratch is safe to drop right after the launch
  torch::Tensor splitk;
  const long long skf = dfa::igemm64_splitk_floats(a, (int)mode);
  if (skf > 0) {
    splitk = torch::empty({skf}, out.options().dtype(at::kFloat));
    a.splitk_ws = splitk.data_ptr<float>();
  }
  check_hip(dfa::igemm_fwd(a, (int)mode, cur_stream()), "igemm_fwd");
}

void igemm_wgrad_py(torch::Tensor dy, torch::Tensor src, torch::Tensor gw, c10::optional<torch::Tensor> gb,
                    torch::Tensor workspace, int64_t M, int64_t N, int64_t K, int64_t ldd, int64_t lda,
                    std::vector<int64_t> geom, int64_t mode, double scale) {
  need(dy, at::kBFloat16, "dy");
  need(src, at::kBFloat16, "src");
  need(gw, at::kFloat, "gw");
  need(workspace, at::kFloat, "workspace");
  TORCH_CHECK(gw.numel() >= N * K, "gw too small");
  TORCH_CHECK(dy.numel() >= (M - 1) * ldd + N, "dy too small");
  dfa::WgradArgs a{};
  set_conv_geom(a, geom, (int)mode);
  if (mode == 0) {
    TORCH_CHECK(src.numel() >= (M - 1) * lda + K, "src too small");
  } else {
    TORCH_CHECK(M % (a.OH * a.OW) == 0, "M must be B*OH*OW");
    TORCH_CHECK(src.numel() >= (M / (a.OH * a.OW)) * a.SH * a.SW * a.SC, "src too small");
    TORCH_CHECK(K == (int64_t)a.KH * a.KW * a.SC, "K must be KH*KW*C");
  }
  if (gb.has_value() && gb->defined()) {
    need(*gb, at::kFloat, "gb");
    TORCH_CHECK(gb->numel() >= N, "gb too small");
  }
  a.dy = reinterpret_cast<const dfa::bf16*>(dy.data_ptr());
  a.src = reinterpret_cast<const dfa::bf16*>(src.data_ptr());
  a.gw = gw.data_ptr<float>();
  a.gb = (gb.has_value() && gb->defined()) ? gb->data_ptr<float>() : nullptr;
  a.M = (int)M; a.N = (int)N; a.K = (int)K; a.ldd = (int)ldd; a.lda = (int)lda;
  a.with_bias = a.gb ? 1 : 0;
  a.scale = (float)scale;
  check_hip(dfa::igemm_wgrad(a, (int)mode, workspace.data_ptr<float>(), (size_t)workspace.numel(), cur_stream()),
            "igemm_wgrad");
}

void maxpool_fwd_py(torch::Tensor x, torch::Tensor y, int64_t B, int64_t H, int64_t W, int64_t C, int64_t P,
                    double drop_p, int64_t drop_seed, c10::optional<torch::Tensor> drop_step, int64_t drop_step_add) {
  need(x, at::kBFloat16, "x");
  need(y, at::kBFloat16, "y");
  TORCH_CHECK(P > 0 && H >= P && W >= P, "bad pool geometry");
  TORCH_CHECK(x.numel() >= B * H * W * C && y.numel() >= B * (H / P) * (W / P) * C, "pool buffers too small");
  check_hip(dfa::maxpool_fwd((const dfa::bf16*)x.data_ptr(), (dfa::bf16*)y.data_ptr(), B, H, W, C, P, cur_stream(),
                             drop_from(drop_p, drop_seed, drop_step, drop_step_add)),
            "maxpool_fwd");
}

void maxpool_bwd_py(torch::Tensor x, torch::Tensor dy, torch::Tensor dx, int64_t B, int64_t H, int64_t W, int64_t C,
                    int64_t P, bool relu_fused) {
  need(x, at::kBFloat16, "x");
  need(dy, at::kBFloat16, "dy");
  need(dx, at::kBFloat16, "dx");
  TORCH_CHECK(P > 0 && H >= P && W >= P, "bad pool geometry");
  TORCH_CHECK(x.numel() >= B * H * W * C && dx.numel() >= B * H * W * C &&
                  dy.numel() >= B * (H / P) * (W / P) * C,
              "pool buffers too small");
  check_hip(dfa::maxpool_bwd((const dfa::bf16*)x.data_ptr(), (const dfa::bf16*)dy.data_ptr(),
                             (dfa::bf16*)dx.data_ptr(), B, H, W, C, P, relu_fused ? 1 : 0, cur_stream()),
            "maxpool_bwd");
}

void softmax_ce_py(torch::Tensor logits, torch::Tensor labels, c10::optional<torch::Tensor> dlogits,
                   c10::optional<torch::Tensor> stats, int64_t B, int64_t C, int64_t ldl, int64_t ldg,
                   double grad_scale) {
  need(logits, at::kFloat, "logits");
  need(labels, at::kInt, "labels");
  TORCH_CHECK(logits.numel() >= (B - 1) * ldl + C && labels.numel() >= B, "softmax_ce inputs too small");
  dfa::bf16* dl = nullptr;
  if (dlogits.has_value() && dlogits->defined()) {
    need(*dlogits, at::kBFloat16, "dlogits");
    TORCH_CHECK(dlogits->numel() >= (B - 1) * ldg + C, "dlogits too small");
    dl = (dfa::bf16*)dlogits->data_ptr();
  }
  float* sp = nullptr;
  if (stats.has_value() && stats->defined()) {
    need(*stats, at::kFloat, "stats");
    TORCH_CHECK(stats->numel() >= 2, "stats needs 2 floats");
    sp = stats->data_ptr<float>();
  }
  check_hip(dfa::softmax_ce(logits.data_ptr<float>(), labels.data_ptr<int>(), dl, sp, B, C, ldl, ldg,
                            (float)grad_scale, cur_stream()),
            "softmax_ce");
}

void dropout_py(torch::Tensor x, torch::Tensor y, double p, int64_t seed, c10::optional<torch::Tensor> mask,
                c10::optional<torch::Tensor> step) {
  const long long* sp = nullptr;
  if (step.has_value() && step->defined()) {
    need(*step, at::kLong, "step");
    sp = reinterpret_cast<const long long*>(step->data_ptr());
  }
  need(x, at::kBFloat16, "x");
  need(y, at::kBFloat16, "y");
  TORCH_CHECK(y.numel() >= x.numel(), "dropout out too small");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout p must be in [0,1)");
  if (mask.has_value() && mask->defined()) {
    need(*mask, at::kBFloat16, "mask");
    TORCH_CHECK(mask->numel() >= x.numel(), "dropout mask too small");
  }
  check_hip(dfa::dropout((const dfa::bf16*)x.data_ptr(), (dfa::bf16*)y.data_ptr(), cptr<dfa::bf16>(mask), x.numel(),
                         (float)p, (unsigned long long)seed, sp, cur_stream()),
            "dropout");
}

void gather_batch_py(torch::Tensor data, c10::optional<torch::Tensor> labels, torch::Tensor idx, torch::Tensor out,
                     c10::optional<torch::Tensor> out_labels, int64_t B, int64_t row, double scale,
                     c10::optional<torch::Tensor> step_inc) {
  TORCH_CHECK(data.is_cuda() && data.is_contiguous(), "data must be a contiguous GPU tensor");
  const bool u8 = data.scalar_type() == at::kByte;
  TORCH_CHECK(u8 || data.scalar_type() == at::kBFloat16, "data must be uint8 or bf16");
  need(idx, at::kLong, "idx");
  need(out, at::kBFloat16, "out");
  TORCH_CHECK(idx.numel() >= B && out.numel() >= B * row, "gather buffers too small");
  TORCH_CHECK(data.dim() >= 1 && data.size(0) > 0 && data.numel() / data.size(0) == row, "data row size mismatch");
  const int* lp = nullptr;
  int* olp = nullptr;
  if (labels.has_value() && labels->defined()) {
    need(*labels, at::kInt, "labels");
    TORCH_CHECK(out_labels.has_value() && out_labels->defined(), "out_labels required with labels");
    need(*out_labels, at::kInt, "out_labels");
    lp = labels->data_ptr<int>();
    olp = out_labels->data_ptr<int>();
  }
  check_hip(dfa::gather_batch(data.data_ptr(), u8 ? 1 : 0, lp, reinterpret_cast<const long long*>(idx.data_ptr<int64_t>()), (dfa::bf16*)out.data_ptr(),
                              olp, B, row, (float)scale, (long long)data.size(0), cur_stream(),
                              step_inc.has_value() && step_inc->defined()
                                  ? reinterpret_cast<long long*>(step_inc->data_ptr<int64_t>())
                                  : nullptr),
            "gather_batch");
}

// Keras merge layer (csrc/merge.hip): inputs [rows][w_i] bf16; fwd writes out, bwd writes grads[i]
static dfa::MergeArgs merge_args(std::vector<torch::Tensor> ins, int64_t kind, int64_t cout) {
  TORCH_CHECK(ins.size() >= 1 && ins.size() <= (size_t)dfa::kMergeMaxIn, "merge: 1..8 inputs");
  dfa::MergeArgs a{};
  a.n = (int)ins.size();
  a.kind = (int)kind;
  a.cout = (int)cout;
  for (int i = 0; i < a.n; ++i) {
    need(ins[i], at::kBFloat16, "merge input");
    const int64_t w = ins[i].size(-1);
    TORCH_CHECK(ins[i].numel() % w == 0, "merge: bad input");
    if (i == 0) a.rows = ins[i].numel() / w;
    TORCH_CHECK(ins[i].numel() / w == a.rows, "merge: inputs differ in rows");
    a.w[i] = (int)w;
    a.in[i] = (const dfa::bf16*)ins[i].data_ptr();
  }
  return a;
}
void merge_fwd_py(std::vector<torch::Tensor> ins, torch::Tensor out, int64_t kind) {
  need(out, at::kBFloat16, "merge out");
  dfa::MergeArgs a = merge_args(ins, kind, out.size(-1));
  TORCH_CHECK(out.numel() == a.rows * (int64_t)a.cout, "merge: out size");
  a.out = (dfa::bf16*)out.data_ptr();
  check_hip(dfa::merge_fwd(a, cur_stream()), "merge_fwd");
}
void merge_bwd_py(std::vector<torch::Tensor> ins, torch::Tensor dy, std::vector<torch::Tensor> grads, int64_t kind) {
  need(dy, at::kBFloat16, "merge dy");
  dfa::MergeArgs a = merge_args(ins, kind, dy.size(-1));
  TORCH_CHECK(grads.size() == ins.size() && dy.numel() == a.rows * (int64_t)a.cout, "merge: grads / dy size");
  a.dy = (const dfa::bf16*)dy.data_ptr();
  for (int i = 0; i < a.n; ++i) {
    need(grads[i], at::kBFloat16, "merge grad");
    TORCH_CHECK(grads[i].numel() == ins[i].numel(), "merge: grad size");
    a.grad[i] = (dfa::bf16*)grads[i].data_ptr();
  }
  check_hip(dfa::merge_bwd(a, cur_stream()), "merge_bwd");
}

void add_act_py(torch::Tensor a, torch::Tensor b, torch::Tensor out, bool relu) {
  need(a, at::kBFloat16, "a");
  need(b, at::kBFloat16, "b");
  need(out, at::kBFloat16, "out");
  TORCH_CHECK(a.numel() == b.numel() && out.numel() >= a.numel(), "add_act size mismatch");
  check_hip(dfa::add_act((const dfa::bf16*)a.data_ptr(), (const dfa::bf16*)b.data_ptr(), (dfa::bf16*)out.data_ptr(),
                         a.numel(), relu ? 1 : 0, cur_stream()),
            "add_act");
}

void relu_bwd_py(torch::Tensor y, torch::Tensor dy, torch::Tensor dx) {
  need(y, at::kBFloat16, "y");
  need(dy, at::kBFloat16, "dy");
  need(dx, at::kBFloat16, "dx");
  TORCH_CHECK(y.numel() == dy.numel() && dx.numel() >= y.numel(), "relu_bwd size mismatch");
  check_hip(dfa::relu_bwd((const dfa::bf16*)y.data_ptr(), (const dfa::bf16*)dy.data_ptr(), (dfa::bf16*)dx.data_ptr(),
                          y.numel(), cur_stream()),
            "relu_bwd");
}

// ---- generic Keras layers (csrc/act.hip)
void act_fwd_py(torch::Tensor x, torch::Tensor y, int64_t kind) {
  need(x, at::kBFloat16, "act x");
  need(y, at::kBFloat16, "act y");
  TORCH_CHECK(y.numel() >= x.numel(), "act: output too small");
  TORCH_CHECK(kind >= dfa::kActLinear && kind <= dfa::kActExp, "act: unknown kind");
  check_hip(dfa::act_fwd((const dfa::bf16*)x.data_ptr(), (dfa::bf16*)y.data_ptr(), x.numel(), (int)kind,
                         cur_stream()),
            "act_fwd");
}

void act_bwd_py(torch::Tensor x, torch::Tensor dy, torch::Tensor dx, int64_t kind, bool in_relu) {
  need(x, at::kBFloat16, "act x");
  need(dy, at::kBFloat16, "act dy");
  need(dx, at::kBFloat16, "act dx");
  TORCH_CHECK(dy.numel() == x.numel() && dx.numel() >= x.numel(), "act_bwd: size mismatch");
  TORCH_CHECK(kind >= dfa::kActLinear && kind <= dfa::kActExp, "act: unknown kind");
  check_hip(dfa::act_bwd((const dfa::bf16*)x.data_ptr(), (const dfa::bf16*)dy.data_ptr(), (dfa::bf16*)dx.data_ptr(),
                         x.numel(), (int)kind, in_relu ? 1 : 0, cur_stream()),
            "act_bwd");
}

void sigmoid_ce_py(torch::Tensor logits, torch::Tensor labels, c10::optional<torch::Tensor> dlogits,
                   c10::optional<torch::Tensor> stats, int64_t B, int64_t C, int64_t ldl, int64_t ldg,
                   double grad_scale) {
  need(logits, at::kFloat, "logits");
  need(labels, at::kInt, "labels");
  TORCH_CHECK(B > 0 && C > 0 && ldl >= C && ldg >= C, "sigmoid_ce: bad shape");
  TORCH_CHECK(logits.numel() >= (B - 1) * ldl + C && labels.numel() >= B, "sigmoid_ce inputs too small");
  dfa::bf16* dl = nullptr;
  if (dlogits.has_value() && dlogits->defined()) {
    need(*dlogits, at::kBFloat16, "dlogits");
    TORCH_CHECK(dlogits->numel() >= (B - 1) * ldg + C, "dlogits too small");
    dl = (dfa::bf16*)dlogits->data_ptr();
  }
  float* sp = nullptr;
  if (stats.has_value() && stats->defined()) {
    need(*stats, at::kFloat, "stats");
    TORCH_CHECK(stats->numel() >= 2, "stats needs 2 floats");
    sp = stats->data_ptr<float>();
  }
  check_hip(dfa::sigmoid_ce(logits.data_ptr<float>(), labels.data_ptr<int>(), dl, sp, B, C, ldl, ldg,
                            (float)grad_scale, cur_stream()),
            "sigmoid_ce");
}

static dfa::Pool2DGeom pool_geom(const std::vector<int64_t>& g) {
  TORCH_CHECK(g.size() == 12, "pool2d: geom = [B, H, W, C, OH, OW, ph, pw, sh, sw, pt, pl]");
  dfa::Pool2DGeom p{};
  p.B = (int)g[0]; p.H = (int)g[1]; p.W = (int)g[2]; p.C = (int)g[3]; p.OH = (int)g[4]; p.OW = (int)g[5];
  p.ph = (int)g[6]; p.pw = (int)g[7]; p.sh = (int)g[8]; p.sw = (int)g[9]; p.pt = (int)g[10]; p.pl = (int)g[11];
  TORCH_CHECK(p.B > 0 && p.H > 0 && p.W > 0 && p.C > 0 && p.OH > 0 && p.OW > 0 && p.ph > 0 && p.pw > 0 && p.sh > 0 &&
                  p.sw > 0 && p.pt >= 0 && p.pl >= 0 && p.pt < p.ph && p.pl < p.pw,
              "pool2d: bad geometry");
  // every window starts inside the padded image
  TORCH_CHECK((p.OH - 1) * p.sh - p.pt < p.H && (p.OW - 1) * p.sw - p.pl < p.W, "pool2d: output too large");
  return p;
}

void pool2d_fwd_py(torch::Tensor x, torch::Tensor y, std::vector<int64_t> geom, bool avg) {
  const dfa::Pool2DGeom g = pool_geom(geom);
  need(x, at::kBFloat16, "pool x");
  need(y, at::kBFloat16, "pool y");
  TORCH_CHECK(x.numel() == (int64_t)g.B * g.H * g.W * g.C && y.numel() == (int64_t)g.B * g.OH * g.OW * g.C,
              "pool2d: tensor sizes do not match the geometry");
  check_hip(dfa::pool2d_fwd((const dfa::bf16*)x.data_ptr(), (dfa::bf16*)y.data_ptr(), g, avg ? 1 : 0, cur_stream()),
            "pool2d_fwd");
}

void pool2d_bwd_py(torch::Tensor x, torch::Tensor dy, torch::Tensor dx, std::vector<int64_t> geom, bool avg,
                   bool in_relu) {
  const dfa::Pool2DGeom g = pool_geom(geom);
  need(x, at::kBFloat16, "pool x");
  need(dy, at::kBFloat16, "pool dy");
  need(dx, at::kBFloat16, "pool dx");
  TORCH_CHECK(x.numel() == (int64_t)g.B * g.H * g.W * g.C && dx.numel() == x.numel() &&
                  dy.numel() == (int64_t)g.B * g.OH * g.OW * g.C,
              "pool2d: tensor sizes do not match the geometry");
  check_hip(dfa::pool2d_bwd((const dfa::bf16*)x.data_ptr(), (const dfa::bf16*)dy.data_ptr(), (dfa::bf16*)dx.data_ptr(),
                            g, avg ? 1 : 0, in_relu ? 1 : 0, cur_stream()),
            "pool2d_bwd");
}

void gap_fwd_py(torch::Tensor x, torch::Tensor y, int64_t B, int64_t HW, int64_t C) {
  need(x, at::kBFloat16, "x");
  need(y, at::kBFloat16, "y");
  TORCH_CHECK(x.numel() >= B * HW * C && y.numel() >= B * C, "gap buffers too small");
  check_hip(dfa::gap_fwd((const dfa::bf16*)x.data_ptr(), (dfa::bf16*)y.data_ptr(), B, HW, C, cur_stream()), "gap_fwd");
}

void gap_bwd_py(torch::Tensor dy, torch::Tensor dx, int64_t B, int64_t HW, int64_t C) {
  need(dy, at::kBFloat16, "dy");
  need(dx, at::kBFloat16, "dx");
  TORCH_CHECK(dx.numel() >= B * HW * C && dy.numel() >= B * C, "gap buffers too small");
  check_hip(dfa::gap_bwd((const dfa::bf16*)dy.data_ptr(), (dfa::bf16*)dx.data_ptr(), B, HW, C, cur_stream()),
            "gap_bwd");
}

// descs: int64 GPU tensor [ndesc][6] laid out as ParamDesc (see optim.hip)
void sgd_multi_py(torch::Tensor descs, int64_t ndesc, int64_t total_blocks, torch::Tensor master, torch::Tensor grad,
                  c10::optional<torch::Tensor> mom, torch::Tensor wbf, torch::Tensor hyper, bool apply_update,
                  c10::optional<torch::Tensor> idx_stream, c10::optional<torch::Tensor> idx_cursor,
                  c10::optional<torch::Tensor> idx_dst, c10::optional<torch::Tensor> descs_host,
                  c10::optional<torch::Tensor> lenet_frag, int64_t frag_w1, int64_t frag_w2,
                  c10::optional<torch::Tensor> lenet_snap, c10::optional<torch::Tensor> step_stats,
                  c10::optional<torch::Tensor> run_stats, uintptr_t gate, uintptr_t mirror) {
  TORCH_CHECK(descs.is_cuda() && descs.scalar_type() == at::kLong && descs.is_contiguous(), "descs must be int64 GPU");
  const dfa::ParamDesc* hd = nullptr;
  if (descs_host.has_value() && descs_host->defined()) {  // same table, host copy: passed in the kernel arguments
    TORCH_CHECK(!descs_host->is_cuda() && descs_host->scalar_type() == at::kLong && descs_host->is_contiguous() &&
                    descs_host->numel() == descs.numel(),
                "descs_host must be the int64 CPU copy of descs");
    hd = reinterpret_cast<const dfa::ParamDesc*>(descs_host->data_ptr());
  }
  static_assert(sizeof(dfa::ParamDesc) == 48, "ParamDesc layout");
  TORCH_CHECK(descs.numel() * 8 >= ndesc * (int64_t)sizeof(dfa::ParamDesc), "descs too small");
  need(master, at::kFloat, "master");
  need(grad, at::kFloat, "grad");
  need(wbf, at::kBFloat16, "wbf");
  need(hyper, at::kFloat, "hyper");
  TORCH_CHECK(hyper.numel() >= 5, "hyper needs [lr, momentum, wd, grad_scale, nesterov]");
  TORCH_CHECK(grad.numel() >= master.numel(), "grad smaller than master");
  float* mp = nullptr;
  if (mom.has_value() && mom->defined()) {
    need(*mom, at::kFloat, "mom");
    TORCH_CHECK(mom->numel() >= master.numel(), "momentum buffer too small");
    mp = mom->data_ptr<float>();
  }
  dfa::IndexStream is{};
  if (idx_stream.has_value() && idx_stream->defined()) {
    TORCH_CHECK(idx_cursor.has_value() && idx_dst.has_value(), "index stream needs cursor and dst");
    need(*idx_stream, at::kLong, "idx_stream");
    need(*idx_cursor, at::kLong, "idx_cursor");
    need(*idx_dst, at::kLong, "idx_dst");
    TORCH_CHECK(idx_stream->dim() == 2 && idx_stream->size(1) == idx_dst->numel() && idx_cursor->numel() >= 1,
                "idx_stream must be [nsteps][B] with B = idx_dst.numel()");
    is.src = reinterpret_cast<const long long*>(idx_stream->data_ptr());
    is.cursor = reinterpret_cast<long long*>(idx_cursor->data_ptr());
    is.dst = reinterpret_cast<long long*>(idx_dst->data_ptr());
    is.B = (int)idx_dst->numel();
    is.nsteps = (int)idx_stream->size(0);
  }
  // device run statistics, with or without an index stream (the same extra workgroup accumulates them)
  if (run_stats.has_value() && run_stats->defined()) {
    TORCH_CHECK(step_stats.has_value() && step_stats->defined(), "run_stats needs step_stats");
    need(*run_stats, at::kFloat, "run_stats");
    need(*step_stats, at::kFloat, "step_stats");
    TORCH_CHECK(run_stats->numel() >= 3 && step_stats->numel() >= 2, "run_stats [3] / step_stats [2]");
    is.run_stats = run_stats->data_ptr<float>();
    is.step_stats = step_stats->data_ptr<float>();
  }
  if (lenet_frag.has_value() && lenet_frag->defined()) {
    TORCH_CHECK(lenet_frag->is_cuda() && lenet_frag->is_contiguous() &&
                    (size_t)lenet_frag->nbytes() >= dfa::lenet_frag_bytes(),
                "lenet_frag: fragment buffer too small");
    TORCH_CHECK(frag_w1 >= 0 && frag_w1 + 150 <= master.numel() && frag_w2 >= 0 && frag_w2 + 2400 <= master.numel(),
                "lenet_frag: conv kernel offsets out of range");
    TORCH_CHECK(!apply_update || (lenet_snap.has_value() && lenet_snap->defined()),
                "lenet_frag: an update needs the pre-update snapshot (lenet_snap)");
    if (lenet_snap.has_value() && lenet_snap->defined()) {
      need(*lenet_snap, at::kFloat, "lenet_snap");
      TORCH_CHECK(lenet_snap->numel() >= 2 * 2550, "lenet_snap must hold 2 x 2550 floats");
      is.snap = lenet_snap->data_ptr<float>();
    }
    is.frag = lenet_frag->data_ptr();
    is.frag_w1 = frag_w1;
    is.frag_w2 = frag_w2;
  }
  // async PS exclusive writer (PSComm.excl_gate / excl_mirror): the update gated on the admission word, the
  // new weights mirrored into the rank's shard
  TORCH_CHECK((gate == 0) == (mirror == 0), "sgd_multi: gate and mirror go together");
  TORCH_CHECK(gate == 0 || (apply_update && !is.frag), "sgd_multi: a gated update without LeNet fragments");
  is.gate = reinterpret_cast<const unsigned*>(gate);
  is.mirror = reinterpret_cast<float*>(mirror);
  const bool any = is.src || is.frag || is.run_stats || is.gate;
  check_hip(dfa::sgd_multi(reinterpret_cast<const dfa::ParamDesc*>(descs.data_ptr()), (int)ndesc, (int)total_blocks,
                           master.data_ptr<float>(), grad.data_ptr<float>(), mp, (dfa::bf16*)wbf.data_ptr(),
                           hyper.data_ptr<float>(), apply_update ? 1 : 0, cur_stream(), any ? &is : nullptr, hd),
            "sgd_multi");
}

void sum_buffers_py(torch::Tensor ptrs, int64_t nin, torch::Tensor out, double scale) {
  TORCH_CHECK(ptrs.is_cuda() && ptrs.scalar_type() == at::kLong && ptrs.numel() >= nin, "ptrs must be int64 GPU");
  need(out, at::kFloat, "out");
  check_hip(dfa::sum_buffers(reinterpret_cast<const float* const*>(ptrs.data_ptr()), (int)nin, out.data_ptr<float>(),
                             out.numel(), (float)scale, cur_stream()),
            "sum_buffers");
}

void axpby_py(torch::Tensor out, torch::Tensor a, torch::Tensor b, double alpha, double beta) {
  need(out, at::kFloat, "out");
  need(a, at::kFloat, "a");
  need(b, at::kFloat, "b");
  TORCH_CHECK(a.numel() == out.numel() && b.numel() == out.numel(), "axpby size mismatch");
  check_hip(dfa::axpby(out.data_ptr<float>(), a.data_ptr<float>(), b.data_ptr<float>(), (float)alpha, (float)beta,
                       out.numel(), cur_stream()),
            "axpby");
}

void bn_check_vec(const torch::Tensor& t, int64_t n, const char* name) {
  need(t, at::kFloat, name);
  TORCH_CHECK(t.numel() >= n, name, " too small");
}

void bn_check_act(const torch::Tensor& t, int64_t n, const char* name) {
  need(t, at::kBFloat16, name);
  TORCH_CHECK(t.numel() >= n, name, " too small");
}

void bn_check_stats_ws(const torch::Tensor& ws, const torch::Tensor& counter, int64_t M, int64_t C) {
  TORCH_CHECK(C > 0 && C <= 1024 && M > 0, "bn: need 0 < C <= 1024 and M > 0");
  TORCH_CHECK(C % 8 == 0 || C <= 256, "bn: C must be a multiple of 8 or <= 256");
  bn_check_vec(ws, dfa::bn_stats_ws_floats((int)M, (int)C), "bn workspace");
  need(counter, at::kInt, "bn counter");
  TORCH_CHECK(counter.numel() >= dfa::bn_stats_counters((int)M, (int)C), "bn counter: need ",
              dfa::bn_stats_counters((int)M, (int)C), " int32 tickets");
}

// forward statistics: batch mean / invstd (+ running statistics) in one launch
void bn_stats_fwd_py(torch::Tensor x, torch::Tensor mean, torch::Tensor invstd, c10::optional<torch::Tensor> run_mean,
                     c10::optional<torch::Tensor> run_var, torch::Tensor ws, torch::Tensor counter, int64_t M,
                     int64_t C, double momentum, double eps) {
  bn_check_act(x, M * C, "x");
  bn_check_vec(mean, C, "mean");
  bn_check_vec(invstd, C, "invstd");
  const bool run = run_mean.has_value() && run_mean->defined();
  if (run) {
    bn_check_vec(*run_mean, C, "run_mean");
    TORCH_CHECK(run_var.has_value() && run_var->defined(), "run_var required with run_mean");
    bn_check_vec(*run_var, C, "run_var");
  }
  bn_check_stats_ws(ws, counter, M, C);
  dfa::BnStatsArgs a{};
  a.x = (const dfa::bf16*)x.data_ptr();
  a.mean_out = mean.data_ptr<float>();
  a.invstd_out = invstd.data_ptr<float>();
  a.run_mean = run ? run_mean->data_ptr<float>() : nullptr;
  a.run_var = run ? run_var->data_ptr<float>() : nullptr;
  a.ws = ws.data_ptr<float>();
  a.counter = reinterpret_cast<unsigned*>(counter.data_ptr<int>());
  a.M = (int)M; a.C = (int)C; a.momentum = (float)momentum; a.eps = (float)eps;
  check_hip(dfa::bn_stats(a, 0, cur_stream()), "bn_stats_fwd");
}

// backward statistics: dgamma/dbeta + dx coefficients coef[3][C]; g = dy * (mask > 0) when mask is given
void bn_stats_bwd_py(torch::Tensor x, c10::optional<torch::Tensor> mask, torch::Tensor dy, torch::Tensor gamma,
                     torch::Tensor mean, torch::Tensor invstd, torch::Tensor dgamma, torch::Tensor dbeta,
                     torch::Tensor coef, torch::Tensor ws, torch::Tensor counter, int64_t M, int64_t C, double gscale) {
  bn_check_act(x, M * C, "x");
  bn_check_act(dy, M * C, "dy");
  if (mask.has_value() && mask->defined()) bn_check_act(*mask, M * C, "mask");
  bn_check_vec(gamma, C, "gamma");
  bn_check_vec(mean, C, "mean");
  bn_check_vec(invstd, C, "invstd");
  bn_check_vec(dgamma, C, "dgamma");
  bn_check_vec(dbeta, C, "dbeta");
  bn_check_vec(coef, 3 * C, "coef");
  bn_check_stats_ws(ws, counter, M, C);
  dfa::BnStatsArgs a{};
  a.x = (const dfa::bf16*)x.data_ptr();
  a.mask = cptr<dfa::bf16>(mask);
  a.dy = (const dfa::bf16*)dy.data_ptr();
  a.gamma = gamma.data_ptr<float>();
  a.mean = mean.data_ptr<float>();
  a.invstd = invstd.data_ptr<float>();
  a.dgamma = dgamma.data_ptr<float>();
  a.dbeta = dbeta.data_ptr<float>();
  a.coef = coef.data_ptr<float>();
  a.ws = ws.data_ptr<float>();
  a.counter = reinterpret_cast<unsigned*>(counter.data_ptr<int>());
  a.M = (int)M; a.C = (int)C; a.gscale = (float)gscale;
  check_hip(dfa::bn_stats(a, 1, cur_stream()), "bn_stats_bwd");
}

// y = act(bn(x) [+ r | + bn_r(r)]); eval: mean/invstd are the running mean / variance
void bn_apply_py(torch::Tensor x, torch::Tensor y, torch::Tensor gamma, torch::Tensor beta, torch::Tensor mean,
                 torch::Tensor invstd, c10::optional<torch::Tensor> r, c10::optional<torch::Tensor> rgamma,
                 c10::optional<torch::Tensor> rbeta, c10::optional<torch::Tensor> rmean,
                 c10::optional<torch::Tensor> rinvstd, int64_t M, int64_t C, bool relu, bool eval, double eps) {
  bn_check_act(x, M * C, "x");
  bn_check_act(y, M * C, "y");
  for (auto* t : {&gamma, &beta, &mean, &invstd}) bn_check_vec(*t, C, "bn vector");
  dfa::BnApplyArgs a{};
  a.x = (const dfa::bf16*)x.data_ptr();
  a.y = (dfa::bf16*)y.data_ptr();
  a.gamma = gamma.data_ptr<float>();
  a.beta = beta.data_ptr<float>();
  a.mean = mean.data_ptr<float>();
  a.invstd = invstd.data_ptr<float>();
  if (r.has_value() && r->defined()) {
    bn_check_act(*r, M * C, "residual");
    a.r = (const dfa::bf16*)r->data_ptr();
    if (rgamma.has_value() && rgamma->defined()) {
      for (auto* t : {&rgamma, &rbeta, &rmean, &rinvstd}) {
        TORCH_CHECK(t->has_value() && (*t)->defined(), "residual BN needs gamma, beta, mean, invstd");
        bn_check_vec(**t, C, "residual bn vector");
      }
      a.rgamma = rgamma->data_ptr<float>();
      a.rbeta = rbeta->data_ptr<float>();
      a.rmean = rmean->data_ptr<float>();
      a.rinvstd = rinvstd->data_ptr<float>();
    }
  }
  a.M = (int)M; a.C = (int)C; a.relu = relu ? 1 : 0; a.eval = eval ? 1 : 0; a.eps = (float)eps;
  check_hip(dfa::bn_apply(a, cur_stream()), "bn_apply");
}

// statistics + apply in one launch (training forward): y = act(bn(x) [+ r | + bn_r(r)]); the generation
// word of the in-launch hand-off is counter[64]
void bn_fwd_fused_py(torch::Tensor x, torch::Tensor y, torch::Tensor gamma, torch::Tensor beta, torch::Tensor mean,
                     torch::Tensor invstd, c10::optional<torch::Tensor> run_mean, c10::optional<torch::Tensor> run_var,
                     c10::optional<torch::Tensor> r, c10::optional<torch::Tensor> rgamma,
                     c10::optional<torch::Tensor> rbeta, c10::optional<torch::Tensor> rmean,
                     c10::optional<torch::Tensor> rinvstd, torch::Tensor ws, torch::Tensor counter, int64_t M,
                     int64_t C, bool relu, double momentum, double eps) {
  TORCH_CHECK(dfa::bn_fused_ok((int)C), "bn_fwd_fused: C must be a multiple of 8 (<= 1024)");
  bn_check_act(x, M * C, "x");
  bn_check_act(y, M * C, "y");
  for (auto* t : {&gamma, &beta, &mean, &invstd}) bn_check_vec(*t, C, "bn vector");
  const bool run = run_mean.has_value() && run_mean->defined();
  if (run) {
    bn_check_vec(*run_mean, C, "run_mean");
    TORCH_CHECK(run_var.has_value() && run_var->defined(), "run_var required with run_mean");
    bn_check_vec(*run_var, C, "run_var");
  }
  bn_check_stats_ws(ws, counter, M, C);
  TORCH_CHECK(counter.numel() >= 65, "bn_fwd_fused: counter needs 65 words (generation at 64)");
  TORCH_CHECK(ws.numel() >= (1008 + 63) * 2 * C, "bn_fwd_fused: workspace needs (1008 + 63) x 2C floats");
  dfa::BnStatsArgs a{};
  a.x = (const dfa::bf16*)x.data_ptr();
  a.mean_out = mean.data_ptr<float>();
  a.invstd_out = invstd.data_ptr<float>();
  a.run_mean = run ? run_mean->data_ptr<float>() : nullptr;
  a.run_var = run ? run_var->data_ptr<float>() : nullptr;
  a.ws = ws.data_ptr<float>();
  a.counter = reinterpret_cast<unsigned*>(counter.data_ptr<int>());
  a.M = (int)M; a.C = (int)C; a.momentum = (float)momentum; a.eps = (float)eps;
  dfa::BnApplyArgs p{};
  p.x = a.x;
  p.y = (dfa::bf16*)y.data_ptr();
  p.gamma = gamma.data_ptr<float>();
  p.beta = beta.data_ptr<float>();
  p.mean = a.mean_out;
  p.invstd = a.invstd_out;
  if (r.has_value() && r->defined()) {
    bn_check_act(*r, M * C, "residual");
    p.r = (const dfa::bf16*)r->data_ptr();
    if (rgamma.has_value() && rgamma->defined()) {
      for (auto* t : {&rgamma, &rbeta, &rmean, &rinvstd}) {
        TORCH_CHECK(t->has_value() && (*t)->defined(), "residual BN needs gamma, beta, mean, invstd");
        bn_check_vec(**t, C, "residual bn vector");
      }
      p.rgamma = rgamma->data_ptr<float>();
      p.rbeta = rbeta->data_ptr<float>();
      p.rmean = rmean->data_ptr<float>();
      p.rinvstd = rinvstd->data_ptr<float>();
    }
  }
  p.M = (int)M; p.C = (int)C; p.relu = relu ? 1 : 0; p.eval = 0; p.eps = (float)eps;
  check_hip(dfa::bn_fwd_fused(a, p, a.counter + 64, cur_stream()), "bn_fwd_fused");
}

// backward statistics + dx in one launch; generation word counter[64]
void bn_bwd_fused_py(torch::Tensor x, c10::optional<torch::Tensor> mask, torch::Tensor dy, torch::Tensor dx,
                     torch::Tensor gamma, torch::Tensor mean, torch::Tensor invstd, torch::Tensor dgamma,
                     torch::Tensor dbeta, torch::Tensor coef, torch::Tensor ws, torch::Tensor counter, int64_t M,
                     int64_t C, double gscale) {
  TORCH_CHECK(dfa::bn_fused_ok((int)C), "bn_bwd_fused: C must be a multiple of 8 (<= 1024)");
  bn_check_act(x, M * C, "x");
  bn_check_act(dy, M * C, "dy");
  bn_check_act(dx, M * C, "dx");
  if (mask.has_value() && mask->defined()) bn_check_act(*mask, M * C, "mask");
  bn_check_vec(gamma, C, "gamma");
  bn_check_vec(mean, C, "mean");
  bn_check_vec(invstd, C, "invstd");
  bn_check_vec(dgamma, C, "dgamma");
  bn_check_vec(dbeta, C, "dbeta");
  bn_check_vec(coef, 3 * C, "coef");
  bn_check_stats_ws(ws, counter, M, C);
  TORCH_CHECK(counter.numel() >= 65, "bn_bwd_fused: counter needs 65 words (generation at 64)");
  TORCH_CHECK(ws.numel() >= (1008 + 63) * 2 * C, "bn_bwd_fused: workspace needs (1008 + 63) x 2C floats");
  dfa::BnStatsArgs a{};
  a.x = (const dfa::bf16*)x.data_ptr();
  a.mask = cptr<dfa::bf16>(mask);
  a.dy = (const dfa::bf16*)dy.data_ptr();
  a.gamma = gamma.data_ptr<float>();
  a.mean = mean.data_ptr<float>();
  a.invstd = invstd.data_ptr<float>();
  a.dgamma = dgamma.data_ptr<float>();
  a.dbeta = dbeta.data_ptr<float>();
  a.coef = coef.data_ptr<float>();
  a.ws = ws.data_ptr<float>();
  a.counter = reinterpret_cast<unsigned*>(counter.data_ptr<int>());
  a.M = (int)M; a.C = (int)C; a.gscale = (float)gscale;
  check_hip(dfa::bn_bwd_fused(a, (dfa::bf16*)dx.data_ptr(), a.counter + 64, cur_stream()), "bn_bwd_fused");
}

void bn_dx_py(torch::Tensor x, c10::optional<torch::Tensor> mask, torch::Tensor dy, torch::Tensor dx,
              torch::Tensor coef, int64_t M, int64_t C) {
  bn_check_act(x, M * C, "x");
  bn_check_act(dy, M * C, "dy");
  bn_check_act(dx, M * C, "dx");
  if (mask.has_value() && mask->defined()) bn_check_act(*mask, M * C, "mask");
  bn_check_vec(coef, 3 * C, "coef");
  check_hip(dfa::bn_dx((const dfa::bf16*)x.data_ptr(), cptr<dfa::bf16>(mask), (const dfa::bf16*)dy.data_ptr(),
                       (dfa::bf16*)dx.data_ptr(), coef.data_ptr<float>(), (int)M, (int)C, cur_stream()),
            "bn_dx");
}

// BatchNorm consumers that finalise epilogue-accumulated sums (csrc/bn.hip, kernels.h BnAccFin)
static dfa::BnAccFin bn_fin(const torch::Tensor& acc, const c10::optional<torch::Tensor>& zero, int64_t C) {
  need(acc, at::kDouble, "bn acc");
  TORCH_CHECK(acc.numel() % (2 * C) == 0 && acc.numel() / (2 * C) <= dfa::kBnAccMaxRep, "bn acc must be [nrep][2][C]");
  dfa::BnAccFin f{};
  f.acc = acc.data_ptr<double>();
  f.nrep = (int)(acc.numel() / (2 * C));
  if (zero.has_value() && zero->defined()) {
    need(*zero, at::kDouble, "bn acc zero");
    TORCH_CHECK(zero->numel() == acc.numel(), "bn acc zero must match acc");
    f.zero = zero->data_ptr<double>();
  }
  return f;
}

// y = act(bn(x) [+ r | + bn_r(r)]) in training mode, statistics from the producer's sums; workgroup 0
// writes mean / invstd / running statistics (of the residual BN too) and clears `zero` / `rzero`
void bn_apply_acc_py(torch::Tensor x, torch::Tensor y, torch::Tensor gamma, torch::Tensor beta, torch::Tensor acc,
                     c10::optional<torch::Tensor> zero, torch::Tensor mean, torch::Tensor invstd,
                     c10::optional<torch::Tensor> run_mean, c10::optional<torch::Tensor> run_var,
                     c10::optional<torch::Tensor> r, std::vector<torch::Tensor> rbn, int64_t M, int64_t C, bool relu,
                     double momentum, double eps) {
  TORCH_CHECK(C % 8 == 0 && C <= 1024, "bn_apply_acc: C % 8 == 0, C <= 1024");
  bn_check_act(x, M * C, "x");
  bn_check_act(y, M * C, "y");
  for (auto* t : {&gamma, &beta, &mean, &invstd}) bn_check_vec(*t, C, "bn vector");
  dfa::BnApplyArgs a{};
  a.x = (const dfa::bf16*)x.data_ptr();
  a.y = (dfa::bf16*)y.data_ptr();
  a.gamma = gamma.data_ptr<float>();
  a.beta = beta.data_ptr<float>();
  a.M = (int)M; a.C = (int)C; a.relu = relu ? 1 : 0; a.eval = 0; a.eps = (float)eps;
  dfa::BnAccFin f = bn_fin(acc, zero, C);
  f.mean = mean.data_ptr<float>();
  f.invstd = invstd.data_ptr<float>();
  const bool run = run_mean.has_value() && run_mean->defined();
  if (run) {
    bn_check_vec(*run_mean, C, "run_mean");
    TORCH_CHECK(run_var.has_value() && run_var->defined(), "run_var with run_mean");
    bn_check_vec(*run_var, C, "run_var");
    f.run_mean = run_mean->data_ptr<float>();
    f.run_var = run_var->data_ptr<float>();
  }
  f.momentum = (float)momentum;
  f.eps = (float)eps;
  dfa::BnAccFin fr{};
  const bool has_rbn = !rbn.empty();
  if (r.has_value() && r->defined()) {
    bn_check_act(*r, M * C, "residual");
    a.r = (const dfa::bf16*)r->data_ptr();
    if (has_rbn) {
      // [gamma, beta, acc, zero (or empty), mean, invstd, run_mean, run_var]
      TORCH_CHECK(rbn.size() == 8, "residual BN: [gamma, beta, acc, zero, mean, invstd, run_mean, run_var]");
      for (int i : {0, 1, 4, 5, 6, 7}) bn_check_vec(rbn[i], C, "residual bn vector");
      a.rgamma = rbn[0].data_ptr<float>();
      a.rbeta = rbn[1].data_ptr<float>();
      fr = bn_fin(rbn[2], rbn[3].numel() ? c10::optional<torch::Tensor>(rbn[3]) : c10::nullopt, C);
      fr.mean = rbn[4].data_ptr<float>();
      fr.invstd = rbn[5].data_ptr<float>();
      fr.run_mean = rbn[6].data_ptr<float>();
      fr.run_var = rbn[7].data_ptr<float>();
      fr.momentum = (float)momentum;
      fr.eps = (float)eps;
      a.rmean = fr.mean;  // non-null marks RES 2
      a.rinvstd = fr.invstd;
    }
  } else {
    TORCH_CHECK(!has_rbn, "residual BN without a residual");
  }
  check_hip(dfa::bn_apply_acc(a, f, has_rbn ? &fr : nullptr, cur_stream()), "bn_apply_acc");
}

// dx = k1 g + k2 x + k3 from the producer's backward sums; workgroup 0 writes dgamma / dbeta (x gscale) and
// coef, and clears `zero`
void bn_dx_acc_py(torch::Tensor x, torch::Tensor g, torch::Tensor dx, torch::Tensor acc,
                  c10::optional<torch::Tensor> zero, torch::Tensor gamma, torch::Tensor mean, torch::Tensor invstd,
                  torch::Tensor dgamma, torch::Tensor dbeta, torch::Tensor coef, int64_t M, int64_t C, double gscale) {
  TORCH_CHECK(C % 8 == 0 && C <= 1024, "bn_dx_acc: C % 8 == 0, C <= 1024");
  bn_check_act(x, M * C, "x");
  bn_check_act(g, M * C, "g");
  bn_check_act(dx, M * C, "dx");
  for (auto* t : {&gamma, &mean, &invstd, &dgamma, &dbeta}) bn_check_vec(*t, C, "bn vector");
  bn_check_vec(coef, 3 * C, "coef");
  dfa::BnAccFin f = bn_fin(acc, zero, C);
  f.mean = mean.data_ptr<float>();
  f.invstd = invstd.data_ptr<float>();
  f.gamma = gamma.data_ptr<float>();
  f.dgamma = dgamma.data_ptr<float>();
  f.dbeta = dbeta.data_ptr<float>();
  f.coef = coef.data_ptr<float>();
  f.gscale = (float)gscale;
  check_hip(dfa::bn_dx_acc((const dfa::bf16*)x.data_ptr(), (const dfa::bf16*)g.data_ptr(), (dfa::bf16*)dx.data_ptr(),
                           f, (int)M, (int)C, cur_stream()),
            "bn_dx_acc");
}

// GAP backward with relu' (mask) and the BatchNorm backward sums of the result (ResNet's last block)
void gap_bwd_bn_py(torch::Tensor dy, torch::Tensor mask, torch::Tensor dx, int64_t B, int64_t HW, int64_t C,
                   torch::Tensor acc, std::vector<torch::Tensor> bn_in) {
  need(dy, at::kBFloat16, "dy");
  need(mask, at::kBFloat16, "mask");
  need(dx, at::kBFloat16, "dx");
  TORCH_CHECK(dy.numel() >= B * C && mask.numel() >= B * HW * C && dx.numel() >= B * HW * C, "gap_bwd_bn sizes");
  TORCH_CHECK(C % 4 == 0 && C <= 1024 && 256 % (C / 4) == 0, "gap_bwd_bn: C / 4 must divide 256");
  need(acc, at::kDouble, "bn acc");
  TORCH_CHECK(acc.numel() % (2 * C) == 0, "bn acc must be [nrep][2][C]");
  TORCH_CHECK(bn_in.size() == 3, "gap_bwd_bn: [x, mean, invstd]");
  need(bn_in[0], at::kBFloat16, "bn x");
  TORCH_CHECK(bn_in[0].numel() >= B * HW * C, "bn x too small");
  bn_check_vec(bn_in[1], C, "bn mean");
  bn_check_vec(bn_in[2], C, "bn invstd");
  dfa::BnAcc e{};
  e.acc = acc.data_ptr<double>();
  e.nrep = (int)(acc.numel() / (2 * C));
  e.mode = 1;
  e.x = (const dfa::bf16*)bn_in[0].data_ptr();
  e.mean = bn_in[1].data_ptr<float>();
  e.invstd = bn_in[2].data_ptr<float>();
  check_hip(dfa::gap_bwd_bn((const dfa::bf16*)dy.data_ptr(), (const dfa::bf16*)mask.data_ptr(),
                            (dfa::bf16*)dx.data_ptr(), (int)B, (int)HW, (int)C, e, cur_stream()),
            "gap_bwd_bn");
}

// geometry: [B, H, W, C, KH, KW, pad, N]
struct CPIn {
  const void* x = nullptr;
  int u8 = 0;
  const long long* idx = nullptr;
  long long nrows = 0;
};

CPIn cp_input(const torch::Tensor& x, const c10::optional<torch::Tensor>& idx, int64_t B, int64_t HWC) {
  CPIn r;
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "x must be a contiguous GPU tensor");
  if (idx.has_value() && idx->defined()) {
    need(*idx, at::kLong, "idx");
    TORCH_CHECK(idx->numel() >= B, "idx shorter than the batch");
    TORCH_CHECK(x.scalar_type() == at::kByte || x.scalar_type() == at::kBFloat16, "dataset must be u8 or bf16");
    TORCH_CHECK(x.dim() >= 1 && x.size(0) > 0 && x.numel() / x.size(0) == HWC, "dataset row size mismatch");
    TORCH_CHECK(x.scalar_type() == at::kByte, "indexed input must be a uint8 dataset");
    r.u8 = 1;
    r.idx = reinterpret_cast<const long long*>(idx->data_ptr<int64_t>());
    r.nrows = x.size(0);
  } else {
    TORCH_CHECK(x.scalar_type() == at::kBFloat16, "x must be bf16");
    TORCH_CHECK(x.numel() >= B * HWC, "x too small");
  }
  r.x = x.data_ptr();
  return r;
}

void convpool_fwd_py(torch::Tensor x, c10::optional<torch::Tensor> idx, double scale, torch::Tensor w,
                     c10::optional<torch::Tensor> bias, torch::Tensor p, c10::optional<torch::Tensor> code,
                     std::vector<int64_t> geom) {
  TORCH_CHECK(geom.size() == 8, "geom = [B,H,W,C,KH,KW,pad,N]");
  const int B = geom[0], H = geom[1], W = geom[2], C = geom[3], KH = geom[4], KW = geom[5], pad = geom[6], N = geom[7];
  TORCH_CHECK(dfa::convpool_supported(H, W, C, KH, KW, pad, N), "convpool: unsupported geometry");
  CPIn in = cp_input(x, idx, B, (int64_t)H * W * C);
  need(w, at::kBFloat16, "w");
  // row-segment layout [Npad16][Kpad2] (ParamSpec.row_pad / row_cp, convpool_fwd_layout)
  int Cp = 0, Kpad2 = 0, pair = 0;
  dfa::convpool_fwd_layout(H, W, C, KH, KW, pad, N, &Cp, &Kpad2, &pair);
  TORCH_CHECK(w.numel() >= (int64_t)((N + 15) / 16 * 16) * Kpad2 && w.size(-1) == Kpad2,
              "w must be the row-segment layout [Npad16][", Kpad2, "] (channel stride ", Cp, ")");
  const int OH = H + 2 * pad - KH + 1, OW = W + 2 * pad - KW + 1;
  const int64_t pn = (int64_t)B * (OH / 2) * (OW / 2) * N;
  need(p, at::kBFloat16, "p");
  TORCH_CHECK(p.numel() >= pn, "p too small");
  uint8_t* cp = nullptr;
  if (code.has_value() && code->defined()) {
    need(*code, at::kByte, "code");
    TORCH_CHECK(code->numel() >= pn, "code too small");
    cp = code->data_ptr<uint8_t>();
  }
  if (bias.has_value() && bias->defined()) {
    need(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() >= N, "bias too small");
  }
  check_hip(dfa::convpool_fwd(in.x, in.u8, in.idx, in.nrows, (float)scale, B, H, W, C, KH, KW, pad, N,
                              (const dfa::bf16*)w.data_ptr(), cptr<float>(bias), (dfa::bf16*)p.data_ptr(), cp,
                              cur_stream()),
            "convpool_fwd");
}

int64_t convpool_wgrad_py(torch::Tensor x, c10::optional<torch::Tensor> idx, double scale, torch::Tensor dp,
                          torch::Tensor code, torch::Tensor gw, c10::optional<torch::Tensor> gb, torch::Tensor ws,
                          std::vector<int64_t> geom, bool defer) {
  TORCH_CHECK(geom.size() == 8, "geom = [B,H,W,C,KH,KW,pad,N]");
  const int B = geom[0], H = geom[1], W = geom[2], C = geom[3], KH = geom[4], KW = geom[5], pad = geom[6], N = geom[7];
  TORCH_CHECK(dfa::convpool_supported(H, W, C, KH, KW, pad, N), "convpool: unsupported geometry");
  CPIn in = cp_input(x, idx, B, (int64_t)H * W * C);
  const int OH = H + 2 * pad - KH + 1, OW = W + 2 * pad - KW + 1;
  const int64_t pn = (int64_t)B * (OH / 2) * (OW / 2) * N;
  need(dp, at::kBFloat16, "dp");
  need(code, at::kByte, "code");
  TORCH_CHECK(dp.numel() >= pn && code.numel() >= pn, "dp/code too small");
  need(gw, at::kFloat, "gw");
  TORCH_CHECK(gw.numel() >= (int64_t)N * KH * KW * C, "gw too small");
  float* gbp = nullptr;
  if (gb.has_value() && gb->defined()) {
    need(*gb, at::kFloat, "gb");
    TORCH_CHECK(gb->numel() >= N, "gb too small");
    gbp = gb->data_ptr<float>();
  }
  need(ws, at::kFloat, "workspace");
  int slabs = 0;
  check_hip(dfa::convpool_wgrad(in.x, in.u8, in.idx, in.nrows, (float)scale, B, H, W, C, KH, KW, pad, N,
                                (const dfa::bf16*)dp.data_ptr(), code.data_ptr<uint8_t>(), gw.data_ptr<float>(), gbp,
                                ws.data_ptr<float>(), (size_t)ws.numel(), cur_stream(), defer ? &slabs : nullptr),
            "convpool_wgrad");
  return slabs;  // > 0: the slab reduction was deferred (run it with slab_reduce_multi)
}

// One launch for several deferred slab reductions: segs = [(partial, gw, gb|None, N, K, Kt, S, scale), ...]
void slab_reduce_multi_py(std::vector<py::tuple> segs) {
  TORCH_CHECK(!segs.empty() && (int)segs.size() <= dfa::kMaxSlabSegs, "slab_reduce_multi: 1..8 segments");
  dfa::SlabSegs ss{};
  ss.n = (int)segs.size();
  for (size_t i = 0; i < segs.size(); ++i) {
    const py::tuple& t = segs[i];
    TORCH_CHECK(t.size() == 8, "segment = (partial, gw, gb, N, K, Kt, S, scale)");
    auto partial = t[0].cast<torch::Tensor>();
    auto gw = t[1].cast<torch::Tensor>();
    const int N = t[3].cast<int>(), K = t[4].cast<int>(), Kt = t[5].cast<int>(), S = t[6].cast<int>();
    need(partial, at::kFloat, "partial");
    need(gw, at::kFloat, "gw");
    TORCH_CHECK(N > 0 && K > 0 && Kt >= K && S > 0, "slab_reduce_multi: bad segment sizes");
    TORCH_CHECK(partial.numel() >= (int64_t)S * N * Kt && gw.numel() >= (int64_t)N * K, "slab_reduce_multi: buffers too small");
    dfa::SlabSeg& sg = ss.s[i];
    sg.partial = partial.data_ptr<float>();
    sg.gw = gw.data_ptr<float>();
    sg.gb = nullptr;
    if (!t[2].is_none()) {
      auto gb = t[2].cast<torch::Tensor>();
      need(gb, at::kFloat, "gb");
      TORCH_CHECK(gb.numel() >= N, "gb too small");
      sg.gb = gb.data_ptr<float>();
    }
    sg.N = N; sg.K = K; sg.Kt = Kt; sg.S = S;
    sg.scale = t[7].cast<float>();
  }
  check_hip(dfa::slab_reduce_multi(ss, cur_stream()), "slab_reduce_multi");
}

void convpool_dgrad_py(torch::Tensor dp, torch::Tensor code, torch::Tensor wt, torch::Tensor dx,
                       std::vector<int64_t> geom) {
  TORCH_CHECK(geom.size() == 8, "geom = [B,H,W,C,KH,KW,pad,N]");
  const int B = geom[0], H = geom[1], W = geom[2], C = geom[3], KH = geom[4], KW = geom[5], pad = geom[6], N = geom[7];
  TORCH_CHECK(dfa::convpool_supported(H, W, C, KH, KW, pad, N), "convpool: unsupported geometry");
  const int OH = H + 2 * pad - KH + 1, OW = W + 2 * pad - KW + 1;
  const int64_t pn = (int64_t)B * (OH / 2) * (OW / 2) * N;
  need(dp, at::kBFloat16, "dp");
  need(code, at::kByte, "code");
  TORCH_CHECK(dp.numel() >= pn && code.numel() >= pn, "dp/code too small");
  need(wt, at::kBFloat16, "wt");
  int pair = 0, K2pad = 0;
  dfa::convpool_dgrad_layout(H, W, C, KH, KW, pad, N, &pair, &K2pad);
  const int rows = pair ? 16 : (C + 15) / 16 * 16;
  TORCH_CHECK(wt.size(-1) == K2pad && wt.numel() >= (int64_t)rows * K2pad, "wt must be the dgrad layout [", rows,
              "][", K2pad, "] (pair ", pair, ")");
  need(dx, at::kBFloat16, "dx");
  TORCH_CHECK(dx.numel() >= (int64_t)B * H * W * C, "dx too small");
  check_hip(dfa::convpool_dgrad((const dfa::bf16*)dp.data_ptr(), code.data_ptr<uint8_t>(),
                                (const dfa::bf16*)wt.data_ptr(), (dfa::bf16*)dx.data_ptr(), B, H, W, C, KH, KW, pad,
                                N, cur_stream()),
            "convpool_dgrad");
}

void gather_labels_py(torch::Tensor labels, torch::Tensor idx, torch::Tensor out) {
  need(labels, at::kInt, "labels");
  need(idx, at::kLong, "idx");
  need(out, at::kInt, "out");
  TORCH_CHECK(out.numel() >= idx.numel() && labels.numel() > 0, "gather_labels sizes");
  check_hip(dfa::gather_labels(labels.data_ptr<int>(), reinterpret_cast<const long long*>(idx.data_ptr<int64_t>()),
                               out.data_ptr<int>(), (int)idx.numel(), labels.numel(), cur_stream()),
            "gather_labels");
}

// Fused dense head: per layer l tensors (w, wt?, b?, gw, gb?, hT?, dzT) and dims (K, N).
void head_train_py(std::vector<torch::Tensor> w, std::vector<c10::optional<torch::Tensor>> wt,
                   std::vector<c10::optional<torch::Tensor>> b, std::vector<torch::Tensor> gw,
                   std::vector<c10::optional<torch::Tensor>> gb, std::vector<c10::optional<torch::Tensor>> hT,
                   std::vector<torch::Tensor> dzT, std::vector<int64_t> K, std::vector<int64_t> N, torch::Tensor x,
                   bool x_relu, torch::Tensor xT, c10::optional<torch::Tensor> dx,
                   c10::optional<torch::Tensor> logits, torch::Tensor labels, c10::optional<torch::Tensor> idx,
                   double grad_scale, torch::Tensor loss_part, torch::Tensor stats, int64_t phases,
                   double dx_scale) {
  const int nl = (int)w.size();
  TORCH_CHECK(phases >= 1 && phases <= 3, "head: phases must be 1, 2 or 3");
  TORCH_CHECK(nl >= 1 && nl <= dfa::kHeadMaxLayers, "head: 1..", dfa::kHeadMaxLayers, " layers");
  TORCH_CHECK((int)wt.size() == nl && (int)b.size() == nl && (int)gw.size() == nl && (int)gb.size() == nl &&
                  (int)hT.size() == nl && (int)dzT.size() == nl && (int)K.size() == nl && (int)N.size() == nl,
              "head: per-layer lists must have equal length");
  need(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() >= 2, "x must be [B, ...]");
  const int64_t B = x.size(0);
  const int64_t ldt = (B + 31) / 32 * 32;
  TORCH_CHECK(x.numel() == B * K[0], "x must have B*K0 elements");
  // (the weight-gradient phase alone streams X^T: any K0; the forward phase stages X rows in LDS)
  TORCH_CHECK(K[0] % 8 == 0 && (K[0] <= 1024 || phases == 2), "head: K0 must be a multiple of 8 and <= 1024");
  TORCH_CHECK(N[nl - 1] <= 16, "head: at most 16 classes");
  dfa::HeadArgs a{};
  a.nl = nl;
  a.B = (int)B;
  a.ldt = (int)ldt;
  a.x_relu = x_relu ? 1 : 0;
  for (int l = 0; l < nl; ++l) {
    dfa::HeadLayer& L = a.L[l];
    L.K = (int)K[l];
    L.N = (int)N[l];
    TORCH_CHECK(L.N <= 256 || l == 0, "head: hidden widths must be <= 256");
    TORCH_CHECK(l == 0 || K[l] == N[l - 1], "head: layer ", l, " input width must equal layer ", l - 1, " width");
    L.Kpad = (L.K + 31) / 32 * 32;
    L.ldwt = (L.N + 31) / 32 * 32;
    need(w[l], at::kBFloat16, "w");
    TORCH_CHECK(w[l].numel() >= (int64_t)((L.N + 15) / 16 * 16) * L.Kpad && w[l].size(-1) == L.Kpad,
                "head: w must be [Npad16][Kpad32]");
    L.w = reinterpret_cast<const dfa::bf16*>(w[l].data_ptr());
    const bool need_wt = l > 0 || (dx.has_value() && dx->defined());
    if (need_wt) {
      TORCH_CHECK(wt[l].has_value() && wt[l]->defined(), "head: dgrad-layout weights required for layer ", l);
      need(*wt[l], at::kBFloat16, "wt");
      TORCH_CHECK(wt[l]->size(-1) == L.ldwt && wt[l]->numel() >= (int64_t)((L.K + 15) / 16 * 16) * L.ldwt,
                  "head: wt must be [Kpad16][pad32(N)]");
      L.wt = reinterpret_cast<const dfa::bf16*>(wt[l]->data_ptr());
    }
    if (b[l].has_value() && b[l]->defined()) {
      need(*b[l], at::kFloat, "b");
      TORCH_CHECK(b[l]->numel() >= L.N, "head: bias too small");
      L.b = b[l]->data_ptr<float>();
    }
    need(gw[l], at::kFloat, "gw");
    TORCH_CHECK(gw[l].numel() >= (int64_t)L.N * L.K, "head: gw too small");
    L.gw = gw[l].data_ptr<float>();
    if (gb[l].has_value() && gb[l]->defined()) {
      need(*gb[l], at::kFloat, "gb");
      TORCH_CHECK(gb[l]->numel() >= L.N, "head: gb too small");
      L.gb = gb[l]->data_ptr<float>();
    }
    if (l < nl - 1) {
      TORCH_CHECK(hT[l].has_value() && hT[l]->defined(), "head: hT required for hidden layers");
      need(*hT[l], at::kBFloat16, "hT");
      TORCH_CHECK(hT[l]->numel() >= (int64_t)L.N * ldt, "head: hT must be [N][round32(B)]");
      L.hT = reinterpret_cast<dfa::bf16*>(hT[l]->data_ptr());
    }
    need(dzT[l], at::kBFloat16, "dzT");
    TORCH_CHECK(dzT[l].numel() >= (int64_t)L.N * ldt, "head: dzT must be [N][round32(B)]");
    L.dzT = reinterpret_cast<dfa::bf16*>(dzT[l].data_ptr());
  }
  a.x = reinterpret_cast<const dfa::bf16*>(x.data_ptr());
  need(xT, at::kBFloat16, "xT");
  TORCH_CHECK(xT.numel() >= K[0] * ldt, "head: xT must be [K0][round32(B)]");
  a.xT = reinterpret_cast<dfa::bf16*>(xT.data_ptr());
  if (dx.has_value() && dx->defined()) {
    need(*dx, at::kBFloat16, "dx");
    TORCH_CHECK(dx->numel() >= B * K[0], "head: dx too small");
    a.dx = reinterpret_cast<dfa::bf16*>(dx->data_ptr());
  }
  if (logits.has_value() && logits->defined()) {
    need(*logits, at::kFloat, "logits");
    TORCH_CHECK(logits->numel() >= B * N[nl - 1], "head: logits too small");
    a.logits = logits->data_ptr<float>();
  }
  need(labels, at::kInt, "labels");
  a.labels = labels.data_ptr<int>();
  a.nrows = labels.numel();
  if (idx.has_value() && idx->defined()) {
    need(*idx, at::kLong, "idx");
    TORCH_CHECK(idx->numel() >= B, "head: idx too small");
    a.idx = reinterpret_cast<const long long*>(idx->data_ptr());
  } else {
    TORCH_CHECK(labels.numel() >= B, "head: labels too small");
  }
  a.grad_scale = (float)grad_scale;
  need(loss_part, at::kFloat, "loss_part");
  TORCH_CHECK(loss_part.numel() >= 2 * ((B + 15) / 16), "head: loss_part must hold 2 floats per 16 rows");
  a.loss_part = loss_part.data_ptr<float>();
  need(stats, at::kFloat, "stats");
  TORCH_CHECK(stats.numel() >= 2, "head: stats must hold 2 floats");
  a.stats = stats.data_ptr<float>();
  TORCH_CHECK(phases == 2 || dfa::head_train_lds(a) <= 160 * 1024, "head: LDS footprint too large");
  a.dx_scale = (float)dx_scale;
  check_hip(dfa::head_train(a, (int)phases, cur_stream()), "head_train");
}

// The reference CNN's dense head (csrc/khead.hip): forward, softmax-CE and both data gradients in one
// launch; the weight gradients then come from head_train(phases=2) over (pT, h1T, dz1T, dz2T).
void khead_train_py(torch::Tensor p, torch::Tensor pT, c10::optional<torch::Tensor> dp, torch::Tensor w1,
                    torch::Tensor w1t, c10::optional<torch::Tensor> b1, torch::Tensor w2, torch::Tensor w2t,
                    c10::optional<torch::Tensor> b2, double drop_p, int64_t drop_seed,
                    c10::optional<torch::Tensor> drop_step, int64_t drop_step_add, double dh_scale, double dp_scale,
                    bool dp_mask, torch::Tensor h1T, torch::Tensor dz1T, torch::Tensor dz2T,
                    c10::optional<torch::Tensor> logits, torch::Tensor labels, c10::optional<torch::Tensor> idx,
                    double grad_scale, torch::Tensor loss_part, torch::Tensor ws) {
  need(p, at::kBFloat16, "p");
  TORCH_CHECK(p.dim() >= 2, "p must be [B, ...]");
  const int64_t B = p.size(0), K = p.numel() / std::max<int64_t>(B, 1);
  const int64_t ldt = (B + 31) / 32 * 32;
  const int64_t C = dz2T.size(0);
  TORCH_CHECK(dfa::khead_supported((int)K, (int)C), "khead: K must be a multiple of 256 (LDS-bounded), 1 <= C <= 16");
  const int N1 = dfa::kKHeadN1;
  dfa::KHeadArgs a{};
  a.B = (int)B;
  a.K = (int)K;
  a.C = (int)C;
  a.ldt = (int)ldt;
  a.p = reinterpret_cast<const dfa::bf16*>(p.data_ptr());
  need(pT, at::kBFloat16, "pT");
  TORCH_CHECK(pT.numel() >= K * ldt, "khead: pT must be [K][round32(B)]");
  a.pT = reinterpret_cast<dfa::bf16*>(pT.data_ptr());
  if (dp.has_value() && dp->defined()) {
    need(*dp, at::kBFloat16, "dp");
    TORCH_CHECK(dp->numel() >= B * K, "khead: dp too small");
    a.dp = reinterpret_cast<dfa::bf16*>(dp->data_ptr());
  }
  need(w1, at::kBFloat16, "w1");
  TORCH_CHECK(w1.dim() == 2 && w1.size(0) >= N1 && w1.size(1) >= K, "khead: w1 must be [128][>= K]");
  a.w1 = reinterpret_cast<const dfa::bf16*>(w1.data_ptr());
  a.ldw1 = (int)w1.size(1);
  need(w1t, at::kBFloat16, "w1t");
  TORCH_CHECK(w1t.dim() == 2 && w1t.size(0) >= K && w1t.size(1) == N1, "khead: w1t must be [>= K][128]");
  a.w1t = reinterpret_cast<const dfa::bf16*>(w1t.data_ptr());
  need(w2, at::kBFloat16, "w2");
  TORCH_CHECK(w2.dim() == 2 && w2.size(0) >= 16 && w2.size(1) == N1, "khead: w2 must be [16][128]");
  a.w2 = reinterpret_cast<const dfa::bf16*>(w2.data_ptr());
  need(w2t, at::kBFloat16, "w2t");
  TORCH_CHECK(w2t.dim() == 2 && w2t.size(0) >= N1 && w2t.size(1) == 32, "khead: w2t must be [128][32]");
  a.w2t = reinterpret_cast<const dfa::bf16*>(w2t.data_ptr());
  if (b1.has_value() && b1->defined()) {
    need(*b1, at::kFloat, "b1");
    TORCH_CHECK(b1->numel() >= N1, "khead: b1 too small");
    a.b1 = b1->data_ptr<float>();
  }
  if (b2.has_value() && b2->defined()) {
    need(*b2, at::kFloat, "b2");
    TORCH_CHECK(b2->numel() >= C, "khead: b2 too small");
    a.b2 = b2->data_ptr<float>();
  }
  a.drop = drop_from(drop_p, drop_seed, drop_step, drop_step_add);
  a.dh_scale = (float)dh_scale;
  a.dp_scale = (float)dp_scale;
  a.dp_mask = dp_mask ? 1 : 0;
  for (auto* t : {&h1T, &dz1T}) {
    need(*t, at::kBFloat16, "h1T/dz1T");
    TORCH_CHECK(t->numel() >= N1 * ldt, "khead: h1T / dz1T must be [128][round32(B)]");
  }
  need(dz2T, at::kBFloat16, "dz2T");
  TORCH_CHECK(dz2T.numel() >= C * ldt, "khead: dz2T must be [C][round32(B)]");
  a.h1T = reinterpret_cast<dfa::bf16*>(h1T.data_ptr());
  a.dz1T = reinterpret_cast<dfa::bf16*>(dz1T.data_ptr());
  a.dz2T = reinterpret_cast<dfa::bf16*>(dz2T.data_ptr());
  if (logits.has_value() && logits->defined()) {
    need(*logits, at::kFloat, "logits");
    TORCH_CHECK(logits->numel() >= B * C, "khead: logits too small");
    a.logits = logits->data_ptr<float>();
  }
  need(labels, at::kInt, "labels");
  a.labels = labels.data_ptr<int>();
  a.nrows = labels.numel();
  if (idx.has_value() && idx->defined()) {
    need(*idx, at::kLong, "idx");
    TORCH_CHECK(idx->numel() >= B, "khead: idx too small");
    a.idx = reinterpret_cast<const long long*>(idx->data_ptr());
  } else {
    TORCH_CHECK(labels.numel() >= B, "khead: labels too small");
  }
  a.grad_scale = (float)grad_scale;
  need(loss_part, at::kFloat, "loss_part");
  TORCH_CHECK(loss_part.numel() >= 2 * ((B + 15) / 16), "khead: loss_part must hold 2 floats per 16 rows");
  a.loss_part = loss_part.data_ptr<float>();
  need(ws, at::kFloat, "ws");
  TORCH_CHECK(ws.numel() >= (int64_t)dfa::khead_ws_floats((int)B, (int)K), "khead: workspace too small");
  const int64_t nt = (B + 31) / 32;
  float* base = ws.data_ptr<float>();
  a.slab = base;
  a.dz1 = reinterpret_cast<dfa::bf16*>(base + nt * dfa::kKHeadChunks * 32 * N1);
  a.sync = reinterpret_cast<unsigned*>(base + nt * dfa::kKHeadChunks * 32 * N1 + nt * 32 * N1 / 2);
  check_hip(dfa::khead_train(a, cur_stream()), "khead_train");
}

// Weight gradients of that head (csrc/khead.hip khead_wgrad_kernel) + the stats reduction: one launch.
void khead_wgrad_py(torch::Tensor pT, torch::Tensor h1T, torch::Tensor dz1T, torch::Tensor dz2T, torch::Tensor gw1,
                    c10::optional<torch::Tensor> gb1, torch::Tensor gw2, c10::optional<torch::Tensor> gb2, int64_t B,
                    int64_t K, int64_t C, torch::Tensor loss_part, torch::Tensor stats) {
  const int64_t ldt = (B + 31) / 32 * 32;
  const int N1 = dfa::kKHeadN1;
  for (auto* t : {&pT, &h1T, &dz1T, &dz2T}) need(*t, at::kBFloat16, "khead wgrad operand");
  TORCH_CHECK(pT.numel() >= K * ldt && h1T.numel() >= N1 * ldt && dz1T.numel() >= N1 * ldt &&
                  dz2T.numel() >= C * ldt, "khead_wgrad: operands must be [rows][round32(B)]");
  need(gw1, at::kFloat, "gw1");
  need(gw2, at::kFloat, "gw2");
  TORCH_CHECK(gw1.numel() >= N1 * K && gw2.numel() >= C * N1, "khead_wgrad: gradient buffers too small");
  dfa::KHeadWgradArgs a{};
  a.ldt = (int)ldt;
  a.L[0] = {reinterpret_cast<const dfa::bf16*>(dz1T.data_ptr()), reinterpret_cast<const dfa::bf16*>(pT.data_ptr()),
            gw1.data_ptr<float>(), nullptr, N1, (int)K, 0, 0};
  a.L[1] = {reinterpret_cast<const dfa::bf16*>(dz2T.data_ptr()), reinterpret_cast<const dfa::bf16*>(h1T.data_ptr()),
            gw2.data_ptr<float>(), nullptr, (int)C, N1, 0, 0};
  if (gb1.has_value() && gb1->defined()) {
    need(*gb1, at::kFloat, "gb1");
    a.L[0].gb = gb1->data_ptr<float>();
  }
  if (gb2.has_value() && gb2->defined()) {
    need(*gb2, at::kFloat, "gb2");
    a.L[1].gb = gb2->data_ptr<float>();
  }
  need(loss_part, at::kFloat, "loss_part");
  need(stats, at::kFloat, "stats");
  a.nloss = (int)((B + 15) / 16);
  TORCH_CHECK(loss_part.numel() >= 2 * a.nloss && stats.numel() >= 2, "khead_wgrad: loss_part / stats too small");
  a.loss_part = loss_part.data_ptr<float>();
  a.stats = stats.data_ptr<float>();
  check_hip(dfa::khead_wgrad(a, cur_stream()), "khead_wgrad");
}

class P2PComm;
static dfa::LLComm p2p_ll_args(const P2PComm& c);
class PSComm;
static dfa::PSArgs ps_lenet_args(const PSComm& c, const torch::Tensor& perm, const torch::Tensor& idx, double lr,
                                 int64_t max_stale);

// Whole-network LeNet-5 training step (csrc/lenet_fused.hip): fills the gradients of all ten
// parameters and stats = [loss sum, correct].  x: uint8 dataset [nrows][28][28][1] read through idx,
// or a bf16 batch [B][28][28][1].  With ``sgd_*`` the reduce launch applies the update; with ``ll``
// (a world > 1 P2PComm) it first sums every gradient over the ranks in-kernel (no all-reduce launch).
void lenet_train_py(torch::Tensor x, c10::optional<torch::Tensor> idx, double scale, torch::Tensor labels,
                    std::vector<torch::Tensor> conv, std::vector<torch::Tensor> dense_w,
                    std::vector<torch::Tensor> dense_wt, std::vector<torch::Tensor> dense_b,
                    std::vector<torch::Tensor> conv_grads, std::vector<torch::Tensor> dense_gw,
                    std::vector<torch::Tensor> dense_gb, std::vector<torch::Tensor> hT, std::vector<torch::Tensor> dzT,
                    torch::Tensor conv_part, torch::Tensor dense_part, torch::Tensor loss_part, torch::Tensor stats,
                    torch::Tensor frag, torch::Tensor ftab, torch::Tensor pxtab, int64_t B, double grad_scale,
                    bool prep, c10::optional<torch::Tensor> snap, std::vector<torch::Tensor> conv_mom,
                    c10::optional<torch::Tensor> sgd_master, c10::optional<torch::Tensor> sgd_mom,
                    c10::optional<torch::Tensor> sgd_wbf, c10::optional<torch::Tensor> sgd_hyper,
                    c10::optional<torch::Tensor> sgd_descs, c10::optional<torch::Tensor> idx_stream,
                    c10::optional<torch::Tensor> idx_cursor, c10::optional<torch::Tensor> idx_dst,
                    const P2PComm* ll, int64_t exch_blocks, c10::optional<torch::Tensor> run_stats,
                    const PSComm* ps, c10::optional<torch::Tensor> ps_perm, c10::optional<torch::Tensor> ps_idx,
                    double ps_lr, int64_t ps_max_stale, bool red_succ) {
  TORCH_CHECK(conv.size() == 4 && conv_grads.size() == 4, "lenet: conv = [w1, b1, w2, b2]");
  TORCH_CHECK(dense_w.size() == 3 && dense_wt.size() == 3 && dense_b.size() == 3 && dense_gw.size() == 3 &&
                  dense_gb.size() == 3 && hT.size() == 3 && dzT.size() == 3,
              "lenet: three dense layers");
  TORCH_CHECK(B > 0 && B < (1 << 30), "lenet: bad batch");
  dfa::LeNetArgs a{};
  const int64_t ldt = (B + 31) / 32 * 32;  // batch columns of H^T / dZ^T the reduce sums over
  // row stride of H^T / dZ^T: any multiple of 32 >= ldt (the trainer pads it off a power of two)
  const int64_t lds = hT.size() == 3 && hT[0].dim() == 2 ? hT[0].size(1) : 0;
  TORCH_CHECK(lds >= ldt && lds % 32 == 0, "lenet: hT rows must hold round32(B) columns, stride a multiple of 32");
  if (x.scalar_type() == at::kByte) {
    TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.numel() % 784 == 0, "lenet: uint8 dataset [N][28][28][1]");
    a.x_u8 = x.data_ptr<uint8_t>();
    a.nrows = x.numel() / 784;
    TORCH_CHECK((idx.has_value() && idx->defined()) || a.nrows >= B,
                "lenet: a uint8 dataset without batch indices must hold the batch (rows 0 .. B-1)");
  } else {
    need(x, at::kBFloat16, "lenet x");
    TORCH_CHECK(x.numel() == B * 784, "lenet: x must be [B][28][28][1]");
    a.x_bf = reinterpret_cast<const dfa::bf16*>(x.data_ptr());
    a.nrows = B;
  }
  if (idx.has_value() && idx->defined()) {
    need(*idx, at::kLong, "lenet idx");
    TORCH_CHECK(idx->numel() == B, "lenet: idx must have B entries");
    a.idx = reinterpret_cast<const long long*>(idx->data_ptr());
    if (a.x_u8 == nullptr) a.nrows = labels.numel();
  }
  need(labels, at::kInt, "lenet labels");
  TORCH_CHECK(labels.numel() >= (a.idx ? 1 : B), "lenet: labels too small");
  if (a.idx) a.nrows = std::min<int64_t>(a.nrows, labels.numel());
  a.labels = labels.data_ptr<int>();
  a.scale = (float)scale;
  const int64_t conv_n[4] = {150, 6, 2400, 16};
  for (int k = 0; k < 4; ++k) {
    need(conv[k], at::kFloat, "lenet conv param");
    need(conv_grads[k], at::kFloat, "lenet conv grad");
    TORCH_CHECK(conv[k].numel() == conv_n[k] && conv_grads[k].numel() == conv_n[k], "lenet: conv param size");
  }
  a.w1 = conv[0].data_ptr<float>();
  a.b1 = conv[1].data_ptr<float>();
  a.w2 = conv[2].data_ptr<float>();
  a.b2 = conv[3].data_ptr<float>();
  const int64_t wsz[3][2] = {{128, 416}, {96, 128}, {16, 96}}, wtsz[3][2] = {{400, 128}, {128, 96}, {96, 32}};
  const int64_t NK[3][2] = {{120, 400}, {84, 120}, {10, 84}};
  const dfa::bf16* dw[3];
  const dfa::bf16* dwt[3];
  const float* db[3];
  for (int l = 0; l < 3; ++l) {
    need(dense_w[l], at::kBFloat16, "lenet dense w");
    need(dense_wt[l], at::kBFloat16, "lenet dense wt");
    need(dense_b[l], at::kFloat, "lenet dense b");
    TORCH_CHECK(dense_w[l].dim() == 2 && dense_w[l].size(0) == wsz[l][0] && dense_w[l].size(1) == wsz[l][1],
                "lenet: dense ", l, " weights must be [", wsz[l][0], "][", wsz[l][1], "]");
    TORCH_CHECK(dense_wt[l].dim() == 2 && dense_wt[l].size(0) == wtsz[l][0] && dense_wt[l].size(1) == wtsz[l][1],
                "lenet: dense ", l, " dgrad weights must be [", wtsz[l][0], "][", wtsz[l][1], "]");
    TORCH_CHECK(dense_b[l].numel() == NK[l][0], "lenet: dense bias size");
    need(dense_gw[l], at::kFloat, "lenet dense gw");
    need(dense_gb[l], at::kFloat, "lenet dense gb");
    TORCH_CHECK(dense_gw[l].numel() == NK[l][0] * NK[l][1] && dense_gb[l].numel() == NK[l][0],
                "lenet: dense grad size");
    need(hT[l], at::kBFloat16, "lenet hT");
    need(dzT[l], at::kBFloat16, "lenet dzT");
    TORCH_CHECK(hT[l].dim() == 2 && hT[l].size(0) == NK[l][1] && hT[l].size(1) == lds, "lenet: hT shape");
    TORCH_CHECK(dzT[l].dim() == 2 && dzT[l].size(0) == NK[l][0] && dzT[l].size(1) == lds, "lenet: dzT shape");
    dw[l] = reinterpret_cast<const dfa::bf16*>(dense_w[l].data_ptr());
    dwt[l] = reinterpret_cast<const dfa::bf16*>(dense_wt[l].data_ptr());
    db[l] = dense_b[l].data_ptr<float>();
  }
  a.d1w = dw[0]; a.d2w = dw[1]; a.d3w = dw[2];
  a.d1wt = dwt[0]; a.d2wt = dwt[1]; a.d3wt = dwt[2];
  a.d1b = db[0]; a.d2b = db[1]; a.d3b = db[2];
  const int nblk = dfa::lenet_blocks((int)B);
  need(conv_part, at::kFloat, "lenet conv_part");
  need(loss_part, at::kFloat, "lenet loss_part");
  need(stats, at::kFloat, "lenet stats");
  TORCH_CHECK(conv_part.numel() >= (int64_t)dfa::kLeNetConvStride * nblk, "lenet: conv_part too small");
  TORCH_CHECK(loss_part.numel() >= 2 * nblk && stats.numel() >= 2, "lenet: loss buffers too small");
  a.conv_part = conv_part.data_ptr<float>();
  a.loss_part = loss_part.data_ptr<float>();
  auto bp = [](torch::Tensor& t) { return reinterpret_cast<dfa::bf16*>(t.data_ptr()); };
  a.h0T = bp(hT[0]); a.h1T = bp(hT[1]); a.h2T = bp(hT[2]);
  a.dz1T = bp(dzT[0]); a.dz2T = bp(dzT[1]); a.dz3T = bp(dzT[2]);
  TORCH_CHECK(frag.is_cuda() && frag.is_contiguous() && (size_t)frag.nbytes() >= dfa::lenet_frag_bytes(),
              "lenet: fragment buffer too small");
  TORCH_CHECK(ftab.is_cuda() && ftab.scalar_type() == at::kByte && ftab.numel() == 98 * 2 * 16, "lenet: ftab");
  TORCH_CHECK(pxtab.is_cuda() && pxtab.scalar_type() == at::kShort && pxtab.numel() == 832, "lenet: pxtab");
  a.frag = frag.data_ptr();
  a.prep = prep ? 1 : 0;
  a.ftab = ftab.data_ptr<uint8_t>();
  a.pxtab = reinterpret_cast<const unsigned short*>(pxtab.data_ptr());
  a.B = (int)B;
  a.ldt = (int)lds;
  a.grad_scale = (float)grad_scale;
  dfa::LeNetRedArgs r{};
  r.kcols = (int)ldt;
  // reduce scratch: job slabs, then the arrival tickets (zero-initialised by the trainer)
  need(dense_part, at::kFloat, "lenet dense_part");
  TORCH_CHECK(dense_part.numel() >= dfa::lenet_dense_part_floats((int)B),
              "lenet: dense_part must hold lenet_dense_part_floats(B) zero-initialised floats");
  dfa::lenet_red_bind_scratch(dense_part.data_ptr<float>(), r);
  r.succ = red_succ ? 1 : 0;  // (the launcher falls back to tickets where successor ownership cannot run)
  r.conv_part = a.conv_part;
  r.loss_part = a.loss_part;
  r.stats = stats.data_ptr<float>();
  r.g_w1 = conv_grads[0].data_ptr<float>();
  r.g_b1 = conv_grads[1].data_ptr<float>();
  r.g_w2 = conv_grads[2].data_ptr<float>();
  r.g_b2 = conv_grads[3].data_ptr<float>();
  for (int l = 0; l < 3; ++l) {
    r.L[l].dzT = reinterpret_cast<const dfa::bf16*>(dzT[l].data_ptr());
    r.L[l].hT = reinterpret_cast<const dfa::bf16*>(hT[l].data_ptr());
    r.L[l].gw = dense_gw[l].data_ptr<float>();
    r.L[l].gb = dense_gb[l].data_ptr<float>();
    r.L[l].N = (int)NK[l][0];
    r.L[l].K = (int)NK[l][1];
  }
  // optional pre-update snapshot of the conv kernels (weights, momentum) for the optimizer's fragment rebuild
  r.w1 = a.w1;
  r.w2 = a.w2;
  if (snap.has_value() && snap->defined()) {
    need(*snap, at::kFloat, "lenet snap");
    TORCH_CHECK(snap->numel() >= 2 * 2550, "lenet: snap must hold 2 x 2550 floats");
    r.snap = snap->data_ptr<float>();
    TORCH_CHECK(conv_mom.empty() || conv_mom.size() == 2, "lenet: conv_mom = [m1, m2] or []");
    if (conv_mom.size() == 2) {
      need(conv_mom[0], at::kFloat, "lenet m1");
      need(conv_mom[1], at::kFloat, "lenet m2");
      TORCH_CHECK(conv_mom[0].numel() == 150 && conv_mom[1].numel() == 2400, "lenet: conv momentum sizes");
      r.m1 = conv_mom[0].data_ptr<float>();
      r.m2 = conv_mom[1].data_ptr<float>();
    }
  }
  if (sgd_master.has_value() && sgd_master->defined()) {
    // single-rank fast path: the reduce kernel applies the SGD update (see LeNetSgd)
    need(*sgd_master, at::kFloat, "lenet sgd master");
    TORCH_CHECK(sgd_wbf.has_value() && sgd_hyper.has_value() && sgd_descs.has_value(),
                "lenet sgd: wbf, hyper and descs are required");
    need(*sgd_wbf, at::kBFloat16, "lenet sgd wbf");
    need(*sgd_hyper, at::kFloat, "lenet sgd hyper");
    TORCH_CHECK(sgd_hyper->numel() >= 5, "lenet sgd: hyper size");
    const torch::Tensor& dh = *sgd_descs;
    TORCH_CHECK(!dh.is_cuda() && dh.scalar_type() == at::kLong && dh.is_contiguous() &&
                    dh.numel() * 8 >= 10 * (int64_t)sizeof(dfa::ParamDesc),
                "lenet sgd: descs must be the host int64 table of the 10 parameters");
    r.sgd_on = 1;
    r.sgd.master = sgd_master->data_ptr<float>();
    r.sgd.mom = (sgd_mom.has_value() && sgd_mom->defined()) ? sgd_mom->data_ptr<float>() : nullptr;
    r.sgd.wbf = reinterpret_cast<dfa::bf16*>(sgd_wbf->data_ptr());
    r.sgd.hyper = sgd_hyper->data_ptr<float>();
    const auto* hd = reinterpret_cast<const dfa::ParamDesc*>(dh.data_ptr());
    for (int k = 0; k < 10; ++k) {
      r.sgd.d[k] = hd[k];
      TORCH_CHECK(hd[k].off >= 0 && hd[k].off + hd[k].numel <= sgd_master->numel(), "lenet sgd: descriptor range");
    }
    TORCH_CHECK(r.sgd.d[0].off == conv[0].data_ptr<float>() - r.sgd.master &&
                    r.sgd.d[2].off == conv[2].data_ptr<float>() - r.sgd.master,
                "lenet sgd: descriptors do not match the conv parameters");
    if (idx_stream.has_value() && idx_stream->defined()) {
      need(*idx_stream, at::kLong, "lenet idx_stream");
      TORCH_CHECK(idx_cursor.has_value() && idx_dst.has_value(), "lenet sgd: index stream needs cursor and dst");
      TORCH_CHECK(idx_stream->dim() == 2 && idx_stream->size(1) == idx_dst->numel(), "lenet sgd: stream shape");
      r.sgd.src = reinterpret_cast<const long long*>(idx_stream->data_ptr());
      r.sgd.cursor = reinterpret_cast<long long*>(idx_cursor->data_ptr());
      r.sgd.dst = reinterpret_cast<long long*>(idx_dst->data_ptr());
      r.sgd.B = (int)idx_dst->numel();
      r.sgd.nsteps = (int)idx_stream->size(0);
    }
    if (run_stats.has_value() && run_stats->defined()) {
      need(*run_stats, at::kFloat, "run_stats");
      TORCH_CHECK(run_stats->numel() >= 3, "run_stats must hold [loss sum, correct, updates]");
      r.sgd.run_stats = run_stats->data_ptr<float>();
    }
    r.sgd.frag = frag.data_ptr();
  }
  if (ll != nullptr) {
    TORCH_CHECK(r.sgd_on, "lenet: the in-kernel LL exchange needs the fused update (sgd_* arguments)");
    r.ll = p2p_ll_args(*ll);
    TORCH_CHECK(r.ll.world > 1, "lenet: LL exchange needs world > 1");
    r.ll_on = 1;
  }
  if (ps != nullptr) {
    TORCH_CHECK(r.sgd_on && !r.ll_on, "lenet: the parameter-server mode needs the fused update and no LL exchange");
    TORCH_CHECK(r.sgd.mom == nullptr, "lenet: the parameter server applies plain SGD (no momentum)");
    TORCH_CHECK(!(idx_stream.has_value() && idx_stream->defined()),
                "lenet: the parameter server stages the next microbatch itself (no index stream)");
    TORCH_CHECK(ps_perm.has_value() && ps_perm->defined() && ps_idx.has_value() && ps_idx->defined(),
                "lenet: the parameter-server mode needs the microbatch table and the index buffer");
    TORCH_CHECK(a.idx == reinterpret_cast<const long long*>(ps_idx->data_ptr()),
                "lenet: the parameter server must stage into the batch index buffer the step reads");
    r.ps = ps_lenet_args(*ps, *ps_perm, *ps_idx, ps_lr, ps_max_stale);
    r.ps_on = 1;
  }
  TORCH_CHECK(exch_blocks >= 0 && exch_blocks <= 512, "lenet: exch_blocks out of range");
  r.exch_blocks = (int)exch_blocks;
  check_hip(dfa::lenet_train(a, r, cur_stream()), "lenet_train");
}

// The reference CNN's conv block (csrc/kcnn_fused.hip).  x: uint8 dataset [nrows][28][28][1] (idx
// required), bf16 dataset rows (idx + scale), or a bf16 batch [B][28][28][1].
static dfa::KcnnArgs kcnn_args(torch::Tensor x, c10::optional<torch::Tensor> idx, double scale, int64_t B,
                               torch::Tensor w1, torch::Tensor b1, int64_t kpad1, torch::Tensor code) {
  dfa::KcnnArgs a{};
  TORCH_CHECK(B > 0 && B < (1 << 30), "kcnn: bad batch");
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.numel() % 784 == 0, "kcnn: x must be [.][28][28][1] on GPU");
  if (idx.has_value() && idx->defined()) {
    need(*idx, at::kLong, "kcnn idx");
    TORCH_CHECK(idx->numel() == B, "kcnn: idx must have B entries");
    a.idx = reinterpret_cast<const long long*>(idx->data_ptr());
  }
  if (x.scalar_type() == at::kByte) {
    TORCH_CHECK(a.idx, "kcnn: a uint8 dataset needs batch indices");
    a.x_u8 = x.data_ptr<uint8_t>();
  } else {
    TORCH_CHECK(x.scalar_type() == at::kBFloat16, "kcnn: x must be uint8 or bf16");
    a.x_bf = reinterpret_cast<const dfa::bf16*>(x.data_ptr());
    TORCH_CHECK(a.idx || x.numel() == B * 784, "kcnn: x must be [B][28][28][1]");
  }
  a.nrows = x.numel() / 784;
  a.scale = (float)scale;
  need(w1, at::kBFloat16, "kcnn w1");
  need(b1, at::kFloat, "kcnn b1");
  TORCH_CHECK(kpad1 >= 9 && w1.numel() >= 32 * kpad1 && b1.numel() == 32, "kcnn: conv1 weights [32][kpad1]");
  a.w1 = reinterpret_cast<const dfa::bf16*>(w1.data_ptr());
  a.b1 = b1.data_ptr<float>();
  a.kpad1 = (int)kpad1;
  TORCH_CHECK(code.is_cuda() && code.is_contiguous() && code.scalar_type() == at::kByte && code.numel() == B * 144 * 32,
              "kcnn: code must be uint8 [B][12][12][32]");
  a.code = code.data_ptr<uint8_t>();
  a.B = (int)B;
  return a;
}

void kcnn_fwd_py(torch::Tensor x, c10::optional<torch::Tensor> idx, double scale, int64_t B, torch::Tensor w1,
                 torch::Tensor b1, int64_t kpad1, torch::Tensor w2, torch::Tensor b2, torch::Tensor pooled,
                 torch::Tensor code, double drop_p, int64_t drop_seed, c10::optional<torch::Tensor> drop_step,
                 int64_t drop_step_add) {
  dfa::KcnnArgs a = kcnn_args(x, idx, scale, B, w1, b1, kpad1, code);
  need(w2, at::kBFloat16, "kcnn w2");
  need(b2, at::kFloat, "kcnn b2");
  need(pooled, at::kBFloat16, "kcnn pooled");
  TORCH_CHECK(w2.numel() >= 32 * 288 && b2.numel() == 32 && pooled.numel() == B * 144 * 32, "kcnn: conv2 / pooled");
  a.w2 = reinterpret_cast<const dfa::bf16*>(w2.data_ptr());
  a.b2 = b2.data_ptr<float>();
  a.pooled = reinterpret_cast<dfa::bf16*>(pooled.data_ptr());
  a.drop = drop_from(drop_p, drop_seed, drop_step, drop_step_add);
  check_hip(dfa::kcnn_fwd(a, cur_stream()), "kcnn_fwd");
}

void kcnn_bwd_py(torch::Tensor x, c10::optional<torch::Tensor> idx, double scale, int64_t B, torch::Tensor w1,
                 torch::Tensor b1, int64_t kpad1, torch::Tensor w2t, torch::Tensor dyp, torch::Tensor code,
                 torch::Tensor slabs, torch::Tensor g_w1, torch::Tensor g_b1, torch::Tensor g_w2, torch::Tensor g_b2,
                 c10::optional<torch::Tensor> step_inc) {
  dfa::KcnnArgs a = kcnn_args(x, idx, scale, B, w1, b1, kpad1, code);
  need(w2t, at::kBFloat16, "kcnn w2t");
  need(dyp, at::kBFloat16, "kcnn dyp");
  need(slabs, at::kFloat, "kcnn slabs");
  TORCH_CHECK(w2t.numel() >= 32 * 288 && dyp.numel() == B * 144 * 32, "kcnn: dgrad weights / pooled gradient");
  TORCH_CHECK((size_t)slabs.numel() >= dfa::kcnn_slab_floats((int)B), "kcnn: slab workspace too small");
  for (auto* t : {&g_w1, &g_b1, &g_w2, &g_b2}) need(*t, at::kFloat, "kcnn grad");
  TORCH_CHECK(g_w1.numel() == 288 && g_b1.numel() == 32 && g_w2.numel() == 32 * 288 && g_b2.numel() == 32,
              "kcnn: gradient sizes");
  a.w2t = reinterpret_cast<const dfa::bf16*>(w2t.data_ptr());
  a.dyp = reinterpret_cast<const dfa::bf16*>(dyp.data_ptr());
  a.slab2 = slabs.data_ptr<float>();
  a.slab1 = a.slab2 + (size_t)dfa::kcnn_blocks((int)B) * 32 * 289;
  long long* sp = nullptr;
  if (step_inc.has_value() && step_inc->defined()) {
    need(*step_inc, at::kLong, "kcnn step");
    sp = reinterpret_cast<long long*>(step_inc->data_ptr());
  }
  check_hip(dfa::kcnn_bwd(a, g_w1.data_ptr<float>(), g_b1.data_ptr<float>(), g_w2.data_ptr<float>(),
                          g_b2.data_ptr<float>(), sp, cur_stream()),
            "kcnn_bwd");
}

void classifier_metrics_py(torch::Tensor z, torch::Tensor labels, int64_t kind, int64_t out_act, torch::Tensor out) {
  need(z, at::kFloat, "metrics logits");
  need(labels, at::kInt, "metrics labels");
  need(out, at::kFloat, "metrics out");
  TORCH_CHECK(z.dim() == 2 && labels.numel() == z.size(0) && out.numel() >= 2, "metrics: z [B][C], labels [B]");
  check_hip(dfa::classifier_metrics(z.data_ptr<float>(), labels.data_ptr<int>(), (int)z.size(0), (int)z.size(1),
                                    (int)kind, (int)out_act, out.data_ptr<float>(), cur_stream()),
            "classifier_metrics");
}

bool convpool_supported_py(int64_t H, int64_t W, int64_t C, int64_t KH, int64_t KW, int64_t pad, int64_t N) {
  return dfa::convpool_supported(H, W, C, KH, KW, pad, N);
}

// A word of host-mapped, coherent pinned memory that kernels write with system-scope stores: the
// host watchdog (parallel/watchdog.py) polls it with a plain load, so a peer timeout seen on the
// device is noticed even while the GPU is busy or hung and without queueing any HIP call.
class HostFlag {
 public:
  HostFlag() {
    check_hip(hipHostMalloc((void**)&host_, 64, hipHostMallocMapped | hipHostMallocCoherent), "host flag alloc");
    memset(host_, 0, 64);
    check_hip(hipHostGetDevicePointer((void**)&dev_, host_, 0), "host flag device pointer");
  }
  ~HostFlag() {
    if (host_) (void)hipHostFree(host_);
  }
  HostFlag(const HostFlag&) = delete;
  HostFlag& operator=(const HostFlag&) = delete;
  int* device() const { return dev_; }
  int64_t read() const { return *reinterpret_cast<volatile int*>(host_); }

 private:
  int* host_ = nullptr;
  int* dev_ = nullptr;
};

// One-shot xGMI all-reduce communicator (csrc/allreduce_p2p.hip): owns this rank's IPC-exported
// flag+staging buffer and the peer mappings.  Handles are exchanged by the Python side over the
// process group (parallel/p2p.py); every launch goes onto PyTorch's current stream (graph capturable).
class P2PComm {
 public:
  P2PComm(int64_t rank, int64_t world, int64_t max_floats, double timeout_s, int64_t ll_slots)
      : rank_((int)rank), world_((int)world) {
    TORCH_CHECK(world >= 1 && world <= dfa::kP2PMaxRanks, "p2p: world must be in [1, 8]");
    TORCH_CHECK(rank >= 0 && rank < world, "p2p: bad rank");
    TORCH_CHECK(max_floats > 0 && max_floats <= (int64_t(1) << 28), "p2p: max_floats out of range");
    TORCH_CHECK(ll_slots >= 0 && ll_slots <= 4096, "p2p: ll_slots out of range");
    check_hip(hipGetDevice(&dev_), "p2p getDevice");
    max_blocks_ = (int)((max_floats + dfa::kP2PChunk - 1) / dfa::kP2PChunk);
    half_ = (int64_t)max_blocks_ * dfa::kP2PChunk;
    flag_bytes_ = ((int64_t)max_blocks_ * dfa::kP2PMaxRanks * 4 + 4095) / 4096 * 4096;
    // in-kernel LL exchange region (csrc/ll_exchange.h) after the staging halves, in the same IPC export
    ll_slots_ = (int)ll_slots;
    ll_off_ = flag_bytes_ + 2 * half_ * 4;
    bytes_ = ll_off_ + 2 * (int64_t)ll_slots_ * dfa::kP2PMaxRanks * dfa::kLLSlot * 8;
    void* p = nullptr;
    hipError_t e = hipExtMallocWithFlags(&p, (size_t)bytes_, hipDeviceMallocUncached);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      check_hip(hipExtMallocWithFlags(&p, (size_t)bytes_, hipDeviceMallocFinegrained), "p2p alloc");
    }
    local_ = (char*)p;
    check_hip(hipMemset(local_, 0, (size_t)bytes_), "p2p memset");
    // per-block counters, then per-slot LL counters, then per-(slot, part) LL counters
    const size_t nep = (size_t)max_blocks_ + (size_t)ll_slots_ * (1 + dfa::kLLParts);
    check_hip(hipMalloc((void**)&epochs_, nep * 4), "p2p epochs alloc");
    check_hip(hipMemset(epochs_, 0, nep * 4), "p2p epochs memset");
    check_hip(hipMalloc((void**)&err_, 4), "p2p err alloc");
    check_hip(hipMemset(err_, 0, 4), "p2p err memset");
    check_hip(hipDeviceSynchronize(), "p2p init sync");
    timeout_ticks_ = (int64_t)(timeout_s * 1e8);  // wall_clock64 runs at 100 MHz
    for (auto& b : bases_) b = nullptr;
    bases_[rank_] = local_;
  }
  ~P2PComm() {
    for (int r = 0; r < world_; ++r)
      if (r != rank_ && bases_[r]) (void)hipIpcCloseMemHandle(bases_[r]);
    if (local_) (void)hipFree(local_);
    if (epochs_) (void)hipFree(epochs_);
    if (err_) (void)hipFree(err_);
  }
  py::bytes handle() const {
    hipIpcMemHandle_t h;
    check_hip(hipIpcGetMemHandle(&h, local_), "hipIpcGetMemHandle");
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }
  void open(const std::vector<std::string>& handles) {
    TORCH_CHECK((int)handles.size() == world_, "p2p: need one handle per rank");
    for (int r = 0; r < world_; ++r) {
      if (r == rank_) continue;
      TORCH_CHECK(handles[r].size() == sizeof(hipIpcMemHandle_t), "p2p: bad handle size");
      hipIpcMemHandle_t h;
      memcpy(&h, handles[r].data(), sizeof(h));
      void* p = nullptr;
      check_hip(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
      bases_[r] = (char*)p;
    }
    opened_ = true;
  }
  void allreduce(torch::Tensor t, double scale) {
    need(t, at::kFloat, "p2p tensor");
    TORCH_CHECK(opened_ || world_ == 1, "p2p: open() the peer handles first");
    TORCH_CHECK(t.get_device() == dev_, "p2p: tensor on the wrong device");
    TORCH_CHECK(t.numel() <= half_, "p2p: tensor larger than the staging buffer");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "p2p: tensor must be 16-byte aligned");
    dfa::P2PArgs a{};
    for (int r = 0; r < dfa::kP2PMaxRanks; ++r) a.bases[r] = bases_[r];
    a.data = t.data_ptr<float>();
    a.n = t.numel();
    a.epochs = epochs_;
    a.err = err_;
    a.herr = herr_.device();
    a.flag_bytes = flag_bytes_;
    a.half_floats = half_;
    a.timeout_ticks = timeout_ticks_;
    a.rank = rank_;
    a.world = world_;
    a.max_blocks = max_blocks_;
    a.scale = (float)scale;
    check_hip(dfa::p2p_allreduce(a, cur_stream()), "p2p_allreduce");
  }
  int64_t error() const {
    int v = 0;
    check_hip(hipMemcpy(&v, err_, 4, hipMemcpyDeviceToHost), "p2p error readback");
    return v;
  }
  int64_t host_error() const { return herr_.read(); }  // no HIP call: safe from a watchdog thread
  // LL exchange self-test over the first in.numel() / kLLSlot slots (every rank the same call)
  void ll_selftest(torch::Tensor in, torch::Tensor out) {
    need(in, at::kFloat, "ll in");
    need(out, at::kFloat, "ll out");
    TORCH_CHECK(in.numel() == out.numel() && in.numel() % dfa::kLLSlot == 0, "ll: whole slots of kLLSlot floats");
    TORCH_CHECK(in.get_device() == dev_ && out.get_device() == dev_, "ll: tensors on the wrong device");
    const int ns = (int)(in.numel() / dfa::kLLSlot);
    TORCH_CHECK(ns >= 1 && ns <= ll_slots_, "ll: more slots than the communicator holds");
    check_hip(dfa::ll_selftest(ll_args(), in.data_ptr<float>(), out.data_ptr<float>(), ns, cur_stream()), "ll_selftest");
  }
  int64_t max_floats() const { return half_; }
  int64_t ll_slots() const { return ll_slots_; }
  void set_timeout(double timeout_s) { timeout_ticks_ = (int64_t)(timeout_s * 1e8); }
  // launch arguments of the in-kernel LL exchange (kernels that fold the all-reduce into their epilogue)
  dfa::LLComm ll_args() const {
    TORCH_CHECK(opened_ || world_ == 1, "p2p: open() the peer handles first");
    TORCH_CHECK(ll_slots_ > 0, "p2p: communicator built without LL slots");
    dfa::LLComm c{};
    for (int r = 0; r < dfa::kP2PMaxRanks; ++r)
      c.bases[r] = bases_[r] ? reinterpret_cast<unsigned long long*>(bases_[r] + ll_off_) : nullptr;
    c.epochs = epochs_ + max_blocks_;
    c.part_epochs = epochs_ + max_blocks_ + ll_slots_;
    c.err = err_;
    c.herr = herr_.device();
    c.timeout_ticks = timeout_ticks_;
    c.rank = rank_;
    c.world = world_;
    c.nslots = ll_slots_;
    return c;
  }

 private:
  int rank_, world_, dev_ = 0, max_blocks_ = 0, ll_slots_ = 0;
  int64_t half_ = 0, flag_bytes_ = 0, bytes_ = 0, timeout_ticks_ = 0, ll_off_ = 0;
  char* local_ = nullptr;
  char* bases_[dfa::kP2PMaxRanks];
  unsigned* epochs_ = nullptr;
  int* err_ = nullptr;
  HostFlag herr_;
  bool opened_ = false;
};

static dfa::LLComm p2p_ll_args(const P2PComm& c) { return c.ll_args(); }

// Device-resident async parameter server (csrc/async_ps.hip, csrc/ps_device.h).  The server rank owns
// the control buffer (version word, FCFS cursor, completion arrays); EVERY rank owns one shard of the fp32
// master (a contiguous, power-of-two-sized parameter range) in its own HBM.  Both kinds of buffer are
// uncached, IPC exported and mapped into every rank, so the applies of different ranks land on
// different shards in parallel over xGMI.  Each shard carries a 64-word self-test area after its range.
class PSComm {
 public:
  static constexpr int kTestWords = 64;
  // joiner: a worker outside the process group that attaches to a running server (late join, SURVEY §5.3
  // elastic membership): `rank` is its id (>= world, used as its drain-lock id), it owns no shard, no inbox
  // and no FedSGD slots, maps every member's, and never writes alone (no exclusive-writer shortcuts)
  // joinable (members): workers may attach later -- the buffers are uncached even at one rank and the
  // exclusive-writer shortcuts are off
  PSComm(int64_t rank, int64_t world, int64_t server_rank, int64_t n, double timeout_s, bool joiner, bool joinable)
      : rank_((int)rank), world_((int)world), server_((int)server_rank), n_(n), joiner_(joiner),
        joinable_(joinable || joiner) {
    TORCH_CHECK(n > 0 && n % 4 == 0, "ps: n must be a positive multiple of 4");
    TORCH_CHECK(world >= 1 && world <= dfa::kP2PMaxRanks, "ps: 1..8 ranks");
    TORCH_CHECK(server_rank >= 0 && server_rank < world, "ps: bad server rank");
    TORCH_CHECK(joiner ? (rank >= world && rank < 1024) : (rank >= 0 && rank < world), "ps: bad rank");
    check_hip(hipGetDevice(&dev_), "ps getDevice");
    // shard length: the smallest power of two >= 64 with world shards covering n
    shift_ = 6;
    while (((n_ - 1) >> shift_) >= world_) ++shift_;
    if (rank_ == server_) shared_ = alloc_shared(256 + 2 * (size_t)dfa::kPSMaxBatches * 4, "ps control");
    if (!joiner_) own_ = (float*)alloc_shared(((size_t)1 << shift_) * 4 + kTestWords * 4, "ps shard");
    check_hip(hipMalloc((void**)&local_, 4096), "ps local alloc");
    check_hip(hipMemset(local_, 0, 4096), "ps local memset");
    // kPSVMin (csrc/ps_device.h): no refresh recorded yet
    check_hip(hipMemset(local_ + 1024 + 4 * dfa::kPSVMinWord, 0xff, 4), "ps vmin init");
    check_hip(hipDeviceSynchronize(), "ps init sync");
    timeout_ticks_ = (int64_t)(timeout_s * 1e8);
    for (auto& p : shard_) p = nullptr;
  }
  ~PSComm() {
    for (int k = 0; k < world_; ++k)
      if (inbox_[k] && k != rank_) (void)hipIpcCloseMemHandle(inbox_[k]);
    if (inbox_own_) (void)hipFree(inbox_own_);
    for (int k = 0; k < world_; ++k)
      if (fed_slot_[k] && k != rank_) (void)hipIpcCloseMemHandle(fed_slot_[k]);
    if (fed_own_) (void)hipFree(fed_own_);
    if (shared_ && rank_ != server_) (void)hipIpcCloseMemHandle(shared_);
    if (shared_ && rank_ == server_) (void)hipFree(shared_);
    for (int k = 0; k < world_; ++k)
      if (shard_[k] && k != rank_) (void)hipIpcCloseMemHandle(shard_[k]);
    if (own_) (void)hipFree(own_);
    if (local_) (void)hipFree(local_);
  }
  py::bytes handle() const {
    TORCH_CHECK(rank_ == server_, "ps: only the server rank exports the control buffer");
    return export_handle(shared_);
  }
  py::bytes shard_handle() const {
    TORCH_CHECK(!joiner_, "ps: a joiner owns no shard");
    return export_handle(own_);
  }
  bool joiner() const { return joiner_; }
  // ctrl: the server's control-buffer handle; shards[k]: rank k's shard handle (every rank's, own included)
  void open(const std::string& ctrl, std::vector<std::string> shards) {
    TORCH_CHECK((int)shards.size() == world_, "ps: one shard handle per rank");
    if (rank_ != server_) shared_ = (char*)open_handle(ctrl);
    for (int k = 0; k < world_; ++k) shard_[k] = k == rank_ ? own_ : (float*)open_handle(shards[k]);
    std::vector<float*> tab(dfa::kP2PMaxRanks, nullptr);
    for (int k = 0; k < world_; ++k) tab[k] = shard_[k] + ((size_t)1 << shift_);  // self-test areas
    check_hip(hipMemcpy(local_ + 2048, tab.data(), tab.size() * sizeof(float*), hipMemcpyHostToDevice), "ps tab");
  }
  int64_t shard_len() const { return (int64_t)1 << shift_; }
  int64_t nshards_used() const { return (n_ - 1) / shard_len() + 1; }
  // every rank: seed its own shard's range of the master (the ranks hold identical initial weights)
  void init_master(torch::Tensor w) {
    TORCH_CHECK(!joiner_, "ps: a joiner seeds no shard (it pulls the current master)");
    need(w, at::kFloat, "ps master");
    TORCH_CHECK(w.numel() == n_, "ps: master size mismatch");
    const int64_t lo = (int64_t)rank_ * shard_len(), hi = std::min<int64_t>(n_, lo + shard_len());
    if (hi > lo)
      check_hip(hipMemcpy(own_, w.data_ptr<float>() + lo, (size_t)(hi - lo) * 4, hipMemcpyDeviceToDevice), "ps init");
    check_hip(hipDeviceSynchronize(), "ps init sync");
  }
  // self-test of the element add on every shard (call on every rank between two barriers): every rank
  // adds (rank + 1) * (j + 1) to word j of every shard's test area
  void selftest_add() {
    TORCH_CHECK(!joiner_, "ps: the shard self-test runs among the members");
    dfa::PSArgs a = args();
    check_hip(dfa::ps_selftest_add(a, reinterpret_cast<float* const*>(local_ + 2048), kTestWords, (float)(rank_ + 1),
                                   cur_stream()),
              "ps selftest");
    check_hip(hipStreamSynchronize(cur_stream()), "ps selftest sync");
  }
  // after every rank's selftest_add: each test word must hold (j + 1) * W (W + 1) / 2 exactly
  bool selftest_check() const {
    std::vector<float> v(kTestWords);
    for (int k = 0; k < world_; ++k) {
      check_hip(hipMemcpy(v.data(), shard_[k] + shard_len(), kTestWords * 4, hipMemcpyDeviceToHost), "ps selftest rd");
      for (int j = 0; j < kTestWords; ++j)
        if (v[j] != (float)((j + 1) * world_ * (world_ + 1) / 2)) return false;
    }
    return true;
  }
  int64_t host_error() const { return herr_.read(); }  // no HIP call: safe from a watchdog thread
  // Epoch-scoped at-least-once dispatch over `nbatches` microbatch ids, `max_epochs` dataset epochs
  // (0 = unbounded).  Called with the same values on every rank before the first step.
  void set_schedule(int64_t nbatches, int64_t max_epochs) {
    TORCH_CHECK(nbatches > 0 && nbatches <= dfa::kPSMaxBatches, "ps: nbatches out of range");
    TORCH_CHECK(max_epochs >= 0, "ps: max_epochs must be >= 0");
    nbatches_ = nbatches;
    max_epochs_ = (int)max_epochs;
  }
  // the device learning rate the applies read (the trainer's hyper tensor; set_lr after capture holds)
  void set_lr_source(torch::Tensor hyper) {
    need(hyper, at::kFloat, "ps lr source");
    TORCH_CHECK(hyper.numel() >= 1 && hyper.get_device() == dev_, "ps: lr source on this device");
    lr_dev_ = hyper.data_ptr<float>();
    lr_keep_ = hyper;
  }
  // [epoch, completed in epoch, completed, redispatched, skipped, duplicates, finished]
  std::vector<int64_t> schedule_stats() const {
    unsigned e[2] = {0, 0};
    unsigned long long c[4] = {0, 0, 0, 0};
    check_hip(hipMemcpy(e, shared_ + 32, 8, hipMemcpyDeviceToHost), "ps sched");
    check_hip(hipMemcpy(c, shared_ + 48, 32, hipMemcpyDeviceToHost), "ps sched ctr");
    const bool fin = max_epochs_ > 0 && (int64_t)e[0] >= max_epochs_;
    return {(int64_t)e[0], (int64_t)e[1], (int64_t)c[0], (int64_t)c[1], (int64_t)c[2], (int64_t)c[3], fin ? 1 : 0};
  }
  // done_epoch[0:nbatches]: e + 1 of the last epoch in which each batch was applied
  std::vector<int64_t> done_epochs() const {
    std::vector<unsigned> v((size_t)nbatches_);
    if (nbatches_ > 0)
      check_hip(hipMemcpy(v.data(), shared_ + 256, (size_t)nbatches_ * 4, hipMemcpyDeviceToHost), "ps done");
    return std::vector<int64_t>(v.begin(), v.end());
  }
  void fetch_pull(torch::Tensor w, c10::optional<torch::Tensor> perm, c10::optional<torch::Tensor> idx) {
    dfa::PSArgs a = args();
    need(w, at::kFloat, "ps local master");
    TORCH_CHECK(w.numel() == n_ && w.get_device() == dev_, "ps: local master mismatch");
    a.w = w.data_ptr<float>();
    if (perm.has_value() && perm->defined()) {
      need(*perm, at::kLong, "ps perm");
      TORCH_CHECK(idx.has_value() && idx->defined(), "ps: idx required with perm");
      need(*idx, at::kLong, "ps idx");
      TORCH_CHECK(perm->dim() == 2 && perm->size(1) == idx->numel(), "ps: perm must be [nbatches][B]");
      TORCH_CHECK(idx->numel() % 2 == 0, "ps: batch size must be even");
      TORCH_CHECK(nbatches_ == 0 || perm->size(0) == nbatches_, "ps: perm rows != scheduled nbatches");
      a.perm = reinterpret_cast<const long long*>(perm->data_ptr());
      a.idx = reinterpret_cast<long long*>(idx->data_ptr());
      a.nbatches = perm->size(0);
      a.B = (int)idx->numel();
    }
    check_hip(dfa::ps_fetch_pull(a, cur_stream()), "ps_fetch_pull");
  }
  // exclusive writer (world 1): admission + next claim / index staging, one workgroup; the update is the
  // optimizer launch gated on excl_gate() that mirrors the new weights into excl_mirror() (ps_excl_step)
  void excl_step(int64_t max_stale, c10::optional<torch::Tensor> perm, c10::optional<torch::Tensor> idx) {
    TORCH_CHECK(world_ == 1 && !owner_on_, "ps: the exclusive-writer step needs one rank (CAS path)");
    dfa::PSArgs a = args();
    a.max_stale = (int)max_stale;
    if (perm.has_value() && perm->defined()) {
      need(*perm, at::kLong, "ps perm");
      TORCH_CHECK(idx.has_value() && idx->defined(), "ps: idx required with perm");
      need(*idx, at::kLong, "ps idx");
      TORCH_CHECK(perm->dim() == 2 && perm->size(1) == idx->numel(), "ps: perm must be [nbatches][B]");
      TORCH_CHECK(idx->numel() % 2 == 0, "ps: batch size must be even");
      TORCH_CHECK(nbatches_ == 0 || perm->size(0) == nbatches_, "ps: perm rows != scheduled nbatches");
      a.perm = reinterpret_cast<const long long*>(perm->data_ptr());
      a.idx = reinterpret_cast<long long*>(idx->data_ptr());
      a.nbatches = perm->size(0);
      a.B = (int)idx->numel();
    }
    check_hip(dfa::ps_excl_step(a, cur_stream()), "ps_excl_step");
  }
  uintptr_t excl_gate() const {
    TORCH_CHECK(world_ == 1, "ps: one rank");
    return reinterpret_cast<uintptr_t>(reinterpret_cast<unsigned*>(local_ + 1024) + dfa::kPSDecisionWord);
  }
  uintptr_t excl_mirror() const {
    TORCH_CHECK(world_ == 1 && shard_[0] != nullptr, "ps: one rank, opened");
    return reinterpret_cast<uintptr_t>(shard_[0]);
  }
  void apply(torch::Tensor g, double lr, int64_t max_stale) {
    dfa::PSArgs a = args();
    need(g, at::kFloat, "ps grad");
    TORCH_CHECK(g.numel() == n_ && g.get_device() == dev_, "ps: gradient mismatch");
    a.g = g.data_ptr<float>();
    a.lr = (float)lr;
    a.max_stale = (int)max_stale;
    check_hip(dfa::ps_apply(a, cur_stream()), "ps_apply");
  }
  // device view of this rank's counters [accepted, rejected, sum staleness, max staleness, admission CAS
  // retries, err, no-op steps, -] (int64): read back asynchronously by the trainer's callbacks
  // audit rows (version at admission, vp, decision) of this rank's next `rows` decisions, written by the
  // admission itself (tests: the true staleness of every admitted gradient); an empty tensor disables it
  void set_audit(torch::Tensor rows) {
    if (!rows.defined() || rows.numel() == 0) {
      audit_ = nullptr, audit_cap_ = 0, audit_keep_ = torch::Tensor();
      return;
    }
    need(rows, at::kInt, "ps audit");
    TORCH_CHECK(rows.dim() == 2 && rows.size(1) == 3 && rows.get_device() == dev_, "ps: audit rows [n][3] int32");
    audit_ = reinterpret_cast<unsigned*>(rows.data_ptr<int>());
    audit_cap_ = rows.size(0);
    audit_keep_ = rows;
  }
  torch::Tensor stats_tensor() const {
    return torch::from_blob(local_ + 64, {8}, torch::TensorOptions().dtype(torch::kLong).device(torch::kCUDA, dev_));
  }
  // ---- device FedSGD count barrier (csrc/fedsgd_ps.hip) on the same shards: K gradient slots per shard
  // (every rank; call fed_init on every rank, exchange the handles, then fed_open)
  py::bytes fed_init(int64_t K) {
    TORCH_CHECK(K >= 1 && K <= dfa::kFedMaxK, "fedsgd: K must be 1..", dfa::kFedMaxK);
    TORCH_CHECK(fed_own_ == nullptr, "fedsgd: already initialised");
    fed_K_ = (int)K;
    fed_own_ = (float*)alloc_shared((size_t)K * ((size_t)1 << shift_) * 4, "fedsgd slots");
    for (auto& p : fed_slot_) p = nullptr;
    check_hip(hipMemset(local_ + 2560, 0, 1536), "fedsgd local");
    check_hip(hipDeviceSynchronize(), "fedsgd init sync");
    return export_handle(fed_own_);
  }
  void fed_open(std::vector<std::string> handles, int64_t K) {
    TORCH_CHECK((joiner_ || fed_own_ != nullptr) && (int)handles.size() == world_,
                "fedsgd: fed_init first (members), one handle per rank");
    if (joiner_) {
      TORCH_CHECK(K >= 1 && K <= dfa::kFedMaxK, "fedsgd: K must be 1..", dfa::kFedMaxK);
      fed_K_ = (int)K;
      check_hip(hipMemset(local_ + 2560, 0, 1536), "fedsgd local");
    }
    for (int k = 0; k < world_; ++k) fed_slot_[k] = k == rank_ ? fed_own_ : (float*)open_handle(handles[k]);
  }
  dfa::FedArgs fed_args() const {
    TORCH_CHECK((joiner_ || fed_own_ != nullptr) && fed_slot_[0] != nullptr, "fedsgd: fed_open first");
    dfa::FedArgs a{};
    a.seq = reinterpret_cast<unsigned*>(shared_ + 80);
    a.tick = reinterpret_cast<unsigned long long*>(shared_ + 88);
    a.land = reinterpret_cast<unsigned long long*>(shared_ + 96);
    a.bad = reinterpret_cast<unsigned long long*>(shared_ + 104);
    for (int k = 0; k < world_; ++k) a.shard[k] = shard_[k], a.slot[k] = fed_slot_[k];
    a.shard_shift = shift_;
    a.nshards = world_;
    a.K = fed_K_;
    a.n = n_;
    a.scratch = reinterpret_cast<unsigned*>(local_ + 2560);
    a.stats = reinterpret_cast<unsigned long long*>(local_ + 3584);
    a.audit = fed_audit_;
    a.audit_cap = fed_audit_cap_;
    a.lr_dev = lr_dev_;
    a.timeout_ticks = timeout_ticks_;
    a.herr = reinterpret_cast<unsigned*>(herr_.device());
    return a;
  }
  void fed_pull(torch::Tensor w) {
    need(w, at::kFloat, "fedsgd local master");
    TORCH_CHECK(w.numel() == n_ && w.get_device() == dev_, "fedsgd: local master mismatch");
    dfa::FedArgs a = fed_args();
    a.w = w.data_ptr<float>();
    check_hip(dfa::fed_pull(a, cur_stream()), "fed_pull");
  }
  // drop_land: fault injection (tests) -- the ticket is taken, nothing is stored or landed (a rank that dies
  // between its admission and its landing)
  void fed_upload(torch::Tensor g, bool drop_land) {
    need(g, at::kFloat, "fedsgd grad");
    TORCH_CHECK(g.numel() == n_ && g.get_device() == dev_, "fedsgd: gradient mismatch");
    dfa::FedArgs a = fed_args();
    a.g = g.data_ptr<float>();
    a.drop_land = drop_land ? 1 : 0;
    check_hip(dfa::fed_upload(a, cur_stream()), "fed_upload");
  }
  void fed_apply(double lr) {
    dfa::FedArgs a = fed_args();
    a.lr = (float)lr;
    check_hip(dfa::fed_apply(a, cur_stream()), "fed_apply");
  }
  void set_fed_audit(torch::Tensor rows) {
    if (!rows.defined() || rows.numel() == 0) {
      fed_audit_ = nullptr, fed_audit_cap_ = 0, fed_audit_keep_ = torch::Tensor();
      return;
    }
    need(rows, at::kInt, "fedsgd audit");
    TORCH_CHECK(rows.dim() == 2 && rows.size(1) == 3 && rows.get_device() == dev_, "fedsgd: audit rows [n][3] int32");
    fed_audit_ = reinterpret_cast<unsigned*>(rows.data_ptr<int>());
    fed_audit_cap_ = rows.size(0);
    fed_audit_keep_ = rows;
  }
  // [admitted, stale, full, failed, versions applied by this rank, error bits, version seqlock word,
  //  stuck versions this rank recovered]
  std::vector<int64_t> fed_stats() const {
    unsigned long long h[8] = {0};
    check_hip(hipMemcpy(h, local_ + 3584, 64, hipMemcpyDeviceToHost), "fedsgd stats");
    unsigned seq = 0;
    check_hip(hipMemcpy(&seq, shared_ + 80, 4, hipMemcpyDeviceToHost), "fedsgd seq");
    return {(int64_t)h[0], (int64_t)h[1], (int64_t)h[2], (int64_t)h[3], (int64_t)h[4], (int64_t)h[7], (int64_t)seq,
            (int64_t)h[5]};
  }
  // device view of [admitted, stale, full, failed, applied-by-me, -, -, err] (trainer callbacks)
  torch::Tensor fed_stats_tensor() const {
    return torch::from_blob(local_ + 3584, {8}, torch::TensorOptions().dtype(torch::kLong).device(torch::kCUDA, dev_));
  }
  // device view of the version seqlock word (int32; version = word / 2)
  torch::Tensor fed_seq_tensor() const {
    return torch::from_blob(shared_ + 80, {1}, torch::TensorOptions().dtype(torch::kInt).device(torch::kCUDA, dev_));
  }

  // ---- owner-applies (csrc/async_ps.hip): an inbox of `ring` slots of this rank's shard length (+ ring
  // flags) on every rank; call owner_init on every rank, exchange the handles, then owner_open
  py::bytes owner_init(int64_t ring) {
    TORCH_CHECK(ring >= 2 && ring <= 255, "ps owner-applies: ring must be 2..255");
    TORCH_CHECK(inbox_own_ == nullptr, "ps owner-applies: already initialised");
    owner_ring_ = (int)ring;
    inbox_own_ = (float*)alloc_shared((size_t)ring * ((size_t)1 << shift_) * 4 + (size_t)ring * 4 + 256,
                                        "ps owner inbox");
    return export_handle(inbox_own_);
  }
  // enable = false: map the inboxes only (the apply-path calibration), owner_enable() switches the path
  void owner_open(std::vector<std::string> handles, bool enable, int64_t ring) {
    TORCH_CHECK((joiner_ || inbox_own_ != nullptr) && (int)handles.size() == world_, "ps owner-applies: owner_init first");
    if (joiner_) {
      TORCH_CHECK(ring >= 2 && ring <= 255, "ps owner-applies: a joiner passes the members' ring length");
      owner_ring_ = (int)ring;
    }
    for (int k = 0; k < world_; ++k) inbox_[k] = k == rank_ ? inbox_own_ : (float*)open_handle(handles[k]);
    owner_on_ = enable;
  }
  void owner_enable(bool on) {
    TORCH_CHECK(!on || inbox_[0] != nullptr, "ps owner-applies: owner_open first");
    owner_on_ = on;
  }
  bool owner_applies() const { return owner_on_; }
  int64_t owner_ring() const { return owner_ring_; }
  // apply-path calibration (collective: every rank calls it at once, between barriers, before init_master):
  // mean microseconds per launch of the CAS adds (mode 0) or the owner-applies traffic (mode 1, needs
  // owner_init / owner_open) over this rank's n elements, `reps` launches after one warm-up launch
  double calibrate(int64_t mode, int64_t reps) {
    dfa::PSArgs a = args();
    TORCH_CHECK(mode == 0 || mode == 1, "ps calibrate: mode 0 (CAS) or 1 (owner-applies)");
    TORCH_CHECK(reps >= 1, "ps calibrate: reps >= 1");
    if (mode == 1) {
      TORCH_CHECK(inbox_[0] != nullptr, "ps calibrate: owner_open first");
      a.owner_ring = owner_ring_;
      a.pref = reinterpret_cast<unsigned*>(shared_ + 192);
      a.dlock = reinterpret_cast<unsigned*>(shared_ + 224);
      for (int k = 0; k < world_; ++k) a.inbox[k] = inbox_[k];
    }
    hipStream_t st = cur_stream();
    check_hip(dfa::ps_calibrate(a, (int)mode, st), "ps_calibrate");
    hipEvent_t e0, e1;
    check_hip(hipEventCreate(&e0), "calib event");
    check_hip(hipEventCreate(&e1), "calib event");
    check_hip(hipEventRecord(e0, st), "calib record");
    for (int64_t r = 0; r < reps; ++r) check_hip(dfa::ps_calibrate(a, (int)mode, st), "ps_calibrate");
    check_hip(hipEventRecord(e1, st), "calib record");
    check_hip(hipEventSynchronize(e1), "calib sync");
    float ms = 0.f;
    check_hip(hipEventElapsedTime(&ms, e0, e1), "calib elapsed");
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return (double)ms * 1e3 / (double)reps;
  }
  // the owner's drain alone (a pull into `w` without a microbatch claim): adds every flagged slot of this
  // rank's inbox into its shard; after the last step of every rank, one drain per rank settles the master
  void drain(torch::Tensor w) { fetch_pull(w, c10::nullopt, c10::nullopt); }
  // [drained sequence count of every owner]
  std::vector<int64_t> owner_prefix() const {
    std::vector<unsigned> v(world_, 0);
    check_hip(hipMemcpy(v.data(), shared_ + 192, (size_t)world_ * 4, hipMemcpyDeviceToHost), "ps pref");
    return std::vector<int64_t>(v.begin(), v.end());
  }

  // launch arguments of the fused LeNet-5 reduce in parameter-server mode (lenet_train_py)
  dfa::PSArgs lenet_args(const torch::Tensor& perm, const torch::Tensor& idx, double lr, int64_t max_stale) const {
    dfa::PSArgs a = args();
    need(perm, at::kLong, "ps perm");
    need(idx, at::kLong, "ps idx");
    TORCH_CHECK(perm.dim() == 2 && perm.size(1) == idx.numel() && idx.numel() % 2 == 0, "ps: perm [nbatches][B]");
    TORCH_CHECK(nbatches_ == 0 || perm.size(0) == nbatches_, "ps: perm rows != scheduled nbatches");
    a.perm = reinterpret_cast<const long long*>(perm.data_ptr());
    a.idx = reinterpret_cast<long long*>(idx.data_ptr());
    a.nbatches = perm.size(0);
    a.B = (int)idx.numel();
    a.lr = (float)lr;
    a.max_stale = (int)max_stale;
    return a;
  }
  // [accepted, rejected, sum staleness, max staleness, admission CAS retries, err, version, batch cursor,
  //  no-op steps, fully applied]
  std::vector<int64_t> stats() const {
    unsigned long long h[8] = {0};
    check_hip(hipMemcpy(h, local_ + 64, 64, hipMemcpyDeviceToHost), "ps stats");
    unsigned ver[3] = {0, 0, 0};
    unsigned long long ctr = 0;
    check_hip(hipMemcpy(ver, shared_, 12, hipMemcpyDeviceToHost), "ps ver");
    check_hip(hipMemcpy(&ctr, shared_ + 16, 8, hipMemcpyDeviceToHost), "ps ctr");
    return {(int64_t)h[0], (int64_t)h[1], (int64_t)h[2], (int64_t)h[3], (int64_t)h[4], (int64_t)h[5],
            (int64_t)ver[0], (int64_t)ctr, (int64_t)h[6], (int64_t)ver[2]};
  }
  // the master, gathered from the shards (call while no worker is stepping)
  void copy_master(torch::Tensor dst) const {
    need(dst, at::kFloat, "ps dst");
    TORCH_CHECK(dst.numel() == n_, "ps: dst size mismatch");
    check_hip(hipDeviceSynchronize(), "ps copy_master sync");
    for (int64_t k = 0; k < nshards_used(); ++k) {
      const int64_t lo = k * shard_len(), hi = std::min<int64_t>(n_, lo + shard_len());
      check_hip(hipMemcpyAsync(dst.data_ptr<float>() + lo, shard_[k], (size_t)(hi - lo) * 4, hipMemcpyDeviceToDevice,
                               cur_stream()),
                "ps copy_master");
    }
  }

 private:
  // Memory other processes map (world > 1): uncached, so every rank's access sees the others' without L2
  // maintenance.  One rank alone shares it with nobody: plain (cached) device memory, whose accesses do not
  // pay the uncached operation rate (~6 k per us chip-wide, profiles/r5/ps_cas_adds_per_us_1gpu.jsonl);
  // IPC export works on either.
  char* alloc_shared(size_t bytes, const char* what) const {
    if (world_ > 1 || joinable_) return alloc_uncached(bytes, what);
    void* p = nullptr;
    check_hip(hipMalloc(&p, bytes), what);
    check_hip(hipMemset(p, 0, bytes), what);
    return (char*)p;
  }
  static char* alloc_uncached(size_t bytes, const char* what) {
    void* p = nullptr;
    hipError_t e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      check_hip(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained), what);
    }
    check_hip(hipMemset(p, 0, bytes), what);
    return (char*)p;
  }
  static py::bytes export_handle(void* p) {
    hipIpcMemHandle_t h;
    check_hip(hipIpcGetMemHandle(&h, p), "hipIpcGetMemHandle");
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }
  static void* open_handle(const std::string& handle) {
    TORCH_CHECK(handle.size() == sizeof(hipIpcMemHandle_t), "ps: bad handle size");
    hipIpcMemHandle_t h;
    memcpy(&h, handle.data(), sizeof(h));
    void* p = nullptr;
    check_hip(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    return p;
  }
  dfa::PSArgs args() const {
    TORCH_CHECK(shared_ != nullptr && shard_[0] != nullptr, "ps: open() the handles first");
    dfa::PSArgs a{};
    a.ver = reinterpret_cast<unsigned*>(shared_);
    a.batch_ctr = reinterpret_cast<unsigned long long*>(shared_ + 16);
    for (int k = 0; k < world_; ++k) a.shard[k] = shard_[k];
    a.shard_shift = shift_;
    a.nshards = world_;
    a.excl = (world_ == 1 && !joinable_) ? 1 : 0;
    a.n = n_;
    a.vpulled = reinterpret_cast<unsigned*>(local_);
    a.applied = reinterpret_cast<unsigned*>(shared_ + 8);  // control buffer word 2 (ps_device.h)
    a.audit = audit_;
    a.audit_cap = audit_cap_;
    a.bid_out = reinterpret_cast<long long*>(local_ + 8);
    a.stats = reinterpret_cast<unsigned long long*>(local_ + 64);
    a.scratch = reinterpret_cast<unsigned*>(local_ + 1024);
    a.timeout_ticks = timeout_ticks_;
    a.max_stale = -1;
    a.lr_dev = lr_dev_;
    a.herr = reinterpret_cast<unsigned*>(herr_.device());
    a.rank = rank_;
    if (owner_on_) {
      a.owner_ring = owner_ring_;
      a.pref = reinterpret_cast<unsigned*>(shared_ + 192);   // control words 48..55 (async_ps.hip layout)
      a.dlock = reinterpret_cast<unsigned*>(shared_ + 224);  // control words 56..63
      for (int k = 0; k < world_; ++k) a.inbox[k] = inbox_[k];
    }
    if (nbatches_ > 0) {
      a.sched = reinterpret_cast<unsigned*>(shared_ + 32);
      a.sched_ctr = reinterpret_cast<unsigned long long*>(shared_ + 48);
      a.done_epoch = reinterpret_cast<unsigned*>(shared_ + 256);
      a.claimed_epoch = a.done_epoch + dfa::kPSMaxBatches;
      a.nbatches = nbatches_;
      a.max_epochs = max_epochs_;
    }
    return a;
  }
  HostFlag herr_;
  int rank_, world_, server_, dev_ = 0, shift_ = 6;
  bool joiner_ = false;
  bool joinable_ = false;  // other processes may attach: uncached buffers, no exclusive-writer shortcuts
  int max_epochs_ = 0;
  int64_t n_, timeout_ticks_ = 0, nbatches_ = 0;
  char* shared_ = nullptr;
  float* own_ = nullptr;
  float* shard_[dfa::kP2PMaxRanks];
  char* local_ = nullptr;
  float* lr_dev_ = nullptr;
  torch::Tensor lr_keep_;
  unsigned* audit_ = nullptr;
  int64_t audit_cap_ = 0;
  torch::Tensor audit_keep_;
  int owner_ring_ = 0;
  bool owner_on_ = false;
  float* inbox_own_ = nullptr;
  float* inbox_[dfa::kP2PMaxRanks] = {};
  int fed_K_ = 0;
  float* fed_own_ = nullptr;
  float* fed_slot_[dfa::kP2PMaxRanks] = {};
  unsigned* fed_audit_ = nullptr;
  int64_t fed_audit_cap_ = 0;
  torch::Tensor fed_audit_keep_;
};

static dfa::PSArgs ps_lenet_args(const PSComm& c, const torch::Tensor& perm, const torch::Tensor& idx, double lr,
                                 int64_t max_stale) {
  return c.lenet_args(perm, idx, lr, max_stale);
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "distriflow_amd native kernels (gfx950 / MI355X) and runtime";
  m.def("igemm_fwd", &igemm_fwd_py, "implicit-GEMM MFMA (dense/conv fwd, dgrad)", py::arg("src"), py::arg("w"),
        py::arg("bias"), py::arg("mask"), py::arg("out"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("Kpad"),
        py::arg("lda"), py::arg("ldc"), py::arg("geom"), py::arg("mode"), py::arg("relu"), py::arg("alpha"),
        py::arg("res") = py::none(), py::arg("resmask") = py::none(), py::arg("drop_p") = 0.0,
        py::arg("drop_seed") = 0, py::arg("drop_step") = py::none(), py::arg("pool_code") = py::none(),
        py::arg("drop_step_add") = 0, py::arg("bn_ws") = py::none(), py::arg("bn_ticket") = py::none(),
        py::arg("bn_mode") = 0, py::arg("bn_vecs") = std::vector<torch::Tensor>{}, py::arg("bn_x") = py::none(),
        py::arg("bn_momentum") = 0.1, py::arg("bn_eps") = 1e-5, py::arg("bn_gscale") = 1.0,
        py::arg("bacc") = py::none(), py::arg("bacc_mode") = 0, py::arg("bacc_in") = std::vector<torch::Tensor>{},
        py::arg("bacc2") = py::none(), py::arg("bacc2_in") = std::vector<torch::Tensor>{});
  m.def("igemm_bacc_supported", [](int64_t M, int64_t N, int64_t K, int64_t Kpad, std::vector<int64_t> geom,
                                   int64_t mode, int64_t bacc_mode, bool two, bool has_res, bool has_mask) {
    // the dispatch decision of igemm_fwd for a launch with these shapes (16-byte aligned operands)
    dfa::IGemmArgs a{};
    set_conv_geom(a, geom, (int)mode);
    a.M = (int)M; a.N = (int)N; a.K = (int)K; a.Kpad = (int)Kpad; a.ldc = (int)N; a.lda = 0;
    static dfa::bf16 dummy[8] __attribute__((aligned(16)));
    static double dacc[2] __attribute__((aligned(16)));
    static float dvec[2] __attribute__((aligned(16)));
    a.src = dummy; a.w = dummy; a.out = dummy;
    if (has_res) a.res = dummy;
    if (has_mask) a.mask = dummy;
    a.bacc.acc = dacc;
    a.bacc.nrep = 1;
    a.bacc.mode = (int)bacc_mode;
    if (bacc_mode == 1) a.bacc.x = dummy, a.bacc.mean = dvec, a.bacc.invstd = dvec;
    if (two) a.bacc.acc2 = dacc, a.bacc.x2 = dummy, a.bacc.mean2 = dvec, a.bacc.invstd2 = dvec;
    return dfa::igemm_bacc_ok(a, (int)mode);
  });
  m.def("igemm64_bn_tiles", [](int64_t M, int64_t N, int64_t K, int64_t Kpad, std::vector<int64_t> geom, int64_t mode) {
    dfa::IGemmArgs a{};
    set_conv_geom(a, geom, (int)mode);
    a.M = (int)M; a.N = (int)N; a.K = (int)K; a.Kpad = (int)Kpad; a.ldc = (int)N;
    static dfa::bf16 layout_dummy[8] __attribute__((aligned(16)));
    a.src = layout_dummy; a.w = layout_dummy; a.out = layout_dummy;
    int ntn = 0;
    const int ntm = dfa::igemm64_bn_layout(a, (int)mode, &ntn);
    return std::make_tuple((int64_t)ntm, (int64_t)ntn);
  });
  m.def("bn_finalize_partials", [](torch::Tensor part, int64_t ntm, int64_t C, int64_t M, torch::Tensor mean,
                                   torch::Tensor invstd, c10::optional<torch::Tensor> run_mean,
                                   c10::optional<torch::Tensor> run_var, double momentum, double eps) {
    need(part, at::kFloat, "bn part");
    need(mean, at::kFloat, "bn mean");
    need(invstd, at::kFloat, "bn invstd");
    TORCH_CHECK(part.numel() >= ntm * 2 * C && mean.numel() >= C && invstd.numel() >= C, "bn_finalize: sizes");
    check_hip(dfa::bn_finalize_partials(part.data_ptr<float>(), (int)ntm, (int)C, M, mean.data_ptr<float>(),
                                        invstd.data_ptr<float>(), const_cast<float*>(cptr<float>(run_mean)),
                                        const_cast<float*>(cptr<float>(run_var)),
                                        (float)momentum, (float)eps, cur_stream()),
              "bn_finalize_partials");
  });
  m.def("igemm64_pool_supported", [](int64_t H, int64_t W, int64_t C, int64_t OH, int64_t OW, int64_t K, int64_t N) {
    dfa::IGemmArgs a{};
    a.SH = (int)H; a.SW = (int)W; a.SC = (int)C; a.OH = (int)OH; a.OW = (int)OW; a.M = 4; a.N = (int)N; a.ldc = (int)N;
    a.K = (int)K; a.Kpad = (int)((K + 31) / 32 * 32);
    static dfa::bf16 layout_dummy[8] __attribute__((aligned(16)));
    static uint8_t codep[4] __attribute__((aligned(4)));
    a.src = layout_dummy; a.w = layout_dummy; a.out = layout_dummy; a.pool_code = codep;
    return dfa::igemm64_pool_supported(a) && N % 8 == 0;
  });
  m.def("unpool2", [](torch::Tensor dyp, torch::Tensor code, torch::Tensor dy) {
    need(dyp, at::kBFloat16, "unpool dyp");
    need(dy, at::kBFloat16, "unpool dy");
    TORCH_CHECK(dy.dim() == 4 && code.is_cuda() && code.is_contiguous() && code.scalar_type() == at::kByte,
                "unpool2: dy [B][OH][OW][N], code uint8");
    const int64_t B = dy.size(0), OH = dy.size(1), OW = dy.size(2), N = dy.size(3);
    TORCH_CHECK(dyp.numel() == B * (OH / 2) * (OW / 2) * N && code.numel() == dyp.numel(), "unpool2: sizes");
    check_hip(dfa::unpool2(reinterpret_cast<const dfa::bf16*>(dyp.data_ptr()), code.data_ptr<uint8_t>(),
                           reinterpret_cast<dfa::bf16*>(dy.data_ptr()), (int)B, (int)OH, (int)OW, (int)N,
                           cur_stream()),
              "unpool2");
  });
  m.def("igemm_wgrad", &igemm_wgrad_py, "implicit-GEMM MFMA weight gradient (split-m slabs + reduce)");
  m.def("maxpool_fwd", &maxpool_fwd_py, py::arg("x"), py::arg("y"), py::arg("B"), py::arg("H"), py::arg("W"),
        py::arg("C"), py::arg("P"), py::arg("drop_p") = 0.0, py::arg("drop_seed") = 0,
        py::arg("drop_step") = py::none(), py::arg("drop_step_add") = 0);
  m.def("maxpool_bwd", &maxpool_bwd_py);
  m.def("softmax_ce", &softmax_ce_py);
  m.def("dropout", &dropout_py);
  m.def("gather_batch", &gather_batch_py, py::arg("data"), py::arg("labels"), py::arg("idx"), py::arg("out"),
        py::arg("out_labels"), py::arg("B"), py::arg("row"), py::arg("scale"), py::arg("step_inc") = py::none());
  m.def("add_act", &add_act_py);
  m.def("merge_fwd", &merge_fwd_py, "Keras merge layer forward (Add / Subtract / Multiply / Average / Maximum / "
        "Minimum / Concatenate)");
  m.def("merge_bwd", &merge_bwd_py, "Keras merge layer: gradient of every input");
  m.def("relu_bwd", &relu_bwd_py);
  m.def("gap_fwd", &gap_fwd_py);
  m.def("gap_bwd", &gap_bwd_py);
  m.def("sgd_multi", &sgd_multi_py, py::arg("descs"), py::arg("ndesc"), py::arg("total_blocks"), py::arg("master"),
        py::arg("grad"), py::arg("mom"), py::arg("wbf"), py::arg("hyper"), py::arg("apply_update"),
        py::arg("idx_stream") = py::none(), py::arg("idx_cursor") = py::none(), py::arg("idx_dst") = py::none(),
        py::arg("descs_host") = py::none(), py::arg("lenet_frag") = py::none(), py::arg("frag_w1") = 0,
        py::arg("frag_w2") = 0, py::arg("lenet_snap") = py::none(), py::arg("step_stats") = py::none(),
        py::arg("run_stats") = py::none(), py::arg("gate") = 0, py::arg("mirror") = 0);
  m.def("sum_buffers", &sum_buffers_py);
  m.def("graph_upload", [](uintptr_t exec) {
    // stage an instantiated graph's kernel arguments / launch packets on the device now, outside any
    // timed region, instead of on its first hipGraphLaunch
    check_hip(hipGraphUpload(reinterpret_cast<hipGraphExec_t>(exec), cur_stream()), "hipGraphUpload");
  }, "hipGraphUpload of a captured graph (torch.cuda.CUDAGraph.raw_cuda_graph_exec()) on the current stream");
  m.def("axpby", &axpby_py);
  m.def("bn_stats_fwd", &bn_stats_fwd_py, "BN forward statistics (partials + last-workgroup finalize, one launch)");
  m.def("bn_stats_bwd", &bn_stats_bwd_py, "BN backward statistics: dgamma, dbeta and dx coefficients");
  m.def("bn_apply", &bn_apply_py, "BN normalize (+ residual join, + ReLU)");
  m.def("bn_dx", &bn_dx_py, "BN input gradient dx = k1*g + k2*x + k3");
  m.def("bn_apply_acc", &bn_apply_acc_py, "BN training apply, statistics finalised from epilogue-accumulated sums");
  m.def("bn_dx_acc", &bn_dx_acc_py, "BN input gradient, coefficients finalised from epilogue-accumulated sums");
  m.def("gap_bwd_bn", &gap_bwd_bn_py, "GAP backward with relu' and BatchNorm backward sums");
  m.def("bn_fwd_fused", &bn_fwd_fused_py, "BN training forward: statistics + apply in one launch");
  m.def("bn_bwd_fused", &bn_bwd_fused_py, "BN backward: statistics + dx in one launch");
  m.def("bn_stats_grid", &dfa::bn_stats_grid, "partial-slab count of a BN statistics launch");
  m.def("convpool_fwd", &convpool_fwd_py, "fused conv+bias+relu+maxpool2x2 (pooled map + argmax codes)");
  m.def("convpool_wgrad", &convpool_wgrad_py, "weight gradient through the fused conv+pool", py::arg("x"),
        py::arg("idx"), py::arg("scale"), py::arg("dp"), py::arg("code"), py::arg("gw"), py::arg("gb"), py::arg("ws"),
        py::arg("geom"), py::arg("defer") = false);
  m.def("slab_reduce_multi", &slab_reduce_multi_py, "several deferred split-m slab reductions in one launch");
  m.def("convpool_dgrad", &convpool_dgrad_py, "data gradient through the fused conv+pool");
  m.def("convpool_set_stamps", [](c10::optional<torch::Tensor> buf) {
    if (buf.has_value() && buf->defined()) {
      TORCH_CHECK(buf->is_cuda() && buf->scalar_type() == at::kLong && buf->numel() >= 4096 * 32,
                  "stamp buffer: int64 GPU tensor of >= 4096*32 elements");
      dfa::convpool_set_stamps(buf->data_ptr());
      dfa::head_set_stamps(buf->data_ptr());
      dfa::lenet_set_stamps(buf->data_ptr());
    } else {
      dfa::convpool_set_stamps(nullptr);
      dfa::head_set_stamps(nullptr);
      dfa::lenet_set_stamps(nullptr);
    }
  }, "profiling aid: per-block phase stamps of the convpool kernels");
  m.def("convpool_fwd_layout", [](int64_t H, int64_t W, int64_t C, int64_t KH, int64_t KW, int64_t pad, int64_t N) {
    int Cp = 0, Kpad2 = 0, pair = 0;
    dfa::convpool_fwd_layout(H, W, C, KH, KW, pad, N, &Cp, &Kpad2, &pair);
    return std::make_tuple(Cp, Kpad2, pair);
  }, "forward weight layout of the fused conv+pool kernel: (channel stride Cp, row length Kpad2, pair)");
  m.def("convpool_dgrad_layout", [](int64_t H, int64_t W, int64_t C, int64_t KH, int64_t KW, int64_t pad, int64_t N) {
    int pair = 0, K2pad = 0;
    dfa::convpool_dgrad_layout(H, W, C, KH, KW, pad, N, &pair, &K2pad);
    return std::make_tuple(pair, K2pad);
  }, "data-gradient weight layout of the fused conv+pool kernel: (pair, row length K2pad)");
  m.def("convpool_supported", &convpool_supported_py);
  m.def("head_train", &head_train_py, "fused dense head: forward + softmax-CE + backward (2 launches)",
        py::arg("w"), py::arg("wt"), py::arg("b"), py::arg("gw"), py::arg("gb"), py::arg("hT"), py::arg("dzT"),
        py::arg("K"), py::arg("N"), py::arg("x"), py::arg("x_relu"), py::arg("xT"), py::arg("dx"), py::arg("logits"),
        py::arg("labels"), py::arg("idx"), py::arg("grad_scale"), py::arg("loss_part"), py::arg("stats"),
        py::arg("phases"), py::arg("dx_scale") = 1.0);
  m.def("khead_train", &khead_train_py,
        "reference CNN dense head: forward + softmax-CE + both data gradients (1 launch, split-K)", py::arg("p"),
        py::arg("pT"), py::arg("dp"), py::arg("w1"), py::arg("w1t"), py::arg("b1"), py::arg("w2"), py::arg("w2t"),
        py::arg("b2"), py::arg("drop_p"), py::arg("drop_seed"), py::arg("drop_step"), py::arg("drop_step_add"),
        py::arg("dh_scale"), py::arg("dp_scale"), py::arg("dp_mask"),
        py::arg("h1T"), py::arg("dz1T"), py::arg("dz2T"), py::arg("logits"), py::arg("labels"), py::arg("idx"),
        py::arg("grad_scale"), py::arg("loss_part"), py::arg("ws"));
  m.def("khead_wgrad", &khead_wgrad_py, "reference CNN dense head: weight gradients + loss stats (1 launch)");
  m.def("khead_set_grid_cap", [](int64_t cus) { dfa::khead_set_grid_cap((int)cus); },
        "persistent dense-head grid cap (CUs) for ranks time-sharing one GPU; 0 = the whole chip");
  m.def("kcnn_set_stamps", [](c10::optional<torch::Tensor> buf) {
    dfa::kcnn_set_stamps(buf.has_value() && buf->defined() ? buf->data_ptr() : nullptr);
  }, "profiling aid: per-image phase clocks of the reference CNN's fused backward ([G][2][16] int64)");
  m.def("khead_set_stamps", [](c10::optional<torch::Tensor> buf) {
    dfa::khead_set_stamps(buf.has_value() && buf->defined() ? buf->data_ptr() : nullptr);
  }, "profiling aid: per-workgroup phase clocks of the khead launch into buf ([G][16] int64), None = off");
  m.def("khead_ws_floats", [](int64_t B, int64_t K) { return (int64_t)dfa::khead_ws_floats((int)B, (int)K); });
  m.def("khead_supported", [](int64_t K, int64_t C) { return dfa::khead_supported((int)K, (int)C); });
  m.def("kcnn_fwd", &kcnn_fwd_py,"reference CNN conv block forward (conv1 + conv2 + pool [+ dropout], 1 launch)",
        py::arg("x"), py::arg("idx"), py::arg("scale"), py::arg("B"), py::arg("w1"), py::arg("b1"), py::arg("kpad1"),
        py::arg("w2"), py::arg("b2"), py::arg("pooled"), py::arg("code"), py::arg("drop_p") = 0.0,
        py::arg("drop_seed") = 0, py::arg("drop_step") = py::none(), py::arg("drop_step_add") = 0);
  m.def("kcnn_bwd", &kcnn_bwd_py, "reference CNN conv block backward (both weight gradients, 2 launches)",
        py::arg("x"), py::arg("idx"), py::arg("scale"), py::arg("B"), py::arg("w1"), py::arg("b1"), py::arg("kpad1"),
        py::arg("w2t"), py::arg("dyp"), py::arg("code"), py::arg("slabs"), py::arg("g_w1"), py::arg("g_b1"),
        py::arg("g_w2"), py::arg("g_b2"), py::arg("step_inc") = py::none());
  m.def("kcnn_slab_floats", [](int64_t B) { return (int64_t)dfa::kcnn_slab_floats((int)B); });
  m.def("classifier_metrics", &classifier_metrics_py,
        "[loss sum, correct] of a classifier batch (one launch); out_act 0 logits, 1 softmax, 2 sigmoid output");
  m.def("act_fwd", &act_fwd_py, "standalone activation y = act(x) (csrc/act.hip)");
  m.def("act_bwd", &act_bwd_py, "dx = dy * act'(x) [* relu'(x)]");
  m.def("sigmoid_ce", &sigmoid_ce_py, "sigmoid cross-entropy on logits vs one-hot labels (+ dlogits)");
  m.def("pool2d_fwd", &pool2d_fwd_py, "general 2-D max / average pooling, any window / stride / padding");
  m.def("pool2d_bwd", &pool2d_bwd_py, "backward of pool2d_fwd (input-centric, no atomics)");
  m.def("lenet_train", &lenet_train_py, "whole-network LeNet-5 training step (fwd + CE + bwd, 2 launches)",
        py::arg("x"), py::arg("idx"), py::arg("scale"), py::arg("labels"), py::arg("conv"), py::arg("dense_w"),
        py::arg("dense_wt"), py::arg("dense_b"), py::arg("conv_grads"), py::arg("dense_gw"), py::arg("dense_gb"),
        py::arg("hT"), py::arg("dzT"), py::arg("conv_part"), py::arg("dense_part"), py::arg("loss_part"),
        py::arg("stats"), py::arg("frag"), py::arg("ftab"), py::arg("pxtab"), py::arg("B"), py::arg("grad_scale"),
        py::arg("prep") = true, py::arg("snap") = py::none(),
        py::arg("conv_mom") = std::vector<torch::Tensor>{}, py::arg("sgd_master") = py::none(),
        py::arg("sgd_mom") = py::none(), py::arg("sgd_wbf") = py::none(), py::arg("sgd_hyper") = py::none(),
        py::arg("sgd_descs") = py::none(), py::arg("idx_stream") = py::none(), py::arg("idx_cursor") = py::none(),
        py::arg("idx_dst") = py::none(), py::arg("ll") = nullptr, py::arg("exch_blocks") = 0, py::arg("run_stats") = py::none(),
        py::arg("ps") = nullptr, py::arg("ps_perm") = py::none(), py::arg("ps_idx") = py::none(),
        py::arg("ps_lr") = 0.0, py::arg("ps_max_stale") = -1, py::arg("red_succ") = true);
  m.def("lenet_blocks", [](int64_t B) { return dfa::lenet_blocks((int)B); });
  m.def("lenet_frag_bytes", []() { return (int64_t)dfa::lenet_frag_bytes(); });
  m.def("lenet_dense_part_floats", [](int64_t B) { return (int64_t)dfa::lenet_dense_part_floats((int)B); });
  m.def("lenet_red_err_offset", []() { return (int64_t)dfa::lenet_red_err_offset(); });
  m.def("gather_labels", &gather_labels_py);
  py::class_<P2PComm>(m, "P2PComm", "one-shot xGMI all-reduce over IPC-mapped peer buffers")
      .def(py::init<int64_t, int64_t, int64_t, double, int64_t>(), py::arg("rank"), py::arg("world"),
           py::arg("max_floats"), py::arg("timeout_s") = 2.0, py::arg("ll_slots") = 256)
      .def("handle", &P2PComm::handle)
      .def("open", &P2PComm::open)
      .def("allreduce", &P2PComm::allreduce, py::arg("t"), py::arg("scale") = 1.0)
      .def("error", &P2PComm::error)
      .def("host_error", &P2PComm::host_error)
      .def("ll_selftest", &P2PComm::ll_selftest, py::arg("inp"), py::arg("out"))
      .def("set_timeout", &P2PComm::set_timeout)
      .def_property_readonly("max_floats", &P2PComm::max_floats)
      .def_property_readonly("ll_slots", &P2PComm::ll_slots);
  py::class_<PSComm>(m, "PSComm", "device-resident bounded-staleness parameter server, master sharded over the ranks")
      .def(py::init<int64_t, int64_t, int64_t, int64_t, double, bool, bool>(), py::arg("rank"), py::arg("world"),
           py::arg("server_rank"), py::arg("n"), py::arg("timeout_s") = 30.0, py::arg("joiner") = false,
           py::arg("joinable") = false)
      .def("joiner", &PSComm::joiner)
      .def("handle", &PSComm::handle)
      .def("shard_handle", &PSComm::shard_handle)
      .def("open", &PSComm::open, py::arg("ctrl"), py::arg("shards"))
      .def("init_master", &PSComm::init_master)
      .def("selftest_add", &PSComm::selftest_add)
      .def("selftest_check", &PSComm::selftest_check)
      .def("set_lr_source", &PSComm::set_lr_source)
      .def_property_readonly("shard_len", &PSComm::shard_len)
      .def_property_readonly("nshards_used", &PSComm::nshards_used)
      .def("excl_step", &PSComm::excl_step, py::arg("max_stale"), py::arg("perm") = py::none(),
           py::arg("idx") = py::none())
      .def("excl_gate", &PSComm::excl_gate)
      .def("excl_mirror", &PSComm::excl_mirror)
      .def("fetch_pull", &PSComm::fetch_pull, py::arg("w"), py::arg("perm") = py::none(), py::arg("idx") = py::none())
      .def("apply", &PSComm::apply, py::arg("g"), py::arg("lr"), py::arg("max_stale"))
      .def("stats", &PSComm::stats)
      .def("host_error", &PSComm::host_error)
      .def("set_schedule", &PSComm::set_schedule, py::arg("nbatches"), py::arg("max_epochs") = 0)
      .def("schedule_stats", &PSComm::schedule_stats)
      .def("done_epochs", &PSComm::done_epochs)
      .def("copy_master", &PSComm::copy_master)
      .def("stats_tensor", &PSComm::stats_tensor)
      .def("set_audit", &PSComm::set_audit, py::arg("rows"))
      .def("owner_init", &PSComm::owner_init, py::arg("ring"))
      .def("owner_open", &PSComm::owner_open, py::arg("handles"), py::arg("enable") = true, py::arg("ring") = 0)
      .def("owner_enable", &PSComm::owner_enable, py::arg("on"))
      .def("owner_applies", &PSComm::owner_applies)
      .def("owner_ring", &PSComm::owner_ring)
      .def("drain", &PSComm::drain)
      .def("owner_prefix", &PSComm::owner_prefix)
      .def("calibrate", &PSComm::calibrate, py::arg("mode"), py::arg("reps") = 20)
      .def("fed_init", &PSComm::fed_init, py::arg("K"))
      .def("fed_open", &PSComm::fed_open, py::arg("handles"), py::arg("K") = 0)
      .def("fed_pull", &PSComm::fed_pull)
      .def("fed_upload", &PSComm::fed_upload, py::arg("g"), py::arg("drop_land") = false)
      .def("fed_apply", &PSComm::fed_apply, py::arg("lr"))
      .def("set_fed_audit", &PSComm::set_fed_audit, py::arg("rows"))
      .def("fed_stats", &PSComm::fed_stats)
      .def("fed_stats_tensor", &PSComm::fed_stats_tensor)
      .def("fed_seq_tensor", &PSComm::fed_seq_tensor);
  dfa::register_runtime(m);
}
