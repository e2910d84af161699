// PyTorch custom-op bindings (TORCH_LIBRARY "dlion") for the gfx950 kernels.
// Every op launches on the caller's current HIP stream, takes pre-built device
// metadata (no host sync, no allocation: safe to capture in a hipGraph) and
// refuses CPU tensors loudly -- there is deliberately no silent fallback here;
// the pure-PyTorch oracle lives in ops/reference.py and is chosen explicitly.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>
#include <vector>

#include "kernels.h"

namespace dlion {
enum class Layout : int { NT = 0, NN = 1, TN = 2, TT = 3 };
bool lt_gemm(const void* a, int64_t lda, const void* b, int64_t ldb, void* c, int64_t ldc, const void* bias,
             int64_t M, int64_t N, int64_t K, int epi, int device, hipStream_t s, Layout lay, bool accumulate);
}

namespace {

using at::Tensor;

void check_dev(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "dlion: ", name, " must be a GPU (HIP) tensor");
  TORCH_CHECK(t.is_contiguous(), "dlion: ", name, " must be contiguous");
}

void check_hip(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "dlion: ", what, " failed: ", hipGetErrorString(e));
}

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

const float* gscale_ptr(const std::optional<Tensor>& gscale) {
  if (!gscale.has_value()) return nullptr;
  check_dev(*gscale, "gscale");
  TORCH_CHECK(gscale->scalar_type() == at::kFloat && gscale->numel() >= 2, "dlion: gscale must be float32[2]");
  return gscale->data_ptr<float>();
}

void lion_local(const Tensor& meta, int64_t seg_off, int64_t chunk_off, int64_t n_chunks, int64_t dtype,
                double decay, double neg_lr, double b1, double omb1, double b2, double omb2,
                const std::optional<Tensor>& gscale) {
  check_dev(meta, "meta");
  TORCH_CHECK(meta.scalar_type() == at::kLong, "dlion: meta must be int64");
  const c10::DeviceGuard g(meta.device());
  const int64_t* base = meta.data_ptr<int64_t>();
  check_hip(dlion::launch_lion_local(static_cast<int>(dtype), base + seg_off, base + chunk_off, n_chunks,
                                     static_cast<float>(decay), static_cast<float>(neg_lr), static_cast<float>(b1),
                                     static_cast<float>(omb1), static_cast<float>(b2), static_cast<float>(omb2),
                                     gscale_ptr(gscale), cur_stream()),
            "lion_local");
}

void lion_encode(const Tensor& meta, int64_t seg_off, int64_t chunk_off, int64_t n_chunks, int64_t dtype,
                 const Tensor& bits, double b1, double omb1, double b2, double omb2, bool update_m,
                 bool stochastic, double rr, int64_t seed, int64_t step, const std::optional<Tensor>& gscale) {
  check_dev(meta, "meta");
  check_dev(bits, "bits");
  TORCH_CHECK(bits.scalar_type() == at::kByte, "dlion: bits must be uint8");
  const c10::DeviceGuard g(meta.device());
  const int64_t* base = meta.data_ptr<int64_t>();
  check_hip(dlion::launch_lion_encode(static_cast<int>(dtype), base + seg_off, base + chunk_off, n_chunks,
                                      bits.data_ptr<uint8_t>(), static_cast<float>(b1), static_cast<float>(omb1),
                                      static_cast<float>(b2), static_cast<float>(omb2), update_m ? 1 : 0,
                                      stochastic ? 1 : 0, static_cast<float>(rr), static_cast<uint64_t>(seed),
                                      static_cast<uint32_t>(step), gscale_ptr(gscale), cur_stream()),
            "lion_encode");
}

// partial[chunk_base + i] = sum of g^2 over chunk i of the bucket
void grad_sumsq(const Tensor& meta, int64_t seg_off, int64_t chunk_off, int64_t n_chunks, int64_t dtype,
                const Tensor& partial, int64_t part_off) {
  check_dev(meta, "meta");
  check_dev(partial, "partial");
  TORCH_CHECK(partial.scalar_type() == at::kFloat && part_off + n_chunks <= partial.numel(),
              "dlion: grad_sumsq partial buffer too small");
  const c10::DeviceGuard g(meta.device());
  const int64_t* base = meta.data_ptr<int64_t>();
  check_hip(dlion::launch_grad_sumsq(static_cast<int>(dtype), base + seg_off, base + chunk_off, n_chunks,
                                     partial.data_ptr<float>() + part_off, cur_stream()),
            "grad_sumsq");
}

// out[0] = sqrt(sum partial), out[1] = min(1, max_norm / (out[0] + 1e-6))
void clip_coef(const Tensor& partial, int64_t n, double max_norm, const Tensor& out) {
  check_dev(partial, "partial");
  check_dev(out, "out");
  TORCH_CHECK(partial.scalar_type() == at::kFloat && out.scalar_type() == at::kFloat && out.numel() >= 2 &&
                  n <= partial.numel(),
              "dlion: clip_coef needs float32 partials and a float32[2] output");
  const c10::DeviceGuard g(partial.device());
  check_hip(dlion::launch_clip_coef(partial.data_ptr<float>(), n, static_cast<float>(max_norm), out.data_ptr<float>(),
                                    cur_stream()),
            "clip_coef");
}

void lion_vote_apply(const Tensor& meta, int64_t seg_off, int64_t chunk_off, int64_t n_chunks, int64_t dtype,
                     const Tensor& planes, int64_t plane_stride, const Tensor& alive, int64_t mode, int64_t tie,
                     const std::optional<Tensor>& neg, double decay, double neg_lr,
                     const std::optional<Tensor>& own, const std::optional<Tensor>& agree) {
  check_dev(meta, "meta");
  check_dev(planes, "planes");
  check_dev(alive, "alive");
  TORCH_CHECK(planes.scalar_type() == at::kByte, "dlion: planes must be uint8");
  TORCH_CHECK(alive.scalar_type() == at::kByte, "dlion: alive must be uint8");
  TORCH_CHECK(mode >= 0 && mode <= 2, "dlion: bad vote mode ", mode);
  const uint8_t* negp = nullptr;
  if (neg.has_value()) {
    check_dev(*neg, "neg");
    negp = neg->data_ptr<uint8_t>();
  }
  unsigned long long* agp = nullptr;
  const uint8_t* ownp = nullptr;
  if (agree.has_value()) {
    TORCH_CHECK(own.has_value(), "dlion: vote agreement needs this rank's own bits");
    check_dev(*own, "own");
    ownp = own->data_ptr<uint8_t>();
    check_dev(*agree, "agree");
    TORCH_CHECK(agree->scalar_type() == at::kLong && agree->numel() >= 2,
                "dlion: agree must be int64 [agreements, ties]");
    agp = reinterpret_cast<unsigned long long*>(agree->data_ptr<int64_t>());
  }
  const c10::DeviceGuard g(meta.device());
  const int64_t* base = meta.data_ptr<int64_t>();
  check_hip(dlion::launch_lion_vote_apply(static_cast<int>(dtype), base + seg_off, base + chunk_off, n_chunks,
                                          planes.data_ptr<uint8_t>(), plane_stride, alive.data_ptr<uint8_t>(),
                                          static_cast<int>(alive.numel()), static_cast<int>(mode),
                                          static_cast<int>(tie), negp, static_cast<float>(decay),
                                          static_cast<float>(neg_lr), ownp, agp,
                                          cur_stream()),
            "lion_vote_apply");
}

void vote_reduce(const Tensor& recv, int64_t nbytes, const Tensor& alive, int64_t tie, const Tensor& out,
                 const std::optional<Tensor>& neg_out, const std::optional<Tensor>& ties) {
  check_dev(recv, "recv");
  check_dev(alive, "alive");
  check_dev(out, "out");
  TORCH_CHECK(nbytes % 4 == 0, "dlion: vote_reduce shard bytes must be a multiple of 4");
  TORCH_CHECK(out.numel() >= nbytes, "dlion: vote_reduce out too small");
  TORCH_CHECK(recv.numel() >= nbytes * alive.numel(), "dlion: vote_reduce recv too small");
  uint8_t* negp = nullptr;
  if (neg_out.has_value()) {
    check_dev(*neg_out, "neg_out");
    negp = neg_out->data_ptr<uint8_t>();
  }
  unsigned long long* tp = nullptr;
  if (ties.has_value()) {
    check_dev(*ties, "ties");
    TORCH_CHECK(ties->scalar_type() == at::kLong && ties->numel() >= 1, "dlion: ties must be int64");
    tp = reinterpret_cast<unsigned long long*>(ties->data_ptr<int64_t>());
  }
  const c10::DeviceGuard g(recv.device());
  check_hip(dlion::launch_vote_reduce(recv.data_ptr<uint8_t>(), nbytes, alive.data_ptr<uint8_t>(),
                                      static_cast<int>(alive.numel()), static_cast<int>(tie),
                                      out.data_ptr<uint8_t>(), negp, tp, cur_stream()),
            "vote_reduce");
}

int dtype_code(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kHalf: return 2;
    default: TORCH_CHECK(false, "dlion: unsupported dtype ", t);
  }
  return -1;
}

// variant: 0 auto, 1 register-resident fp32 row, 2 streaming, 3/4/5 packed 16-bit row with 256/512/1024 threads
Tensor softmax_xent_(const Tensor& logits, const Tensor& labels, int64_t v, int64_t variant) {
  check_dev(logits, "logits");
  check_dev(labels, "labels");
  TORCH_CHECK(logits.dim() == 2, "dlion: logits must be [N, Vpad]");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == logits.size(0), "dlion: labels must be int64[N]");
  TORCH_CHECK(logits.size(1) % 8 == 0 && v <= logits.size(1), "dlion: padded vocab must be a multiple of 8");
  const c10::DeviceGuard g(logits.device());
  auto loss = at::empty({logits.size(0)}, logits.options().dtype(at::kFloat));
  check_hip(dlion::launch_softmax_xent(dtype_code(logits.scalar_type()), logits.data_ptr(), labels.data_ptr<int64_t>(),
                                       logits.size(0), logits.size(1), static_cast<int>(v), loss.data_ptr<float>(),
                                       static_cast<int>(variant), cur_stream()),
            "softmax_xent");
  return loss;
}

// ------------------------------------------------------------ flash attention
void check_bthd(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16, "dlion attn: ", name, " must be a bf16 GPU tensor");
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1, "dlion attn: ", name, " must be [B,T,H,D] with contiguous D");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0 &&
                  t.stride(0) % 8 == 0,
              "dlion attn: ", name, " must be 16-byte aligned");
}

dlion::AttnArgs attn_args(const Tensor& q, const Tensor& k, const Tensor& v, double p, int64_t seed) {
  check_bthd(q, "q");
  check_bthd(k, "k");
  check_bthd(v, "v");
  const int64_t B = q.size(0), T = q.size(1), H = q.size(2), D = q.size(3), Hkv = k.size(2);
  TORCH_CHECK(k.size(0) == B && k.size(1) == T && k.size(3) == D && v.sizes() == k.sizes(), "dlion attn: shape mismatch");
  TORCH_CHECK(H % Hkv == 0, "dlion attn: H must be a multiple of Hkv");
  TORCH_CHECK(T >= 1 && (D == 64 || D == 128), "dlion attn: need T >= 1 and D in {64, 128}");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dlion attn: dropout must be in [0, 1)");
  dlion::AttnArgs a{};
  a.q = static_cast<const __bf16*>(q.data_ptr());
  a.k = static_cast<const __bf16*>(k.data_ptr());
  a.v = static_cast<const __bf16*>(v.data_ptr());
  a.q_sb = q.stride(0); a.q_st = q.stride(1); a.q_sh = q.stride(2);
  a.k_sb = k.stride(0); a.k_st = k.stride(1); a.k_sh = k.stride(2);
  a.v_sb = v.stride(0); a.v_st = v.stride(1); a.v_sh = v.stride(2);
  a.B = static_cast<int>(B); a.T = static_cast<int>(T); a.H = static_cast<int>(H); a.Hkv = static_cast<int>(Hkv);
  a.scale = static_cast<float>(1.0 / std::sqrt(static_cast<double>(D)));
  a.scale_log2 = static_cast<float>(1.4426950408889634 / std::sqrt(static_cast<double>(D)));
  uint32_t th = static_cast<uint32_t>(std::llround(p * 65536.0));
  if (th > 65535u) th = 65535u;
  a.thresh16 = th;
  a.inv_keep = static_cast<float>(65536.0 / (65536.0 - th));
  a.seed = static_cast<uint32_t>(seed);
  return a;
}

void set_window(dlion::AttnArgs& a, int64_t window, int64_t D) {
  TORCH_CHECK(window >= 0, "dlion attn: window must be >= 0 (0 = plain causal)");
  a.window = window >= a.T ? 0 : static_cast<int>(window);  // a window covering T is plain causal
  TORCH_CHECK(a.window == 0 || D == 128, "dlion attn: a sliding window needs head_dim 128");
}

std::tuple<Tensor, Tensor> attn_fwd(const Tensor& q, const Tensor& k, const Tensor& v, double p, int64_t seed,
                                    int64_t window) {
  auto a = attn_args(q, k, v, p, seed);
  set_window(a, window, q.size(3));
  const c10::DeviceGuard g(q.device());
  auto out = at::empty({q.size(0), q.size(1), q.size(2), q.size(3)}, q.options());
  auto lse = at::empty({q.size(0), q.size(2), q.size(1)}, q.options().dtype(at::kFloat));
  a.out = static_cast<__bf16*>(out.data_ptr());
  a.o_sb = out.stride(0); a.o_st = out.stride(1); a.o_sh = out.stride(2);
  a.lse = lse.data_ptr<float>();
  check_hip(dlion::launch_attn_fwd(a, static_cast<int>(q.size(3)), a.thresh16 > 0, cur_stream()), "attn_fwd");
  return {out, lse};
}

void attn_bwd(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& out, const Tensor& dout,
              const Tensor& lse, double p, int64_t seed, const Tensor& dq, const Tensor& dk, const Tensor& dv,
              const std::optional<Tensor>& colsum, const std::optional<Tensor>& rope_cos,
              const std::optional<Tensor>& rope_sin, int64_t window) {
  auto a = attn_args(q, k, v, p, seed);
  set_window(a, window, q.size(3));
  check_bthd(out, "out");
  check_bthd(dout, "dout");
  check_bthd(dq, "dq");
  check_bthd(dk, "dk");
  check_bthd(dv, "dv");
  TORCH_CHECK(out.strides() == dout.strides(), "dlion attn: out and dout must share strides");
  TORCH_CHECK(dk.strides() == dv.strides(), "dlion attn: dk and dv must share strides");
  TORCH_CHECK(lse.is_contiguous() && lse.scalar_type() == at::kFloat, "dlion attn: lse must be contiguous fp32");
  const c10::DeviceGuard g(q.device());
  auto delta = at::empty_like(lse);
  a.o = static_cast<const __bf16*>(out.data_ptr());
  a.dout = static_cast<const __bf16*>(dout.data_ptr());
  a.o_sb = out.stride(0); a.o_st = out.stride(1); a.o_sh = out.stride(2);
  a.lse = lse.data_ptr<float>();
  a.delta = delta.data_ptr<float>();
  a.dq = static_cast<__bf16*>(dq.data_ptr());
  a.dk = static_cast<__bf16*>(dk.data_ptr());
  a.dv = static_cast<__bf16*>(dv.data_ptr());
  a.dq_sb = dq.stride(0); a.dq_st = dq.stride(1); a.dq_sh = dq.stride(2);
  a.dk_sb = dk.stride(0); a.dk_st = dk.stride(1); a.dk_sh = dk.stride(2);
  a.colsum = nullptr;
  if (colsum.has_value()) {
    TORCH_CHECK(a.H == a.Hkv, "dlion attn: bias-gradient partials need H == Hkv");
    TORCH_CHECK(colsum->is_cuda() && colsum->scalar_type() == at::kFloat && colsum->is_contiguous() &&
                    colsum->dim() == 2 && colsum->size(0) == q.size(0) * ((q.size(1) + 31) / 32) &&
                    colsum->size(1) == 3 * q.size(2) * q.size(3),
                "dlion attn: colsum must be fp32 [B * ceil(T / 32), 3 * H * D]");
    a.colsum = colsum->data_ptr<float>();
  }
  a.rope_cos = a.rope_sin = nullptr;
  if (rope_cos.has_value() || rope_sin.has_value()) {
    TORCH_CHECK(rope_cos.has_value() && rope_sin.has_value() && !colsum.has_value(),
                "dlion attn: rope tables come as a pair, and not with bias-gradient partials");
    for (const Tensor* t : {&*rope_cos, &*rope_sin}) {
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() && t->dim() == 2 &&
                      t->size(0) >= q.size(1) && t->size(1) == q.size(3),
                  "dlion attn: rope tables must be contiguous bf16 [>= T, D]");
    }
    a.rope_cos = static_cast<const __bf16*>(rope_cos->data_ptr());
    a.rope_sin = static_cast<const __bf16*>(rope_sin->data_ptr());
  }
  check_hip(dlion::launch_attn_bwd(a, static_cast<int>(q.size(3)), a.thresh16 > 0, cur_stream()), "attn_bwd");
}

// ------------------------------------------------- residual + dropout + norm
void check_rows(const Tensor& t, const char* name, int64_t C) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous(), "dlion norm: ", name,
              " must be a contiguous bf16 GPU tensor");
  TORCH_CHECK(t.size(-1) == C, "dlion norm: ", name, " last dim mismatch");
}

std::pair<uint32_t, float> drop_params(double p) {
  uint32_t th = static_cast<uint32_t>(std::llround(p * 65536.0));
  if (th > 65535u) th = 65535u;
  return {th, static_cast<float>(65536.0 / (65536.0 - th))};
}

// returns (xo, h, mean, rstd); y may be None (plain norm, xo == x); bias is added to y
std::tuple<Tensor, Tensor, Tensor, Tensor> add_norm_fwd(const Tensor& x, const std::optional<Tensor>& y,
                                                        const std::optional<Tensor>& bias, const Tensor& gamma,
                                                        const std::optional<Tensor>& beta, double eps, bool rms,
                                                        double p, int64_t seed) {
  const int64_t C = x.size(-1), rows = x.numel() / C;
  check_rows(x, "x", C);
  check_rows(gamma, "gamma", C);
  TORCH_CHECK((C % 256 == 0 && C <= 1024) || (C % 1024 == 0 && C >= 2048 && C <= 8192 && C != 7168),
              "dlion norm: hidden size must be one of 256, 512, 768, 1024, 2048, 3072, 4096, 5120, 6144, 8192");
  TORCH_CHECK(rms || beta.has_value(), "dlion norm: LayerNorm needs beta");
  if (y.has_value()) check_rows(*y, "y", C);
  if (bias.has_value()) check_rows(*bias, "bias", C);
  const c10::DeviceGuard g(x.device());
  Tensor xo = y.has_value() ? at::empty_like(x) : x;
  Tensor h = at::empty_like(x);
  auto mean = at::empty({rows}, x.options().dtype(at::kFloat));
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  const auto dp = drop_params(y.has_value() ? p : 0.0);
  check_hip(dlion::launch_add_norm_fwd(x.data_ptr(), y.has_value() ? y->data_ptr() : nullptr,
                                       bias.has_value() ? bias->data_ptr() : nullptr, gamma.data_ptr(),
                                       beta.has_value() ? beta->data_ptr() : nullptr, xo.data_ptr(), h.data_ptr(),
                                       mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, static_cast<int>(C),
                                       static_cast<float>(eps), rms, static_cast<uint32_t>(seed), dp.first, dp.second,
                                       cur_stream()),
            "add_norm_fwd");
  return {xo, h, mean, rstd};
}

// returns (dx, dy, part[parts, 3, C] =dgamma / dbeta / dbias partials); dy only when want_dy
std::tuple<Tensor, Tensor, Tensor> add_norm_bwd(const Tensor& dh, const std::optional<Tensor>& dxo_in,
                                                const Tensor& xo, const Tensor& gamma, const Tensor& mean,
                                                const Tensor& rstd, bool rms, double p, int64_t seed, bool want_dy,
                                                int64_t parts) {
  const int64_t C = xo.size(-1), rows = xo.numel() / C;
  check_rows(dh, "dh", C);
  check_rows(xo, "xo", C);
  check_rows(gamma, "gamma", C);
  if (dxo_in.has_value()) check_rows(*dxo_in, "dxo_in", C);
  const c10::DeviceGuard g(xo.device());
  auto dx = at::empty_like(xo);
  Tensor dy = want_dy ? at::empty_like(xo) : Tensor();
  TORCH_CHECK(parts >= 1 && parts <= 65535, "add_norm_bwd: parts out of range");
  auto part = at::empty({parts, 3, C}, xo.options().dtype(at::kFloat));
  const auto dp = drop_params(want_dy ? p : 0.0);
  check_hip(dlion::launch_add_norm_bwd(dh.data_ptr(), dxo_in.has_value() ? dxo_in->data_ptr() : nullptr, xo.data_ptr(),
                                       gamma.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(), dx.data_ptr(),
                                       want_dy ? dy.data_ptr() : nullptr, part.data_ptr<float>(),
                                       static_cast<int>(parts), rows, static_cast<int>(C), rms,
                                       static_cast<uint32_t>(seed), dp.first, dp.second, cur_stream()),
            "add_norm_bwd");
  return {dx, dy, part};
}

// ---------------------------------------------------------------- bias + GELU
Tensor bias_gelu_fwd(const Tensor& z, const Tensor& b, bool exact) {
  const int64_t N = z.size(-1), rows = z.numel() / N;
  check_rows(z, "z", N);
  check_rows(b, "b", N);
  TORCH_CHECK(N % 8 == 0 && N <= 16384, "dlion gelu: N must be a multiple of 8 and <= 16384");
  const c10::DeviceGuard g(z.device());
  auto h = at::empty_like(z);
  check_hip(dlion::launch_bias_gelu_fwd(z.data_ptr(), b.data_ptr(), h.data_ptr(), rows, static_cast<int>(N), exact,
                                        cur_stream()),
            "bias_gelu_fwd");
  return h;
}

std::tuple<Tensor, Tensor> bias_gelu_bwd(const Tensor& dh, const Tensor& z, const Tensor& b, bool exact,
                                         int64_t parts) {
  const int64_t N = z.size(-1), rows = z.numel() / N;
  check_rows(dh, "dh", N);
  check_rows(z, "z", N);
  check_rows(b, "b", N);
  const c10::DeviceGuard g(z.device());
  auto dz = at::empty_like(z);
  auto part = at::empty({parts, N}, z.options().dtype(at::kFloat));
  check_hip(dlion::launch_bias_gelu_bwd(dh.data_ptr(), z.data_ptr(), b.data_ptr(), dz.data_ptr(),
                                        part.data_ptr<float>(), static_cast<int>(parts), rows, static_cast<int>(N),
                                        exact, cur_stream()),
            "bias_gelu_bwd");
  return {dz, part};
}

// sum of fp32 partials over dim 0 -> bf16 (split-K weight grads, bias / norm param grads)
// partials: a [S, ...] contiguous stack, or a row-strided 2-D view [S, n]
// (stride(1) == 1, e.g. one of the three [S, 3, C] norm parameter slices)
struct Partials {
  const float* ptr;
  int64_t S, n, ld;
};
Partials partials(const Tensor& part) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat, "dlion: partials must be fp32 on the GPU");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(part.data_ptr()) % 16 == 0, "dlion: partials must be 16-byte aligned");
  if (part.is_contiguous()) return {part.data_ptr<float>(), part.size(0), part.numel() / part.size(0),
                                    part.numel() / part.size(0)};
  TORCH_CHECK(part.dim() == 2 && part.stride(1) == 1 && part.stride(0) % 4 == 0,
              "dlion: strided partials must be 2-D with unit column stride");
  return {part.data_ptr<float>(), part.size(0), part.size(1), part.stride(0)};
}

// narrow tall stacks go through the row-split two-pass reduction (elementwise_kernels.hip);
// returns false when the one-pass kernels are the better fit
bool sum_partials_split(const std::vector<const float*>& ptrs, const std::vector<int64_t>& rows,
                        const std::vector<int64_t>& lds, int64_t n, void* out, bool accumulate, const float* scale,
                        const at::TensorOptions& opt) {
  int64_t total = 0;
  for (auto r : rows) total += r;
  const int Y = dlion::sum_partials_split_factor(n, total);
  if (Y <= 1) return false;
  auto scratch = at::empty({Y, n}, opt.dtype(at::kFloat));
  check_hip(dlion::launch_sum_partials_split(ptrs.data(), rows.data(), lds.data(), static_cast<int>(ptrs.size()), n, Y,
                                             scratch.data_ptr<float>(), out, accumulate, scale, cur_stream()),
            "sum_partials_split");
  return true;
}

bool sum_partials_split1(const Partials& P, void* out, bool accumulate, const float* scale,
                         const at::TensorOptions& opt) {
  return sum_partials_split({P.ptr}, {P.S}, {P.ld}, P.n, out, accumulate, scale, opt);
}

Tensor sum_partials(const Tensor& part) {
  const auto P = partials(part);
  TORCH_CHECK(P.n % 4 == 0, "dlion: partial row length must be a multiple of 4");
  const c10::DeviceGuard g(part.device());
  auto sizes = part.sizes().vec();
  sizes.erase(sizes.begin());
  auto out = at::empty(sizes, part.options().dtype(at::kBFloat16));
  if (sum_partials_split1(P, out.data_ptr(), false, nullptr, part.options())) return out;
  check_hip(dlion::launch_sum_partials(P.ptr, static_cast<int>(P.S), P.n, P.ld, out.data_ptr(), false, cur_stream()),
            "sum_partials");
  return out;
}

// out += sum_s part[s] in place (bf16 out, one rounding): gradient accumulation
// fused into the partial-sum reduction
void sum_partials_acc_(const Tensor& part, const Tensor& out) {
  const auto P = partials(part);
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kBFloat16 && out.is_contiguous() && out.numel() == P.n,
              "dlion: accumulation target must be a contiguous bf16 tensor of the partial row size");
  TORCH_CHECK(P.n % 4 == 0, "dlion: partial row length must be a multiple of 4");
  const c10::DeviceGuard g(part.device());
  if (sum_partials_split1(P, out.data_ptr(), true, nullptr, part.options())) return;
  check_hip(dlion::launch_sum_partials(P.ptr, static_cast<int>(P.S), P.n, P.ld, out.data_ptr(), true, cur_stream()),
            "sum_partials_acc_");
}

// out (+)= bf16(sum of every row of every stack in `parts`) -- a fusion window's per-micro-batch
// partial stacks reduced in one kernel, no concatenation
void sum_partials_multi_(at::TensorList parts, const Tensor& out, bool accumulate) {
  TORCH_CHECK(!parts.empty() && parts.size() <= 16, "dlion: 1..16 partial stacks");
  std::vector<const float*> ptrs;
  std::vector<int64_t> rows, lds;
  int64_t n = -1;
  for (const auto& t : parts) {
    const auto P = partials(t);
    TORCH_CHECK(n < 0 || P.n == n, "dlion: partial stacks must have the same row length");
    n = P.n;
    ptrs.push_back(P.ptr);
    rows.push_back(P.S);
    lds.push_back(P.ld);
  }
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kBFloat16 && out.is_contiguous() && out.numel() == n,
              "dlion: target must be a contiguous bf16 tensor of the partial row size");
  TORCH_CHECK(n % 4 == 0, "dlion: partial row length must be a multiple of 4");
  const c10::DeviceGuard g(out.device());
  if (sum_partials_split(ptrs, rows, lds, n, out.data_ptr(), accumulate, nullptr, out.options())) return;
  check_hip(dlion::launch_sum_partials_multi(ptrs.data(), rows.data(), lds.data(), static_cast<int>(parts.size()), n,
                                             out.data_ptr(), accumulate, cur_stream()),
            "sum_partials_multi_");
}

// out (+)= bf16(s[0] * sum_s part[s]): the LM head's split-K weight gradient scaled by the
// loss gradient (a device scalar) and accumulated into .grad in one pass
void sum_partials_scaled_(const Tensor& part, const Tensor& s, const Tensor& out, bool accumulate) {
  const auto P = partials(part);
  check_dev(s, "s");
  TORCH_CHECK(s.scalar_type() == at::kFloat && s.numel() >= 1, "dlion: scale must be float32");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kBFloat16 && out.is_contiguous() && out.numel() == P.n,
              "dlion: target must be a contiguous bf16 tensor of the partial row size");
  TORCH_CHECK(P.n % 4 == 0, "dlion: partial row length must be a multiple of 4");
  const c10::DeviceGuard g(part.device());
  if (sum_partials_split1(P, out.data_ptr(), accumulate, s.data_ptr<float>(), part.options())) return;
  check_hip(dlion::launch_sum_partials(P.ptr, static_cast<int>(P.S), P.n, P.ld, out.data_ptr(), accumulate, cur_stream(),
                                       s.data_ptr<float>()),
            "sum_partials_scaled_");
}

// fp32 [parts, N] column-sum partials of a bf16 [rows, N] matrix
Tensor colsum_partials(const Tensor& x, int64_t parts) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous(),
              "dlion colsum: x must be a contiguous bf16 GPU tensor");
  const int64_t N = x.size(-1), rows = x.numel() / N;
  TORCH_CHECK(N % 8 == 0 && N <= 16384 && parts >= 1 && parts <= 65535, "dlion colsum: bad shape");
  const c10::DeviceGuard g(x.device());
  auto part = at::empty({parts, N}, x.options().dtype(at::kFloat));
  check_hip(dlion::launch_colsum(x.data_ptr(), part.data_ptr<float>(), static_cast<int>(parts), rows,
                                 static_cast<int>(N), cur_stream()),
            "colsum");
  return part;
}

// ---------------------------------------------------------------- SwiGLU / RoPE
// [..., F] bf16 GPU tensor whose leading dims collapse to `rows` rows at a
// uniform row stride `ld` (unit column stride): contiguous tensors and column
// slices of a fused [..., 2F] projection output both qualify.
void rows_of(const Tensor& t, const char* what, int64_t& rows, int64_t& ld) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() >= 2 && t.stride(-1) == 1, "dlion ", what,
              ": operands must be bf16 GPU tensors [..., F] with unit column stride");
  ld = t.stride(-2);
  rows = 1;
  for (int64_t i = 0; i < t.dim() - 1; ++i) rows *= t.size(i);
  for (int64_t i = 0; i + 2 < t.dim(); ++i)
    TORCH_CHECK(t.size(i) == 1 || t.stride(i) == t.stride(i + 1) * t.size(i + 1), "dlion ", what,
                ": leading dims must collapse to rows of one stride");
  TORCH_CHECK(t.size(-1) % 8 == 0 && ld % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "dlion ",
              what, ": F, the row stride and the base must be 16-byte aligned");
}

void check_pair(const Tensor& g, const Tensor& u, int64_t& rows, int64_t& ld) {
  rows_of(g, "swiglu", rows, ld);
  int64_t r2, ld2;
  rows_of(u, "swiglu", r2, ld2);
  TORCH_CHECK(g.sizes() == u.sizes() && ld == ld2, "dlion swiglu: gate / up shapes or strides differ");
}

Tensor swiglu_fwd(const Tensor& g, const Tensor& u) {
  int64_t rows, ld;
  check_pair(g, u, rows, ld);
  const c10::DeviceGuard dg(g.device());
  auto h = at::empty(g.sizes(), g.options());
  check_hip(dlion::launch_swiglu_fwd(g.data_ptr(), u.data_ptr(), h.data_ptr(), rows, g.size(-1), ld, cur_stream()),
            "swiglu_fwd");
  return h;
}

std::tuple<Tensor, Tensor> swiglu_bwd(const Tensor& dh, const Tensor& g, const Tensor& u) {
  int64_t rows, ld;
  check_pair(g, u, rows, ld);
  TORCH_CHECK(dh.is_contiguous() && dh.sizes() == g.sizes() && dh.scalar_type() == at::kBFloat16,
              "dlion swiglu: dh must be contiguous bf16 of the gate's shape");
  const c10::DeviceGuard dg(g.device());
  const int64_t F = g.size(-1);
  auto dgate = at::empty(g.sizes(), g.options()), dup = at::empty(g.sizes(), g.options());
  check_hip(dlion::launch_swiglu_bwd(dh.data_ptr(), g.data_ptr(), u.data_ptr(), dgate.data_ptr(), dup.data_ptr(),
                                     rows, F, ld, F, cur_stream()),
            "swiglu_bwd");
  return {dgate, dup};
}

// gradient of a fused [gate | up] projection output: one [..., 2F] tensor
// (dgate in the first F columns, dup in the last F)
Tensor swiglu_bwd_fused(const Tensor& dh, const Tensor& g, const Tensor& u) {
  int64_t rows, ld;
  check_pair(g, u, rows, ld);
  TORCH_CHECK(dh.is_contiguous() && dh.sizes() == g.sizes() && dh.scalar_type() == at::kBFloat16,
              "dlion swiglu: dh must be contiguous bf16 of the gate's shape");
  const c10::DeviceGuard dg(g.device());
  const int64_t F = g.size(-1);
  auto shape = g.sizes().vec();
  shape.back() = 2 * F;
  auto dgu = at::empty(shape, g.options());
  auto* base = static_cast<uint16_t*>(dgu.data_ptr());
  check_hip(dlion::launch_swiglu_bwd(dh.data_ptr(), g.data_ptr(), u.data_ptr(), base, base + F, rows, F, ld, 2 * F,
                                     cur_stream()),
            "swiglu_bwd_fused");
  return dgu;
}

// swiglu_fwd plus the token-contiguous copy hT [F, rows] (rows % 64 == 0, F % 64 == 0)
std::tuple<Tensor, Tensor> swiglu_fwd_t(const Tensor& g, const Tensor& u) {
  int64_t rows, ld;
  check_pair(g, u, rows, ld);
  const int64_t F = g.size(-1);
  TORCH_CHECK(rows % 64 == 0 && F % 64 == 0, "dlion swiglu_fwd_t: rows and F must be multiples of 64");
  const c10::DeviceGuard dg(g.device());
  auto h = at::empty(g.sizes(), g.options());
  auto ht = at::empty({F, rows}, g.options());
  check_hip(dlion::launch_swiglu_fwd_t(g.data_ptr(), u.data_ptr(), h.data_ptr(), ht.data_ptr(), rows, F, ld,
                                       cur_stream()),
            "swiglu_fwd_t");
  return {h, ht};
}

// swiglu_bwd_fused plus the token-contiguous copy dguT [2F, rows] of its result
// (rows % 64 == 0, F % 64 == 0)
std::tuple<Tensor, Tensor> swiglu_bwd_fused_t(const Tensor& dh, const Tensor& g, const Tensor& u) {
  int64_t rows, ld;
  check_pair(g, u, rows, ld);
  TORCH_CHECK(dh.is_contiguous() && dh.sizes() == g.sizes() && dh.scalar_type() == at::kBFloat16,
              "dlion swiglu: dh must be contiguous bf16 of the gate's shape");
  const int64_t F = g.size(-1);
  TORCH_CHECK(rows % 64 == 0 && F % 64 == 0, "dlion swiglu_bwd_fused_t: rows and F must be multiples of 64");
  const c10::DeviceGuard dg(g.device());
  auto shape = g.sizes().vec();
  shape.back() = 2 * F;
  auto dgu = at::empty(shape, g.options());
  auto dgut = at::empty({2 * F, rows}, g.options());
  check_hip(dlion::launch_swiglu_bwd_t(dh.data_ptr(), g.data_ptr(), u.data_ptr(), dgu.data_ptr(), dgut.data_ptr(),
                                       rows, F, ld, cur_stream()),
            "swiglu_bwd_fused_t");
  return {dgu, dgut};
}

// x [B, T, H, D] with unit-stride heads (stride(2) == D) and any token stride
// (a q or k slice of a fused projection output), cos / sin [>= T, D] bf16
// (row t = position t); y contiguous.
Tensor rope(const Tensor& x, const Tensor& cos, const Tensor& sin, bool inverse) {
  TORCH_CHECK(x.dim() == 4 && x.is_cuda() && x.scalar_type() == at::kBFloat16, "dlion rope: x must be bf16 [B, T, H, D]");
  const int64_t B = x.size(0), T = x.size(1), H = x.size(2), D = x.size(3);
  TORCH_CHECK(x.stride(3) == 1 && x.stride(2) == D && (B == 1 || x.stride(0) == T * x.stride(1)) &&
                  x.stride(1) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "dlion rope: x must have contiguous heads and a uniform, 16-byte aligned token stride");
  TORCH_CHECK(D % 8 == 0, "dlion rope: head_dim must be a multiple of 8");
  for (const Tensor* t : {&cos, &sin})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() && t->dim() == 2 &&
                    t->size(0) >= T && t->size(1) == D,
                "dlion rope: cos/sin must be contiguous bf16 [>=T, D]");
  const c10::DeviceGuard dg(x.device());
  auto y = at::empty(x.sizes(), x.options());
  check_hip(dlion::launch_rope(x.data_ptr(), cos.data_ptr(), sin.data_ptr(), y.data_ptr(), B * T,
                               static_cast<int>(T), static_cast<int>(H), static_cast<int>(D), inverse, x.stride(1),
                               H * D, cur_stream()),
            "rope");
  return y;
}

// in place on x (same layout rules as rope): each lane reads its rotate-half
// pair before writing it, so x may be a strided slice of a packed gradient
void rope_(const Tensor& x, const Tensor& cos, const Tensor& sin, bool inverse) {
  TORCH_CHECK(x.dim() == 4 && x.is_cuda() && x.scalar_type() == at::kBFloat16, "dlion rope_: x must be bf16 [B, T, H, D]");
  const int64_t B = x.size(0), T = x.size(1), H = x.size(2), D = x.size(3);
  TORCH_CHECK(x.stride(3) == 1 && x.stride(2) == D && (B == 1 || x.stride(0) == T * x.stride(1)) &&
                  x.stride(1) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && D % 8 == 0,
              "dlion rope_: x must have contiguous heads and a uniform, 16-byte aligned token stride");
  for (const Tensor* t : {&cos, &sin})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() && t->dim() == 2 &&
                    t->size(0) >= T && t->size(1) == D,
                "dlion rope_: cos/sin must be contiguous bf16 [>=T, D]");
  const c10::DeviceGuard dg(x.device());
  check_hip(dlion::launch_rope(x.data_ptr(), cos.data_ptr(), sin.data_ptr(), x.data_ptr(), B * T,
                               static_cast<int>(T), static_cast<int>(H), static_cast<int>(D), inverse, x.stride(1),
                               x.stride(1), cur_stream()),
            "rope_");
}

// ---------------------------------------------------------------- GEMM (NT)
// a [M, K], b [N, K] (rows may be strided, unit column stride) -> c [M, N] bf16
void check_gemm_operand(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 2 && t.stride(1) == 1,
              "dlion gemm: ", name, " must be a 2-D bf16 GPU tensor with unit column stride");
  TORCH_CHECK(t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              "dlion gemm: ", name, " rows must be 16-byte aligned");
}

bool gemm_nt_supported(const Tensor& a, const Tensor& b) {
  return a.dim() == 2 && b.dim() == 2 && a.size(1) == b.size(1) && a.size(1) % 128 == 0 && b.size(0) % 8 == 0 &&
         a.size(0) * a.stride(0) < (1ll << 31) && b.size(0) * b.stride(0) < (1ll << 31);
}

void gemm_nt_launch(const Tensor& a, const Tensor& b, const Tensor& c, const Tensor* bias, const Tensor* aux,
                    int64_t epi, const Tensor* part = nullptr) {
  check_gemm_operand(a, "a");
  check_gemm_operand(b, "b");
  check_gemm_operand(c, "out");
  TORCH_CHECK(gemm_nt_supported(a, b), "dlion gemm: unsupported shape a=", a.sizes(), " b=", b.sizes(),
              " (needs K % 128 == 0, N % 8 == 0)");
  TORCH_CHECK(c.size(0) == a.size(0) && c.size(1) == b.size(0), "dlion gemm: output shape mismatch");
  if (bias) {
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() &&
                    bias->numel() == b.size(0),
                "dlion gemm: bias must be a contiguous bf16 [N] tensor");
  }
  if (aux) {
    check_gemm_operand(*aux, "aux");
    TORCH_CHECK(aux->size(0) == c.size(0) && aux->size(1) == c.size(1), "dlion gemm: aux must match the output shape");
  }
  if (part) {
    TORCH_CHECK(part->is_cuda() && part->scalar_type() == at::kFloat && part->is_contiguous() &&
                    part->size(0) == 2 * ((a.size(0) + 255) / 256) && part->size(1) == b.size(0),
                "dlion gemm: part must be fp32 [2 * ceil(M / 256), N]");
  }
  const c10::DeviceGuard g(a.device());
  check_hip(dlion::launch_gemm_nt(a.data_ptr(), static_cast<int>(a.stride(0)), b.data_ptr(),
                                  static_cast<int>(b.stride(0)), c.data_ptr(), static_cast<int>(c.stride(0)),
                                  bias ? bias->data_ptr() : nullptr, aux ? aux->data_ptr() : nullptr,
                                  aux ? static_cast<int>(aux->stride(0)) : 0, static_cast<int>(a.size(0)),
                                  static_cast<int>(b.size(0)), static_cast<int>(a.size(1)), static_cast<int>(epi),
                                  part ? part->data_ptr<float>() : nullptr, cur_stream()),
            "gemm_nt");
}

Tensor gemm_nt(const Tensor& a, const Tensor& b, const std::optional<Tensor>& bias) {
  auto c = at::empty({a.size(0), b.size(0)}, a.options());
  gemm_nt_launch(a, b, c, bias.has_value() ? &*bias : nullptr, nullptr, bias.has_value() ? 1 : 0);
  return c;
}

void gemm_nt_out(const Tensor& a, const Tensor& b, const std::optional<Tensor>& bias, const Tensor& out) {
  gemm_nt_launch(a, b, out, bias.has_value() ? &*bias : nullptr, nullptr, bias.has_value() ? 1 : 0);
}

// h = gelu(z + bias), z = a . b^T (bf16): returns (h, z) -- z is what the bias+GELU backward reads
std::tuple<Tensor, Tensor> gemm_nt_gelu(const Tensor& a, const Tensor& b, const Tensor& bias, bool exact) {
  auto h = at::empty({a.size(0), b.size(0)}, a.options());
  auto z = at::empty_like(h);
  gemm_nt_launch(a, b, h, &bias, &z, exact ? 3 : 2);
  return {h, z};
}

// ------------------------------------------- hipBLASLt GEMM + epilogue (lt_gemm.cpp)
// out [M, N] = epi(a [M, K] . b [N, K]^T); epi 0 plain, 1 + bias, 2 gelu_tanh(z + bias).
// Returns false when hipBLASLt has no kernel for the case (caller falls back).
bool lt_gemm_nt(const Tensor& a, const Tensor& b, const std::optional<Tensor>& bias, int64_t epi, const Tensor& out) {
  check_gemm_operand(a, "a");
  check_gemm_operand(b, "b");
  check_gemm_operand(out, "out");
  TORCH_CHECK(epi >= 0 && epi <= 2, "dlion lt_gemm: bad epilogue ", epi);
  TORCH_CHECK(a.size(1) == b.size(1) && out.size(0) == a.size(0) && out.size(1) == b.size(0),
              "dlion lt_gemm: shape mismatch a=", a.sizes(), " b=", b.sizes(), " out=", out.sizes());
  TORCH_CHECK(bias.has_value() == (epi != 0), "dlion lt_gemm: epilogue ", epi, epi ? " needs" : " takes no", " bias");
  if (bias.has_value()) {
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() &&
                    bias->numel() == b.size(0),
                "dlion lt_gemm: bias must be a contiguous bf16 [N] tensor");
  }
  const c10::DeviceGuard g(a.device());
  return dlion::lt_gemm(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), out.data_ptr(), out.stride(0),
                        bias.has_value() ? bias->data_ptr() : nullptr, a.size(0), b.size(0), a.size(1),
                        static_cast<int>(epi), a.device().index(), cur_stream(), dlion::Layout::NT, false);
}

// out [M, N] = a [M, K] . b [K, N] (b row-major, e.g. an nn.Linear weight in an
// input gradient dY . W); plain epilogue.  False when hipBLASLt has no kernel.
bool lt_gemm_nn(const Tensor& a, const Tensor& b, const Tensor& out) {
  check_gemm_operand(a, "a");
  check_gemm_operand(b, "b");
  check_gemm_operand(out, "out");
  TORCH_CHECK(a.size(1) == b.size(0) && out.size(0) == a.size(0) && out.size(1) == b.size(1),
              "dlion lt_gemm_nn: shape mismatch a=", a.sizes(), " b=", b.sizes(), " out=", out.sizes());
  const c10::DeviceGuard g(a.device());
  return dlion::lt_gemm(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), out.data_ptr(), out.stride(0), nullptr,
                        a.size(0), b.size(1), a.size(1), 0, a.device().index(), cur_stream(), dlion::Layout::NN, false);
}

// out [M, N] (+)= a [M, K] . b [N, K]^T, plain epilogue, beta = 1 when accumulating (a weight gradient from
// token-contiguous operand copies).
bool lt_gemm_nt_acc(const Tensor& a, const Tensor& b, const Tensor& out, bool accumulate) {
  check_gemm_operand(a, "a");
  check_gemm_operand(b, "b");
  check_gemm_operand(out, "out");
  TORCH_CHECK(a.size(1) == b.size(1) && out.size(0) == a.size(0) && out.size(1) == b.size(0),
              "dlion lt_gemm_nt_acc: shape mismatch a=", a.sizes(), " b=", b.sizes(), " out=", out.sizes());
  const c10::DeviceGuard g(a.device());
  return dlion::lt_gemm(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), out.data_ptr(), out.stride(0), nullptr,
                        a.size(0), b.size(0), a.size(1), 0, a.device().index(), cur_stream(), dlion::Layout::NT,
                        accumulate);
}

// Any of the four layouts with beta = 1 when accumulating: out [M, N] (+)= op(a) . op(b) with
// layout 0 NT: a [M, K], b [N, K];  1 NN: a [M, K], b [K, N];  2 TN: a [K, M], b [K, N];  3 TT: a [K, M], b [N, K].
bool lt_gemm_layout(const Tensor& a, const Tensor& b, const Tensor& out, int64_t layout, bool accumulate) {
  check_gemm_operand(a, "a");
  check_gemm_operand(b, "b");
  check_gemm_operand(out, "out");
  TORCH_CHECK(layout >= 0 && layout <= 3, "dlion lt_gemm_layout: layout must be 0..3");
  const bool at = layout >= 2, bt = layout == 0 || layout == 3;  // a stored [K, M]; b stored [N, K]
  const int64_t M = at ? a.size(1) : a.size(0), K = at ? a.size(0) : a.size(1), N = bt ? b.size(0) : b.size(1);
  TORCH_CHECK((bt ? b.size(1) : b.size(0)) == K && out.size(0) == M && out.size(1) == N,
              "dlion lt_gemm_layout: shape mismatch a=", a.sizes(), " b=", b.sizes(), " out=", out.sizes(),
              " layout ", layout);
  const c10::DeviceGuard g(a.device());
  return dlion::lt_gemm(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), out.data_ptr(), out.stride(0), nullptr,
                        M, N, K, 0, a.device().index(), cur_stream(), static_cast<dlion::Layout>(layout), accumulate);
}

// out [M, N] (+)= a [K, M]^T . b [K, N] (a weight gradient over the token axis; accumulate: beta = 1).
bool lt_gemm_tn(const Tensor& a, const Tensor& b, const Tensor& out, bool accumulate) {
  check_gemm_operand(a, "a");
  check_gemm_operand(b, "b");
  check_gemm_operand(out, "out");
  TORCH_CHECK(a.size(0) == b.size(0) && out.size(0) == a.size(1) && out.size(1) == b.size(1),
              "dlion lt_gemm_tn: shape mismatch a=", a.sizes(), " b=", b.sizes(), " out=", out.sizes());
  const c10::DeviceGuard g(a.device());
  return dlion::lt_gemm(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), out.data_ptr(), out.stride(0), nullptr,
                        a.size(1), b.size(1), a.size(0), 0, a.device().index(), cur_stream(), dlion::Layout::TN,
                        accumulate);
}

// ------------------------------------------------------------- embedding
void check_bf16_contig(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous() &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              "dlion embed: ", name, " must be a contiguous, 16-byte aligned bf16 GPU tensor");
}

// out [B, T, C] = dropout(wte[ids] + wpe[t]) for ids [B, T]
int32_t* err_ptr(const std::optional<Tensor>& err, const Tensor& like) {
  if (!err.has_value()) return nullptr;
  TORCH_CHECK(err->scalar_type() == at::kInt && err->numel() >= 1 && err->device() == like.device(),
              "dlion: the index-error flag must be an int32 tensor on the ids' device");
  return err->data_ptr<int32_t>();
}

// err[0] |= code when any of ids is outside [0, hi) and != ignore
void index_check_(const Tensor& ids, int64_t hi, int64_t ignore, const Tensor& err, int64_t code) {
  check_dev(ids, "ids");
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous(), "dlion index_check: ids must be contiguous int64");
  const c10::DeviceGuard g(ids.device());
  check_hip(dlion::launch_index_check(ids.data_ptr<int64_t>(), ids.numel(), hi, ignore, err_ptr(err, ids),
                                      static_cast<int>(code), cur_stream()),
            "index_check");
}

Tensor embed_fwd(const Tensor& ids, const Tensor& wte, const Tensor& wpe, double p, int64_t seed,
                 const std::optional<Tensor>& err) {
  check_dev(ids, "ids");
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.dim() == 2, "dlion embed: ids must be int64 [B, T]");
  check_bf16_contig(wte, "wte");
  check_bf16_contig(wpe, "wpe");
  const int64_t C = wte.size(1), T = ids.size(1);
  TORCH_CHECK(wpe.size(1) == C && T <= wpe.size(0) && C % 8 == 0, "dlion embed: shape mismatch / C % 8 != 0");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dlion embed: dropout must be in [0, 1)");
  const c10::DeviceGuard g(ids.device());
  auto out = at::empty({ids.size(0), T, C}, wte.options());
  const auto dp = drop_params(p);
  check_hip(dlion::launch_embed_fwd(ids.data_ptr<int64_t>(), wte.data_ptr(), wpe.data_ptr(), out.data_ptr(), ids.numel(),
                                    static_cast<int>(C), static_cast<int>(T), wte.size(0), static_cast<uint32_t>(seed),
                                    dp.first, dp.second, err_ptr(err, ids), cur_stream()),
            "embed_fwd");
  return out;
}

// dwte[sid] += segmented row sums of the dropout-backward of dx; dwpe (+)= batch sums per position
void embed_bwd_(const Tensor& dx, const std::optional<Tensor>& sid, const std::optional<Tensor>& perm,
                const std::optional<Tensor>& dwte, const std::optional<Tensor>& dwpe, int64_t T, bool pos_accumulate,
                double p, int64_t seed) {
  check_bf16_contig(dx, "dx");
  const int64_t C = dx.size(-1), n = dx.numel() / C;
  TORCH_CHECK(T > 0 && n % T == 0 && C % 8 == 0, "dlion embed: dx must be [B*T, C] with C % 8 == 0");
  int64_t V = 0;
  if (dwte.has_value()) {
    check_bf16_contig(*dwte, "dwte");
    TORCH_CHECK(dwte->dim() == 2 && dwte->size(1) == C, "dlion embed: dwte must be [V, C]");
    TORCH_CHECK(sid.has_value() && perm.has_value() && sid->numel() == n && perm->numel() == n &&
                    sid->scalar_type() == at::kLong && perm->scalar_type() == at::kLong && sid->is_contiguous() &&
                    perm->is_contiguous(),
                "dlion embed: the token gradient needs sorted ids and their permutation (int64 [n])");
    V = dwte->size(0);
  }
  if (dwpe.has_value()) {
    check_bf16_contig(*dwpe, "dwpe");
    TORCH_CHECK(dwpe->size(-1) == C && dwpe->size(0) >= T, "dlion embed: dwpe must be [>= T, C]");
  }
  const c10::DeviceGuard g(dx.device());
  const auto dp = drop_params(p);
  check_hip(dlion::launch_embed_bwd(dx.data_ptr(), dwte.has_value() ? sid->data_ptr<int64_t>() : nullptr,
                                    dwte.has_value() ? perm->data_ptr<int64_t>() : nullptr,
                                    dwte.has_value() ? dwte->data_ptr() : nullptr,
                                    dwpe.has_value() ? dwpe->data_ptr() : nullptr, n, static_cast<int>(C),
                                    static_cast<int>(T), V, pos_accumulate ? 1 : 0, static_cast<uint32_t>(seed),
                                    dp.first, dp.second, cur_stream()),
            "embed_bwd");
}

// y (+)= bf16(x * bf16(s)), s a 1-element fp32 device tensor (no host sync)
void scale_acc_(const Tensor& x, const Tensor& s, const Tensor& y, bool accumulate) {
  check_bf16_contig(x, "x");
  check_bf16_contig(y, "y");
  check_dev(s, "s");
  TORCH_CHECK(s.scalar_type() == at::kFloat && s.numel() >= 1, "dlion scale_acc: s must be float32");
  TORCH_CHECK(x.numel() == y.numel() && x.numel() % 8 == 0, "dlion scale_acc: size mismatch / numel % 8 != 0");
  const c10::DeviceGuard g(x.device());
  check_hip(dlion::launch_scale_acc(x.data_ptr(), s.data_ptr<float>(), y.data_ptr(), x.numel(), accumulate ? 1 : 0,
                                    cur_stream()),
            "scale_acc");
}

// diagnostic: c = a . b^T with per-block timestamps stamps [blocks, 8] int64
Tensor gemm_nt_stamped(const Tensor& a, const Tensor& b, const Tensor& stamps) {
  check_gemm_operand(a, "a");
  check_gemm_operand(b, "b");
  TORCH_CHECK(gemm_nt_supported(a, b), "dlion gemm: unsupported shape");
  const int64_t blocks = ((a.size(0) + 255) / 256) * ((b.size(0) + 255) / 256);
  TORCH_CHECK(stamps.is_cuda() && stamps.scalar_type() == at::kLong && stamps.is_contiguous() &&
                  stamps.numel() >= blocks * 8,
              "dlion gemm: stamps must be int64 [blocks, 8]");
  auto c = at::empty({a.size(0), b.size(0)}, a.options());
  const c10::DeviceGuard g(a.device());
  check_hip(dlion::launch_gemm_nt_stamped(a.data_ptr(), static_cast<int>(a.stride(0)), b.data_ptr(),
                                          static_cast<int>(b.stride(0)), c.data_ptr(), static_cast<int>(c.stride(0)),
                                          static_cast<int>(a.size(0)), static_cast<int>(b.size(0)),
                                          static_cast<int>(a.size(1)),
                                          reinterpret_cast<unsigned long long*>(stamps.data_ptr<int64_t>()),
                                          cur_stream()),
            "gemm_nt_stamped");
  return c;
}

// dz = (a . b^T) * gelu'(z + bias) -> (dz [M, N] bf16, part [2 * ceil(M/256), N] fp32 bias-grad partials):
// the MLP down-projection's input gradient fused with the bias+GELU backward
// (h, d) = (gelu(a . b^T + bias), gelu'(a . b^T + bias)) in one GEMM drain (EPI 6 / 7)
std::tuple<Tensor, Tensor> gemm_nt_gelu_d(const Tensor& a, const Tensor& b, const Tensor& bias, bool exact) {
  auto h = at::empty({a.size(0), b.size(0)}, a.options());
  auto d = at::empty({a.size(0), b.size(0)}, a.options());
  gemm_nt_launch(a, b, h, &bias, &d, exact ? 7 : 6);
  return {h, d};
}

// (dz, part) = (bf16(a . b^T) * d, fp32 [2 * ceil(M/256), N] column-sum partials of dz) (EPI 8)
std::tuple<Tensor, Tensor> gemm_nt_dmul(const Tensor& a, const Tensor& b, const Tensor& d) {
  auto dz = at::empty({a.size(0), b.size(0)}, a.options());
  auto part = at::empty({2 * ((a.size(0) + 255) / 256), b.size(0)}, a.options().dtype(at::kFloat));
  gemm_nt_launch(a, b, dz, nullptr, &d, 8, &part);
  return {dz, part};
}

std::tuple<Tensor, Tensor> gemm_nt_dgelu(const Tensor& a, const Tensor& b, const Tensor& bias, const Tensor& z,
                                         bool exact) {
  auto dz = at::empty({a.size(0), b.size(0)}, a.options());
  auto part = at::empty({2 * ((a.size(0) + 255) / 256), b.size(0)}, a.options().dtype(at::kFloat));
  gemm_nt_launch(a, b, dz, &bias, &z, exact ? 5 : 4, &part);
  return {dz, part};
}

// ------------------------------------------------------------- weight-gradient GEMM
// out [splits, M, N] fp32: out[z] = sum over split z's rows of P^T Q, the rows running over the
// concatenation of the segments P[i] [rows, M] / Q[i] [rows, N] (same shape and row stride each)
void gemm_tn_check_launch(at::TensorList P, at::TensorList Q, int64_t splits, const Tensor& out, bool accumulate) {
  TORCH_CHECK(!P.empty() && P.size() == Q.size() && P.size() <= 16, "dlion gemm_tn: 1..16 segment pairs");
  const int64_t rows = P[0].size(0), M = P[0].size(1), N = Q[0].size(1);
  const int64_t ldp = P[0].stride(0), ldq = Q[0].stride(0);
  std::vector<const void*> pp, qq;
  for (size_t i = 0; i < P.size(); ++i) {
    for (const Tensor* t : {&P[i], &Q[i]}) {
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->dim() == 2 && t->stride(1) == 1 &&
                      reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                  "dlion gemm_tn: operands must be 2-D bf16 GPU tensors with unit column stride, 16-byte aligned");
    }
    TORCH_CHECK(P[i].size(0) == rows && Q[i].size(0) == rows && P[i].size(1) == M && Q[i].size(1) == N &&
                    P[i].stride(0) == ldp && Q[i].stride(0) == ldq,
                "dlion gemm_tn: every segment must have the same shape and row stride");
    pp.push_back(P[i].data_ptr());
    qq.push_back(Q[i].data_ptr());
  }
  TORCH_CHECK(rows % 128 == 0 && M % 8 == 0 && N % 8 == 0 && ldp % 8 == 0 && ldq % 8 == 0,
              "dlion gemm_tn: rows % 128, M % 8, N % 8 and row strides % 8 must be 0");
  TORCH_CHECK(splits >= 1 && splits <= static_cast<int64_t>(P.size()) * rows / 128, "dlion gemm_tn: bad split count");
  const bool bf16_out = out.scalar_type() == at::kBFloat16;
  if (bf16_out) {
    TORCH_CHECK(splits == 1 && out.is_cuda() && out.is_contiguous() && out.numel() == M * N &&
                    reinterpret_cast<uintptr_t>(out.data_ptr()) % 8 == 0,
                "dlion gemm_tn: a bf16 out must be one contiguous [M, N] (unsplit) tensor");
  } else {
    TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() && out.dim() == 3 &&
                    out.size(0) == splits && out.size(1) == M && out.size(2) == N,
                "dlion gemm_tn: out must be a contiguous fp32 [splits, M, N] tensor");
  }
  const c10::DeviceGuard g(P[0].device());
  check_hip(dlion::launch_gemm_tn(pp.data(), qq.data(), static_cast<int>(P.size()), rows, static_cast<int>(ldp),
                                  static_cast<int>(ldq), bf16_out ? nullptr : out.data_ptr<float>(),
                                  static_cast<int>(M), static_cast<int>(N), static_cast<int>(splits), accumulate,
                                  cur_stream(), bf16_out ? out.data_ptr() : nullptr),
            "gemm_tn");
}

Tensor gemm_tn(at::TensorList P, at::TensorList Q, int64_t splits) {
  TORCH_CHECK(!P.empty() && !Q.empty(), "dlion gemm_tn: no operands");
  auto out = at::empty({splits, P[0].size(1), Q[0].size(1)}, P[0].options().dtype(at::kFloat));
  gemm_tn_check_launch(P, Q, splits, out, false);
  return out;
}

// out[z] (+)= the split-z partial of P^T Q (out: the fp32 [splits, M, N] accumulator), or, for a
// bf16 out (any contiguous shape of M * N elements), out (+)= bf16(P^T Q) unsplit
void gemm_tn_(at::TensorList P, at::TensorList Q, const Tensor& out, bool accumulate) {
  if (out.scalar_type() == at::kBFloat16) {
    gemm_tn_check_launch(P, Q, 1, out, accumulate);
    return;
  }
  TORCH_CHECK(out.dim() == 3, "dlion gemm_tn_: out must be [splits, M, N]");
  gemm_tn_check_launch(P, Q, out.size(0), out, accumulate);
}

// ------------------------------------------------------------- LoRA
void check_lora_rows(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 2 && t.stride(1) == 1 &&
                  t.stride(0) % 8 == 0 && t.size(1) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              "dlion lora: ", name, " must be a 2-D bf16 GPU tensor, unit column stride, row stride and width % 8 == 0");
}

// u [M, r] = scale * drop(x) . w^T, w [r, K]
Tensor lora_rows(const Tensor& x, const Tensor& w, double scale, double p, int64_t seed) {
  check_lora_rows(x, "x");
  check_bf16_contig(w, "w");
  const int64_t r = w.size(0);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == x.size(1) && (r == 8 || r == 16) && x.size(1) % 32 == 0,
              "dlion lora: w must be [8|16, K] with K % 32 == 0");
  const c10::DeviceGuard g(x.device());
  auto u = at::empty({x.size(0), r}, x.options());
  const auto dp = drop_params(p);
  check_hip(dlion::launch_lora_rows(x.data_ptr(), x.stride(0), w.data_ptr(), u.data_ptr(), x.size(0),
                                    static_cast<int>(x.size(1)), static_cast<int>(r), static_cast<float>(scale),
                                    static_cast<uint32_t>(seed), dp.first, dp.second, cur_stream()),
            "lora_rows");
  return u;
}

// out [M, N] = o + bf16(s * u . b^T)
Tensor lora_up(const Tensor& o, const Tensor& u, const Tensor& b, double s) {
  check_lora_rows(o, "o");
  check_bf16_contig(u, "u");
  check_bf16_contig(b, "b");
  const int64_t r = u.size(1);
  TORCH_CHECK(u.dim() == 2 && u.size(0) == o.size(0) && b.dim() == 2 && b.size(0) == o.size(1) && b.size(1) == r &&
                  (r == 8 || r == 16),
              "dlion lora: shape mismatch (u [M, r], b [N, r], r in {8, 16})");
  const c10::DeviceGuard g(o.device());
  auto out = at::empty({o.size(0), o.size(1)}, o.options());
  check_hip(dlion::launch_lora_up(o.data_ptr(), o.stride(0), u.data_ptr(), b.data_ptr(), out.data_ptr(), o.size(0),
                                  static_cast<int>(o.size(1)), static_cast<int>(r), static_cast<float>(s), cur_stream()),
            "lora_up");
  return out;
}

// no a: (part [P, N, r] = yscale * per-range g^T y, -);
// a:    (part [P, r, N] = yscale * per-range y^T drop(g), dx = drop'(y . a))
std::tuple<Tensor, Tensor> lora_cols(const Tensor& g, const Tensor& y, const std::optional<Tensor>& a, double yscale,
                                     double p, int64_t seed) {
  check_lora_rows(g, "g");
  check_bf16_contig(y, "y");
  const int64_t r = y.size(1), M = g.size(0), N = g.size(1);
  TORCH_CHECK(y.dim() == 2 && y.size(0) == M && (r == 8 || r == 16), "dlion lora: y must be [M, 8|16]");
  const bool mode1 = a.has_value();
  if (mode1) {
    check_bf16_contig(*a, "a");
    TORCH_CHECK(a->dim() == 2 && a->size(0) == r && a->size(1) == N, "dlion lora: a must be [r, N]");
  }
  const c10::DeviceGuard dg(g.device());
  const int parts = dlion::lora_cols_parts(M, static_cast<int>(N));
  auto part = mode1 ? at::empty({parts, r, N}, g.options().dtype(at::kFloat))
                    : at::empty({parts, N, r}, g.options().dtype(at::kFloat));
  Tensor dx = mode1 ? at::empty({M, N}, g.options()) : Tensor();
  const auto dp = drop_params(mode1 ? p : 0.0);
  check_hip(dlion::launch_lora_cols(g.data_ptr(), g.stride(0), y.data_ptr(), mode1 ? a->data_ptr() : nullptr,
                                    mode1 ? dx.data_ptr() : nullptr, part.data_ptr<float>(), M, static_cast<int>(N),
                                    static_cast<int>(r), parts, mode1 ? 1 : 0, static_cast<float>(yscale),
                                    static_cast<uint32_t>(seed), dp.first,
                                    dp.second, cur_stream()),
            "lora_cols");
  return {part, dx};
}


// 4-bit blockwise quantization (quant.hip): w (any float dtype, numel % 64 == 0) -> (q uint8 [n/2], absmax fp32 [n/64])
std::tuple<Tensor, Tensor> quant4(const Tensor& w, const Tensor& code) {
  check_dev(w, "w");
  check_dev(code, "code");
  TORCH_CHECK(code.scalar_type() == at::kFloat && code.numel() == 16, "dlion quant4: code must be float32[16]");
  const int64_t n = w.numel();
  TORCH_CHECK(n % 64 == 0, "dlion quant4: numel must be a multiple of 64, got ", n);
  TORCH_CHECK(w.is_contiguous() && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              "dlion quant4: w must be contiguous and 16-byte aligned (the kernel reads it as flat vectors)");
  const c10::DeviceGuard g(w.device());
  auto q = at::empty({n / 2}, w.options().dtype(at::kByte));
  auto absmax = at::empty({n / 64}, w.options().dtype(at::kFloat));
  check_hip(dlion::launch_quant4(dtype_code(w.scalar_type()), w.data_ptr(), code.data_ptr<float>(),
                                 q.data_ptr<uint8_t>(), absmax.data_ptr<float>(), n, cur_stream()),
            "quant4");
  return {q, absmax};
}

// out (contiguous, numel n = 2 * q.numel(), any float dtype) = code[q] * absmax
void dequant4_(const Tensor& q, const Tensor& absmax, const Tensor& code, const Tensor& out) {
  check_dev(q, "q");
  check_dev(absmax, "absmax");
  check_dev(code, "code");
  check_dev(out, "out");
  TORCH_CHECK(q.scalar_type() == at::kByte && absmax.scalar_type() == at::kFloat && code.scalar_type() == at::kFloat &&
                  code.numel() == 16,
              "dlion dequant4: q uint8, absmax / code float32");
  const int64_t n = out.numel();
  TORCH_CHECK(n % 64 == 0 && q.numel() == n / 2 && absmax.numel() == n / 64,
              "dlion dequant4: out numel ", n, " does not match q ", q.numel(), " / absmax ", absmax.numel());
  TORCH_CHECK(reinterpret_cast<uintptr_t>(q.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "dlion dequant4: q and out must be 16-byte aligned");
  TORCH_CHECK(out.is_contiguous() && q.is_contiguous() && absmax.is_contiguous(),
              "dlion dequant4: q, absmax and out must be contiguous (out is written linearly)");
  const c10::DeviceGuard g(out.device());
  check_hip(dlion::launch_dequant4(dtype_code(out.scalar_type()), q.data_ptr<uint8_t>(), absmax.data_ptr<float>(),
                                   code.data_ptr<float>(), out.data_ptr(), n, cur_stream()),
            "dequant4");
}

// out [C, Rp] = x [R, C]^T zero-padded to Rp columns (16-bit dtypes; the per-step weight layouts)
Tensor transpose_pad(const Tensor& x, int64_t rows_out) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1 && x.element_size() == 2,
              "dlion transpose_pad: x must be a 2-D 16-bit GPU tensor with unit column stride");
  const int64_t R = x.size(0), C = x.size(1);
  const int64_t Rp = rows_out < 0 ? R : rows_out;
  TORCH_CHECK(Rp >= R && Rp % 8 == 0 && x.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "dlion transpose_pad: needs rows_out >= rows, rows_out % 8 == 0, row stride % 8 == 0, 16-byte alignment");
  const c10::DeviceGuard g(x.device());
  auto out = at::empty({C, Rp}, x.options());
  check_hip(dlion::launch_transpose_pad(x.data_ptr(), R, C, x.stride(0), out.data_ptr(), Rp, cur_stream()),
            "transpose_pad");
  return out;
}

// out [K, N] (a 2-D view, unit column stride, any row stride: e.g. a column block of a
// concatenated W^T) = W^T of the 4-bit W [N, K]
void dequant4_t_(const Tensor& q, const Tensor& absmax, const Tensor& code, const Tensor& out) {
  check_dev(q, "q");
  check_dev(absmax, "absmax");
  check_dev(code, "code");
  TORCH_CHECK(out.is_cuda() && out.dim() == 2 && out.stride(1) == 1 && out.element_size() == 2,
              "dlion dequant4_t: out must be a 2-D 16-bit GPU view with unit column stride");
  const int64_t K = out.size(0), N = out.size(1);
  TORCH_CHECK(q.scalar_type() == at::kByte && q.numel() * 2 == N * K && absmax.numel() * 64 == N * K &&
                  code.numel() == 16 && code.scalar_type() == at::kFloat,
              "dlion dequant4_t: q / absmax do not match out");
  const c10::DeviceGuard g(out.device());
  check_hip(dlion::launch_dequant4_t(dtype_code(out.scalar_type()), q.data_ptr<uint8_t>(), absmax.data_ptr<float>(),
                                     code.data_ptr<float>(), out.data_ptr(), static_cast<int>(N), static_cast<int>(K),
                                     out.stride(0), cur_stream()),
            "dequant4_t");
}
}  // namespace

TORCH_LIBRARY(dlion, m) {
  m.def("dequant4_t_(Tensor q, Tensor absmax, Tensor code, Tensor(a!) out) -> ()");
  m.def("transpose_pad(Tensor x, int rows_out=-1) -> Tensor");
  m.def("quant4(Tensor w, Tensor code) -> (Tensor, Tensor)");
  m.def("dequant4_(Tensor q, Tensor absmax, Tensor code, Tensor(a!) out) -> ()");
  m.def("gemm_tn(Tensor[] P, Tensor[] Q, int splits) -> Tensor");
  m.def("gemm_tn_(Tensor[] P, Tensor[] Q, Tensor(a!) out, bool accumulate) -> ()");
  m.def("lora_rows(Tensor x, Tensor w, float scale, float p, int seed) -> Tensor");
  m.def("lora_up(Tensor o, Tensor u, Tensor b, float s) -> Tensor");
  m.def("lora_cols(Tensor g, Tensor y, Tensor? a, float yscale, float p, int seed) -> (Tensor, Tensor)");
  m.def("gemm_nt_dgelu(Tensor a, Tensor b, Tensor bias, Tensor z, bool exact) -> (Tensor, Tensor)");
  m.def("gemm_nt_gelu_d(Tensor a, Tensor b, Tensor bias, bool exact) -> (Tensor, Tensor)");
  m.def("gemm_nt_dmul(Tensor a, Tensor b, Tensor d) -> (Tensor, Tensor)");
  m.def("gemm_nt_stamped(Tensor a, Tensor b, Tensor(a!) stamps) -> Tensor");
  m.def("embed_fwd(Tensor ids, Tensor wte, Tensor wpe, float p, int seed, Tensor(a!)? err=None) -> Tensor");
  m.def("index_check_(Tensor ids, int hi, int ignore, Tensor(a!) err, int code) -> ()");
  m.def(
      "embed_bwd_(Tensor dx, Tensor? sid, Tensor? perm, Tensor(a!)? dwte, Tensor(b!)? dwpe, int T, bool pos_accumulate,"
      " float p, int seed) -> ()");
  m.def("scale_acc_(Tensor x, Tensor s, Tensor(a!) y, bool accumulate) -> ()");
  m.def("lt_gemm_nt(Tensor a, Tensor b, Tensor? bias, int epi, Tensor(a!) out) -> bool");
  m.def("lt_gemm_nn(Tensor a, Tensor b, Tensor(a!) out) -> bool");
  m.def("lt_gemm_tn(Tensor a, Tensor b, Tensor(a!) out, bool accumulate) -> bool");
  m.def("lt_gemm_nt_acc(Tensor a, Tensor b, Tensor(a!) out, bool accumulate) -> bool");
  m.def("lt_gemm_layout(Tensor a, Tensor b, Tensor(a!) out, int layout, bool accumulate) -> bool");
  m.def("gemm_nt(Tensor a, Tensor b, Tensor? bias) -> Tensor");
  m.def("gemm_nt_out(Tensor a, Tensor b, Tensor? bias, Tensor(a!) out) -> ()");
  m.def("gemm_nt_gelu(Tensor a, Tensor b, Tensor bias, bool exact) -> (Tensor, Tensor)");
  m.def("swiglu_fwd(Tensor g, Tensor u) -> Tensor");
  m.def("swiglu_bwd(Tensor dh, Tensor g, Tensor u) -> (Tensor, Tensor)");
  m.def("swiglu_bwd_fused(Tensor dh, Tensor g, Tensor u) -> Tensor");
  m.def("swiglu_bwd_fused_t(Tensor dh, Tensor g, Tensor u) -> (Tensor, Tensor)");
  m.def("swiglu_fwd_t(Tensor g, Tensor u) -> (Tensor, Tensor)");
  m.def("rope(Tensor x, Tensor cos, Tensor sin, bool inverse) -> Tensor");
  m.def("rope_(Tensor(a!) x, Tensor cos, Tensor sin, bool inverse) -> ()");
  m.def(
      "add_norm_fwd(Tensor x, Tensor? y, Tensor? bias, Tensor gamma, Tensor? beta, float eps, bool rms, float p,"
      " int seed) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def(
      "add_norm_bwd(Tensor dh, Tensor? dxo_in, Tensor xo, Tensor gamma, Tensor mean, Tensor rstd, bool rms,"
      " float p, int seed, bool want_dy, int parts) -> (Tensor, Tensor, Tensor)");
  m.def("bias_gelu_fwd(Tensor z, Tensor b, bool exact) -> Tensor");
  m.def("bias_gelu_bwd(Tensor dh, Tensor z, Tensor b, bool exact, int parts) -> (Tensor, Tensor)");
  m.def("sum_partials(Tensor part) -> Tensor");
  m.def("sum_partials_acc_(Tensor part, Tensor(a!) out) -> ()");
  m.def("sum_partials_scaled_(Tensor part, Tensor s, Tensor(a!) out, bool accumulate) -> ()");
  m.def("sum_partials_multi_(Tensor[] parts, Tensor(a!) out, bool accumulate) -> ()");
  m.def("colsum_partials(Tensor x, int parts) -> Tensor");
  m.def("attn_fwd(Tensor q, Tensor k, Tensor v, float p, int seed, int window=0) -> (Tensor, Tensor)");
  m.def(
      "attn_bwd(Tensor q, Tensor k, Tensor v, Tensor out, Tensor dout, Tensor lse, float p, int seed,"
      " Tensor(a!) dq, Tensor(b!) dk, Tensor(c!) dv, Tensor(d!)? colsum=None, Tensor? rope_cos=None,"
      " Tensor? rope_sin=None, int window=0) -> ()");
  m.def("softmax_xent_(Tensor(a!) logits, Tensor labels, int v, int variant=0) -> Tensor");
  m.def(
      "lion_local(Tensor meta, int seg_off, int chunk_off, int n_chunks, int dtype, float decay, float neg_lr,"
      " float b1, float omb1, float b2, float omb2, Tensor? gscale=None) -> ()");
  m.def(
      "lion_encode(Tensor meta, int seg_off, int chunk_off, int n_chunks, int dtype, Tensor(a!) bits, float b1,"
      " float omb1, float b2, float omb2, bool update_m, bool stochastic, float rr, int seed, int step,"
      " Tensor? gscale=None) -> ()");
  m.def("grad_sumsq(Tensor meta, int seg_off, int chunk_off, int n_chunks, int dtype, Tensor(a!) partial,"
        " int part_off) -> ()");
  m.def("clip_coef(Tensor partial, int n, float max_norm, Tensor(a!) out) -> ()");
  m.def(
      "lion_vote_apply(Tensor meta, int seg_off, int chunk_off, int n_chunks, int dtype, Tensor planes,"
      " int plane_stride, Tensor alive, int mode, int tie, Tensor? neg, float decay, float neg_lr,"
      " Tensor? own, Tensor(b!)? agree) -> ()");
  m.def("vote_reduce(Tensor recv, int nbytes, Tensor alive, int tie, Tensor(a!) out, Tensor(b!)? neg_out,"
        " Tensor(c!)? ties=None) -> ()");
}

TORCH_LIBRARY_IMPL(dlion, CUDA, m) {
  m.impl("lion_local", &lion_local);
  m.impl("lion_encode", &lion_encode);
  m.impl("lion_vote_apply", &lion_vote_apply);
  m.impl("vote_reduce", &vote_reduce);
  m.impl("grad_sumsq", &grad_sumsq);
  m.impl("clip_coef", &clip_coef);
  m.impl("softmax_xent_", &softmax_xent_);
  m.impl("attn_fwd", &attn_fwd);
  m.impl("attn_bwd", &attn_bwd);
  m.impl("add_norm_fwd", &add_norm_fwd);
  m.impl("add_norm_bwd", &add_norm_bwd);
  m.impl("bias_gelu_fwd", &bias_gelu_fwd);
  m.impl("bias_gelu_bwd", &bias_gelu_bwd);
  m.impl("sum_partials", &sum_partials);
  m.impl("sum_partials_acc_", &sum_partials_acc_);
  m.impl("sum_partials_scaled_", &sum_partials_scaled_);
  m.impl("sum_partials_multi_", &sum_partials_multi_);
  m.impl("colsum_partials", &colsum_partials);
  m.impl("swiglu_fwd", &swiglu_fwd);
  m.impl("swiglu_bwd", &swiglu_bwd);
  m.impl("swiglu_bwd_fused", &swiglu_bwd_fused);
  m.impl("swiglu_bwd_fused_t", &swiglu_bwd_fused_t);
  m.impl("swiglu_fwd_t", &swiglu_fwd_t);
  m.impl("rope", &rope);
  m.impl("rope_", &rope_);
  m.impl("gemm_nt", &gemm_nt);
  m.impl("gemm_nt_out", &gemm_nt_out);
  m.impl("gemm_nt_gelu", &gemm_nt_gelu);
  m.impl("gemm_nt_dgelu", &gemm_nt_dgelu);
  m.impl("gemm_nt_gelu_d", &gemm_nt_gelu_d);
  m.impl("gemm_nt_dmul", &gemm_nt_dmul);
  m.impl("gemm_nt_stamped", &gemm_nt_stamped);
  m.impl("embed_fwd", &embed_fwd);
  m.impl("index_check_", &index_check_);
  m.impl("embed_bwd_", &embed_bwd_);
  m.impl("scale_acc_", &scale_acc_);
  m.impl("lt_gemm_nt", &lt_gemm_nt);
  m.impl("lt_gemm_nn", &lt_gemm_nn);
  m.impl("lt_gemm_tn", &lt_gemm_tn);
  m.impl("lt_gemm_nt_acc", &lt_gemm_nt_acc);
  m.impl("lt_gemm_layout", &lt_gemm_layout);
  m.impl("gemm_tn", &gemm_tn);
  m.impl("gemm_tn_", &gemm_tn_);
  m.impl("lora_rows", &lora_rows);
  m.impl("lora_up", &lora_up);
  m.impl("lora_cols", &lora_cols);
  m.impl("quant4", &quant4);
  m.impl("dequant4_", &dequant4_);
  m.impl("dequant4_t_", &dequant4_t_);
  m.impl("transpose_pad", &transpose_pad);
}
