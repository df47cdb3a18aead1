// LayerNorm / BatchNorm1d between the layers of the student MLP and of the SAGE
// teacher, each fused with the ReLU and dropout that follow it:
//   MLP.forward   h = dropout(relu(norm_l(Linear_l(h))))   src/models.py:45-54 (norms :27-37)
//   SAGE.forward  x = dropout(relu(norm_l(conv_l(x))))     src/models.py:110-119 (norms :90-101)
// nn.LayerNorm(H) normalises each row over its H features; nn.BatchNorm1d(H)
// normalises each column over the batch's rows (training: batch statistics and a
// momentum update of running_mean / running_var; eval: the running statistics).
//
// Layout: y (the layer's pre-norm output) and out (the post-ReLU/dropout
// activations) are row-major [M, H] with leading dimensions.  stats (f32) holds
// mean and 1/sqrt(var + eps): LayerNorm [2][M] (per row), BatchNorm [2][H] (per
// column).  Column sums (BatchNorm statistics, the backward's sum(g), sum(g*xhat),
// which are also dbeta / dgamma) are f64, reduced over fixed row chunks then over
// the chunks in order, so every call is deterministic and a caller can SUM-all-reduce
// the [2][H] totals across ranks between the sum and the apply (a batch split over
// ranks then normalises exactly as the whole batch on one device).
#include "llp_common.h"

#include <algorithm>
#include <math.h>

namespace {

constexpr int COLS = 256;      // columns per column-sum block (one per thread)
constexpr int MAX_CHUNKS = 128;

enum { LN = 1, BN = 2 };
enum { SUM_STATS = 0, SUM_BWD_ROW = 1, SUM_BWD_COL = 2 };

template <typename T>
__device__ __forceinline__ float ldv(const T* p, int64_t i) {
  if constexpr (sizeof(T) == 2) return bf2f(p[i]); else return p[i];
}
template <typename T>
__device__ __forceinline__ void stv(T* p, int64_t i, float v) {
  if constexpr (sizeof(T) == 2) p[i] = f2bf(v); else p[i] = v;
}

__device__ __forceinline__ int64_t live_rows(int64_t M, const int32_t* m_dev) {
  if (!m_dev) return M;
  const int64_t c = *m_dev;
  return c < M ? (c > 0 ? c : 0) : M;
}

// dropout(relu(v)) of element (r, c) of an [M, H] tensor: its keep draw (drop_keep) of the
// layer's Philox stream, as the GEMM epilogue and llp_act_2d draw
struct Drop {
  uint32_t thr;
  float scale;
  uint64_t seed;
  const int64_t* ctr;
  int64_t off;
};

__device__ __forceinline__ float relu_drop(float v, int relu, const Drop& d, uint64_t stream, int64_t r, int64_t c,
                                           int64_t H) {
  if (relu) v = fmaxf(v, 0.f);
  if (d.thr) v = drop_keep(d.thr, d.seed, stream, r, c, H) ? v * d.scale : 0.f;
  return v;
}

// the upstream gradient through ReLU / dropout: alpha * gout * (out > 0) (out NULL: no mask)
template <typename T>
__device__ __forceinline__ float grad_in(const T* gout, int64_t ldg, const T* out, int64_t ldo, float alpha,
                                         int64_t r, int64_t c) {
  float g = alpha * ldv<T>(gout, r * ldg + c);
  if (out && !(ldv<T>(out, r * ldo + c) > 0.f)) g = 0.f;
  return g;
}

// ---------------------------------------------------------------- column sums
// chunk blockIdx.y of the live rows, 256 columns per block; four rows in flight
//   SUM_STATS:   q0 = y, q1 = y*y                                   (BatchNorm statistics)
//   SUM_BWD_ROW: g = grad_in, xhat = (y - mean[r]) * rstd[r]; q0 = g, q1 = g*xhat   (LayerNorm)
//   SUM_BWD_COL: the same with the column's mean / rstd                             (BatchNorm)
template <typename T, int MODE>
__global__ __launch_bounds__(COLS) void colsum_partial_kernel(int64_t M, int64_t H, const T* __restrict__ y,
                                                              int64_t ldy, const T* __restrict__ gout, int64_t ldg,
                                                              const T* __restrict__ out, int64_t ldo, float alpha,
                                                              const float* __restrict__ stats,
                                                              const int32_t* __restrict__ m_dev,
                                                              double* __restrict__ part) {
  const int64_t c = (int64_t)blockIdx.x * COLS + threadIdx.x;
  const int64_t Ml = live_rows(M, m_dev);
  const int nch = gridDim.y, ch = blockIdx.y;
  const int64_t r0 = Ml * ch / nch, r1 = Ml * (ch + 1) / nch;
  if (c >= H) return;
  float cmean = 0.f, crstd = 0.f;
  if constexpr (MODE == SUM_BWD_COL) {
    cmean = stats[c];
    crstd = stats[H + c];
  }
  double s0 = 0.0, s1 = 0.0;
  auto term = [&](int64_t r) {
    if constexpr (MODE == SUM_STATS) {
      const double v = ldv<T>(y, r * ldy + c);
      s0 += v;
      s1 += v * v;
    } else {
      const float g = grad_in<T>(gout, ldg, out, ldo, alpha, r, c);
      float xh;
      if constexpr (MODE == SUM_BWD_ROW) xh = (ldv<T>(y, r * ldy + c) - stats[r]) * stats[M + r];
      else xh = (ldv<T>(y, r * ldy + c) - cmean) * crstd;
      s0 += (double)g;
      s1 += (double)g * (double)xh;
    }
  };
  int64_t r = r0;
  for (; r + 4 <= r1; r += 4) {
    term(r);
    term(r + 1);
    term(r + 2);
    term(r + 3);
  }
  for (; r < r1; ++r) term(r);
  part[((int64_t)ch * 2) * H + c] = s0;
  part[((int64_t)ch * 2 + 1) * H + c] = s1;
}

// totals over the chunks in order: sums[0:H] = sum q0, sums[H:2H] = sum q1; the backward
// also writes dgamma = sum g*xhat, dbeta = sum g (f32)
__global__ void colsum_final_kernel(int64_t H, int nch, const double* __restrict__ part, double* __restrict__ sums,
                                    float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= H) return;
  double t0 = 0.0, t1 = 0.0;
  for (int ch = 0; ch < nch; ++ch) {
    t0 += part[((int64_t)ch * 2) * H + c];
    t1 += part[((int64_t)ch * 2 + 1) * H + c];
  }
  sums[c] = t0;
  sums[H + c] = t1;
  if (dgamma) dgamma[c] = (float)t1;
  if (dbeta) dbeta[c] = (float)t0;
}

// ---------------------------------------------------------------- BatchNorm
// per column: batch statistics from the totals (training, with the running-stat
// momentum update, unbiased variance as torch) or the running statistics (eval)
__global__ void bn_stats_kernel(int64_t H, const double* __restrict__ sums, double count, float eps, float momentum,
                                int training, float* __restrict__ running_mean, float* __restrict__ running_var,
                                int64_t* __restrict__ num_batches_tracked, float* __restrict__ stats) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (training && c == 0 && num_batches_tracked) num_batches_tracked[0] += 1;
  if (c >= H) return;
  if (training) {
    const double mean = sums[c] / count;
    double var = sums[H + c] / count - mean * mean;
    var = var > 0.0 ? var : 0.0;
    stats[c] = (float)mean;
    stats[H + c] = (float)(1.0 / sqrt(var + (double)eps));
    if (running_mean) running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
    if (running_var) running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)(var * count / (count - 1.0));
  } else {
    stats[c] = running_mean[c];
    stats[H + c] = (float)(1.0 / sqrt((double)running_var[c] + (double)eps));
  }
}

// out = dropout(relu(y * a + b)), a = rstd * gamma, b = beta - mean * a (torch's per-channel form)
template <typename T>
__global__ void bn_apply_kernel(int64_t M, int64_t H, const T* __restrict__ y, int64_t ldy,
                                const float* __restrict__ stats, const float* __restrict__ gamma,
                                const float* __restrict__ beta, int relu, Drop d, T* __restrict__ out, int64_t ldo) {
  const uint64_t stream = d.ctr ? (uint64_t)(LLP_STREAMS_PER_STEP * (*d.ctr) + d.off) : 0;
  const int64_t n = M * H;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / H, c = i % H;
    const float a = stats[H + c] * (gamma ? gamma[c] : 1.f);
    const float b = (beta ? beta[c] : 0.f) - stats[c] * a;
    const float v = fmaf(ldv<T>(y, r * ldy + c), a, b);
    stv<T>(out, r * ldo + c, relu_drop(v, relu, d, stream, r, c, H));
  }
}

// gy = gamma * rstd * (g - sum(g)/n - xhat * sum(g*xhat)/n)
template <typename T>
__global__ void bn_bwd_kernel(int64_t M, int64_t H, const T* __restrict__ gout, int64_t ldg, const T* __restrict__ out,
                              int64_t ldo, float alpha, const T* __restrict__ y, int64_t ldy,
                              const float* __restrict__ gamma, const float* __restrict__ stats,
                              const double* __restrict__ sums, double count, T* __restrict__ gy, int64_t ldgy) {
  const int64_t n = M * H;
  const float inv_n = (float)(1.0 / count);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / H, c = i % H;
    const float rstd = stats[H + c];
    const float g = grad_in<T>(gout, ldg, out, ldo, alpha, r, c);
    const float xh = (ldv<T>(y, r * ldy + c) - stats[c]) * rstd;
    const float mg = (float)sums[c] * inv_n, mgx = (float)sums[H + c] * inv_n;
    stv<T>(gy, r * ldgy + c, (gamma ? gamma[c] : 1.f) * rstd * (g - mg - xh * mgx));
  }
}

// ---------------------------------------------------------------- LayerNorm
// one wave per row (4 per block): mean, then the centred second moment, both as f32
// lane sums in column order reduced across the wave; then the normalised row
template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int64_t M, int64_t H, const T* __restrict__ y, int64_t ldy,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float eps, float* __restrict__ stats,
                                                     const int32_t* __restrict__ m_dev, int relu, Drop d,
                                                     T* __restrict__ out, int64_t ldo) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= live_rows(M, m_dev)) return;
  const T* yr = y + r * ldy;
  float s = 0.f;
  for (int64_t c = lane; c < H; c += 64) s += ldv<T>(yr, c);
  const float mean = wave_sum(s) / (float)H;
  float q = 0.f;
  for (int64_t c = lane; c < H; c += 64) {
    const float t = ldv<T>(yr, c) - mean;
    q = fmaf(t, t, q);
  }
  const float var = wave_sum(q) / (float)H;
  const float rstd = 1.f / sqrtf(var + eps);
  if (lane == 0) {
    stats[r] = mean;
    stats[M + r] = rstd;
  }
  const uint64_t stream = d.ctr ? (uint64_t)(LLP_STREAMS_PER_STEP * (*d.ctr) + d.off) : 0;
  for (int64_t c = lane; c < H; c += 64) {
    float v = (ldv<T>(yr, c) - mean) * rstd;
    v = fmaf(v, gamma ? gamma[c] : 1.f, beta ? beta[c] : 0.f);
    stv<T>(out, r * ldo + c, relu_drop(v, relu, d, stream, r, c, H));
  }
}

// gy = rstd * (a - mean(a) - xhat * mean(a * xhat)), a = gamma * g
template <typename T>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int64_t M, int64_t H, const T* __restrict__ gout, int64_t ldg,
                                                     const T* __restrict__ out, int64_t ldo, float alpha,
                                                     const T* __restrict__ y, int64_t ldy,
                                                     const float* __restrict__ gamma, const float* __restrict__ stats,
                                                     const int32_t* __restrict__ m_dev, T* __restrict__ gy,
                                                     int64_t ldgy) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= live_rows(M, m_dev)) return;
  const float mean = stats[r], rstd = stats[M + r];
  float sa = 0.f, sax = 0.f;
  for (int64_t c = lane; c < H; c += 64) {
    const float a = grad_in<T>(gout, ldg, out, ldo, alpha, r, c) * (gamma ? gamma[c] : 1.f);
    const float xh = (ldv<T>(y, r * ldy + c) - mean) * rstd;
    sa += a;
    sax = fmaf(a, xh, sax);
  }
  const float ma = wave_sum(sa) / (float)H, max_ = wave_sum(sax) / (float)H;
  for (int64_t c = lane; c < H; c += 64) {
    const float a = grad_in<T>(gout, ldg, out, ldo, alpha, r, c) * (gamma ? gamma[c] : 1.f);
    const float xh = (ldv<T>(y, r * ldy + c) - mean) * rstd;
    stv<T>(gy, r * ldgy + c, rstd * (a - ma - xh * max_));
  }
}

unsigned grid_for(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 16384)); }

int chunks_for(int64_t M) { return (int)std::max<int64_t>(1, std::min<int64_t>(MAX_CHUNKS, M / 64)); }

int make_drop(const llp_dropout* dropout, Drop& d, const char* fn) {
  d = Drop{0u, 1.f, 0ull, nullptr, 0};
  if (dropout && dropout->p > 0.f) {
    LLP_CHECK_ARG(dropout->p < 1.f && dropout->step_ctr, "%s: dropout p in (0,1) needs step_ctr", fn);
    d.thr = llp::drop_code(dropout->p);
    d.scale = 1.f / (1.f - dropout->p);
    d.seed = dropout->seed;
    d.ctr = dropout->step_ctr;
    d.off = dropout->stream_offset;
  }
  return LLP_OK;
}

template <typename T, int MODE>
void launch_colsum(int64_t M, int64_t H, const void* y, int64_t ldy, const void* gout, int64_t ldg, const void* out,
                   int64_t ldo, float alpha, const float* stats, const int32_t* m_dev, double* sums, float* dgamma,
                   float* dbeta, void* ws, hipStream_t s) {
  const int nch = chunks_for(M);
  double* part = (double*)ws;
  hipLaunchKernelGGL((colsum_partial_kernel<T, MODE>), dim3(ceil_div_u(H, COLS), nch), dim3(COLS), 0, s, M, H,
                     (const T*)y, ldy, (const T*)gout, ldg, (const T*)out, ldo, alpha, stats, m_dev, part);
  hipLaunchKernelGGL(colsum_final_kernel, dim3(ceil_div_u(H, 256)), dim3(256), 0, s, H, nch, (const double*)part,
                     sums, dgamma, dbeta);
}

}  // namespace

extern "C" int64_t llp_norm_workspace_bytes(int64_t M, int64_t H) {
  return (int64_t)MAX_CHUNKS * 2 * std::max<int64_t>(H, 1) * (int64_t)sizeof(double) + 256;
}

extern "C" int llp_norm_colsums(int dtype, int64_t M, int64_t H, const void* y, int64_t ldy, const int32_t* m_dev,
                                double* sums, void* ws, void* stream) {
  LLP_CHECK_ARG((H == 0) || (sums && ws && (y || M == 0)), "llp_norm_colsums: null pointer");   // M = 0: zero sums
  LLP_CHECK_ARG(dtype == LLP_F32 || dtype == LLP_BF16, "llp_norm_colsums: dtype");
  if (H == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == LLP_BF16)
    launch_colsum<bf16_t, SUM_STATS>(M, H, y, ldy, nullptr, 0, nullptr, 0, 1.f, nullptr, m_dev, sums, nullptr,
                                     nullptr, ws, s);
  else
    launch_colsum<float, SUM_STATS>(M, H, y, ldy, nullptr, 0, nullptr, 0, 1.f, nullptr, m_dev, sums, nullptr, nullptr,
                                    ws, s);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_norm_fwd(int kind, int dtype, int64_t M, int64_t H, const void* y, int64_t ldy, const float* gamma,
                            const float* beta, float eps, int training, const double* sums, double count,
                            float momentum, float* running_mean, float* running_var, int64_t* num_batches_tracked,
                            float* stats, const int32_t* m_dev, int relu, const llp_dropout* dropout, void* out,
                            int64_t ldo, void* stream) {
  LLP_CHECK_ARG(kind == LN || kind == BN, "llp_norm_fwd: kind must be LLP_NORM_LAYER or LLP_NORM_BATCH");
  LLP_CHECK_ARG(dtype == LLP_F32 || dtype == LLP_BF16, "llp_norm_fwd: dtype");
  LLP_CHECK_ARG((M == 0 || H == 0) || (y && out && stats), "llp_norm_fwd: null pointer");
  Drop d;
  if (int e = make_drop(dropout, d, "llp_norm_fwd")) return e;
  if (M == 0 || H == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  if (kind == LN) {
    if (dtype == LLP_BF16)
      hipLaunchKernelGGL(ln_fwd_kernel<bf16_t>, dim3(ceil_div_u(M, 4)), dim3(256), 0, s, M, H, (const bf16_t*)y, ldy,
                         gamma, beta, eps, stats, m_dev, relu, d, (bf16_t*)out, ldo);
    else
      hipLaunchKernelGGL(ln_fwd_kernel<float>, dim3(ceil_div_u(M, 4)), dim3(256), 0, s, M, H, (const float*)y, ldy,
                         gamma, beta, eps, stats, m_dev, relu, d, (float*)out, ldo);
    LLP_LAUNCH_CHECK();
    return LLP_OK;
  }
  LLP_CHECK_ARG(!m_dev, "llp_norm_fwd: BatchNorm statistics need the host row count (no m_dev)");
  if (training) {
    LLP_CHECK_ARG(sums, "llp_norm_fwd: BatchNorm training needs the column sums (llp_norm_colsums)");
    LLP_CHECK_ARG(count > 1.0, "llp_norm_fwd: BatchNorm training needs more than 1 value per channel");
  } else {
    LLP_CHECK_ARG(running_mean && running_var, "llp_norm_fwd: BatchNorm eval needs the running statistics");
  }
  hipLaunchKernelGGL(bn_stats_kernel, dim3(ceil_div_u(H, 256)), dim3(256), 0, s, H, sums, count, eps, momentum,
                     training, running_mean, running_var, num_batches_tracked, stats);
  if (dtype == LLP_BF16)
    hipLaunchKernelGGL(bn_apply_kernel<bf16_t>, dim3(grid_for(M * H)), dim3(256), 0, s, M, H, (const bf16_t*)y, ldy,
                       (const float*)stats, gamma, beta, relu, d, (bf16_t*)out, ldo);
  else
    hipLaunchKernelGGL(bn_apply_kernel<float>, dim3(grid_for(M * H)), dim3(256), 0, s, M, H, (const float*)y, ldy,
                       (const float*)stats, gamma, beta, relu, d, (float*)out, ldo);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_norm_bwd_sums(int kind, int dtype, int64_t M, int64_t H, const void* gout, int64_t ldg,
                                 const void* out, int64_t ldo, float alpha, const void* y, int64_t ldy,
                                 const float* stats, const int32_t* m_dev, double* sums, float* dgamma, float* dbeta,
                                 void* ws, void* stream) {
  LLP_CHECK_ARG(kind == LN || kind == BN, "llp_norm_bwd_sums: kind");
  LLP_CHECK_ARG(dtype == LLP_F32 || dtype == LLP_BF16, "llp_norm_bwd_sums: dtype");
  LLP_CHECK_ARG((H == 0) || (sums && ws && (M == 0 || (gout && y && stats))), "llp_norm_bwd_sums: null pointer");
  LLP_CHECK_ARG(kind == LN || !m_dev, "llp_norm_bwd_sums: BatchNorm takes no device row count");
  if (H == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  if (kind == LN) {
    if (dtype == LLP_BF16)
      launch_colsum<bf16_t, SUM_BWD_ROW>(M, H, y, ldy, gout, ldg, out, ldo, alpha, stats, m_dev, sums, dgamma, dbeta,
                                         ws, s);
    else
      launch_colsum<float, SUM_BWD_ROW>(M, H, y, ldy, gout, ldg, out, ldo, alpha, stats, m_dev, sums, dgamma, dbeta,
                                        ws, s);
  } else {
    if (dtype == LLP_BF16)
      launch_colsum<bf16_t, SUM_BWD_COL>(M, H, y, ldy, gout, ldg, out, ldo, alpha, stats, nullptr, sums, dgamma,
                                         dbeta, ws, s);
    else
      launch_colsum<float, SUM_BWD_COL>(M, H, y, ldy, gout, ldg, out, ldo, alpha, stats, nullptr, sums, dgamma, dbeta,
                                        ws, s);
  }
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_norm_bwd(int kind, int dtype, int64_t M, int64_t H, const void* gout, int64_t ldg, const void* out,
                            int64_t ldo, float alpha, const void* y, int64_t ldy, const float* gamma,
                            const float* stats, const double* sums, double count, const int32_t* m_dev, void* gy,
                            int64_t ldgy, void* stream) {
  LLP_CHECK_ARG(kind == LN || kind == BN, "llp_norm_bwd: kind");
  LLP_CHECK_ARG(dtype == LLP_F32 || dtype == LLP_BF16, "llp_norm_bwd: dtype");
  LLP_CHECK_ARG((M == 0 || H == 0) || (gout && y && stats && gy), "llp_norm_bwd: null pointer");
  if (M == 0 || H == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  if (kind == LN) {
    if (dtype == LLP_BF16)
      hipLaunchKernelGGL(ln_bwd_kernel<bf16_t>, dim3(ceil_div_u(M, 4)), dim3(256), 0, s, M, H, (const bf16_t*)gout, ldg,
                         (const bf16_t*)out, ldo, alpha, (const bf16_t*)y, ldy, gamma, stats, m_dev, (bf16_t*)gy, ldgy);
    else
      hipLaunchKernelGGL(ln_bwd_kernel<float>, dim3(ceil_div_u(M, 4)), dim3(256), 0, s, M, H, (const float*)gout, ldg,
                         (const float*)out, ldo, alpha, (const float*)y, ldy, gamma, stats, m_dev, (float*)gy, ldgy);
  } else {
    LLP_CHECK_ARG(sums && count > 0.0 && !m_dev, "llp_norm_bwd: BatchNorm needs the column sums and the row count");
    if (dtype == LLP_BF16)
      hipLaunchKernelGGL(bn_bwd_kernel<bf16_t>, dim3(grid_for(M * H)), dim3(256), 0, s, M, H, (const bf16_t*)gout, ldg,
                         (const bf16_t*)out, ldo, alpha, (const bf16_t*)y, ldy, gamma, stats, sums, count,
                         (bf16_t*)gy, ldgy);
    else
      hipLaunchKernelGGL(bn_bwd_kernel<float>, dim3(grid_for(M * H)), dim3(256), 0, s, M, H, (const float*)gout, ldg,
                         (const float*)out, ldo, alpha, (const float*)y, ldy, gamma, stats, sums, count, (float*)gy,
                         ldgy);
  }
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}
