// Small elementwise kernels behind the module-level autograd ops (llp_ops.py):
// ReLU/dropout backward, transpose, products, sigmoid backward.
#include "llp_common.h"

namespace {

template <typename T>
__device__ __forceinline__ float ldv(const T* p, int64_t i) {
  if constexpr (sizeof(T) == 2) return bf2f(p[i]); else return p[i];
}
template <typename T>
__device__ __forceinline__ void stv(T* p, int64_t i, float v) {
  if constexpr (sizeof(T) == 2) p[i] = f2bf(v); else p[i] = v;
}

template <typename T>
__global__ void relu_bwd_kernel(int64_t n, int64_t cols, const T* __restrict__ gy, const T* __restrict__ y,
                                float alpha, T* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float g = alpha * ldv<T>(gy, i);
    if (y && !(ldv<T>(y, i) > 0.f)) g = 0.f;
    stv<T>(out, i, g);
  }
}

template <typename T>
__global__ void transpose_kernel(int64_t rows, int64_t cols, const T* __restrict__ src, T* __restrict__ dst) {
  __shared__ float tile[32][33];
  const int64_t c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  for (int i = threadIdx.y; i < 32; i += blockDim.y) {
    const int64_t r = r0 + i, c = c0 + threadIdx.x;
    tile[i][threadIdx.x] = (r < rows && c < cols) ? ldv<T>(src, r * cols + c) : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.y; i < 32; i += blockDim.y) {
    const int64_t c = c0 + i, r = r0 + threadIdx.x;
    if (r < rows && c < cols) stv<T>(dst, c * rows + r, tile[threadIdx.x][i]);
  }
}

template <typename T>
__global__ void mul_kernel(int64_t n, const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    stv<T>(out, i, ldv<T>(a, i) * ldv<T>(b, i));
}

template <typename T>
__global__ void row_scale_kernel(int64_t rows, int64_t cols, const T* __restrict__ z, const float* __restrict__ s,
                                 T* __restrict__ out) {
  const int64_t n = rows * cols;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    stv<T>(out, i, ldv<T>(z, i) * s[i / cols]);
}

__global__ void sigmoid_bwd_kernel(int64_t n, const float* __restrict__ gprob, const float* __restrict__ prob,
                                   float* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) {
    const float p = prob[i];
    out[i] = gprob[i] * (1.f - p) * p;   // torch sigmoid_backward: grad * (1 - y) * y
  }
}

unsigned grid_for(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 16384)); }

// y = dropout(relu(x)) on a strided [rows, cols] view; the keep draw of element (r, c)
// (drop_keep) of Philox stream LLP_STREAMS_PER_STEP*(*ctr) + stream_off, as the GEMM
// epilogue draws.
template <typename T>
__global__ void act_2d_kernel(int64_t rows, int64_t cols, const T* __restrict__ x, int64_t ldx, T* __restrict__ y,
                              int64_t ldy, int relu, uint32_t thr, float scale, uint64_t seed,
                              const int64_t* __restrict__ ctr, int64_t stream_off) {
  const int64_t n = rows * cols;
  const uint64_t stream = ctr ? (uint64_t)(LLP_STREAMS_PER_STEP * (*ctr) + stream_off) : 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cols, c = i % cols;
    float v = ldv<T>(x, r * ldx + c);
    // torch.relu propagates NaN (fmaxf would turn it into 0); bf16 follows the 256-tile GEMM
    // epilogues' sign-bit rule (a -NaN becomes 0 there)
    if (relu) v = sizeof(T) == 2 ? (__float_as_int(v) < 0 ? 0.f : v) : (v < 0.f ? 0.f : v);
    if (thr) v = drop_keep(thr, seed, stream, r, c, cols) ? v * scale : 0.f;
    stv<T>(y, r * ldy + c, v);
  }
}

template <typename T>
__global__ void relu_bwd_2d_kernel(int64_t rows, int64_t cols, const T* __restrict__ gy, int64_t ldg,
                                   const T* __restrict__ y, int64_t ldy, float alpha, T* __restrict__ out,
                                   int64_t ldo) {
  const int64_t n = rows * cols;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cols, c = i % cols;
    float g = alpha * ldv<T>(gy, r * ldg + c);
    if (!(ldv<T>(y, r * ldy + c) > 0.f)) g = 0.f;
    stv<T>(out, r * ldo + c, g);
  }
}

}  // namespace

extern "C" int llp_act_2d(int dtype, int64_t rows, int64_t cols, const void* x, int64_t ldx, void* y, int64_t ldy,
                          int act, const llp_dropout* dropout, void* stream) {
  LLP_CHECK_ARG((rows == 0 || cols == 0) || (x && y), "llp_act_2d: null pointer");
  LLP_CHECK_ARG(act == LLP_ACT_NONE || act == LLP_ACT_RELU, "llp_act_2d: act must be NONE or RELU");
  if (rows == 0 || cols == 0) return LLP_OK;
  uint32_t thr = 0;
  float scale = 1.f;
  uint64_t seed = 0;
  const int64_t* ctr = nullptr;
  int64_t off = 0;
  if (dropout && dropout->p > 0.f) {
    LLP_CHECK_ARG(dropout->p < 1.f && dropout->step_ctr, "llp_act_2d: dropout p in (0,1) needs step_ctr");
    thr = llp::drop_code(dropout->p);
    scale = 1.f / (1.f - dropout->p);
    seed = dropout->seed;
    ctr = dropout->step_ctr;
    off = dropout->stream_offset;
  }
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = rows * cols;
  if (dtype == LLP_BF16)
    hipLaunchKernelGGL(act_2d_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, s, rows, cols, (const bf16_t*)x, ldx,
                       (bf16_t*)y, ldy, act == LLP_ACT_RELU, thr, scale, seed, ctr, off);
  else
    hipLaunchKernelGGL(act_2d_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, rows, cols, (const float*)x, ldx,
                       (float*)y, ldy, act == LLP_ACT_RELU, thr, scale, seed, ctr, off);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_relu_bwd_2d(int dtype, int64_t rows, int64_t cols, const void* gy, int64_t ldg, const void* y,
                               int64_t ldy, float alpha, void* out, int64_t ldo, void* stream) {
  LLP_CHECK_ARG((rows == 0 || cols == 0) || (gy && y && out), "llp_relu_bwd_2d: null pointer");
  if (rows == 0 || cols == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = rows * cols;
  if (dtype == LLP_BF16)
    hipLaunchKernelGGL(relu_bwd_2d_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, s, rows, cols, (const bf16_t*)gy,
                       ldg, (const bf16_t*)y, ldy, alpha, (bf16_t*)out, ldo);
  else
    hipLaunchKernelGGL(relu_bwd_2d_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, rows, cols, (const float*)gy,
                       ldg, (const float*)y, ldy, alpha, (float*)out, ldo);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_relu_bwd(int dtype, int64_t n, const void* gy, const void* y, float alpha, void* out,
                            void* stream) {
  LLP_CHECK_ARG((n == 0) || (gy && out), "llp_relu_bwd: null pointer");
  if (n == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == LLP_BF16)
    hipLaunchKernelGGL(relu_bwd_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, s, n, (int64_t)0, (const bf16_t*)gy,
                       (const bf16_t*)y, alpha, (bf16_t*)out);
  else
    hipLaunchKernelGGL(relu_bwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, n, (int64_t)0, (const float*)gy,
                       (const float*)y, alpha, (float*)out);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_transpose(int dtype, int64_t rows, int64_t cols, const void* src, void* dst, void* stream) {
  LLP_CHECK_ARG((rows == 0 || cols == 0) || (src && dst), "llp_transpose: null pointer");
  if (rows == 0 || cols == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(ceil_div_u(cols, 32), ceil_div_u(rows, 32));
  if (dtype == LLP_BF16)
    hipLaunchKernelGGL(transpose_kernel<bf16_t>, grid, dim3(32, 8), 0, s, rows, cols, (const bf16_t*)src,
                       (bf16_t*)dst);
  else
    hipLaunchKernelGGL(transpose_kernel<float>, grid, dim3(32, 8), 0, s, rows, cols, (const float*)src, (float*)dst);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_mul(int dtype, int64_t n, const void* a, const void* b, void* out, void* stream) {
  LLP_CHECK_ARG(a && b && out, "llp_mul: null pointer");
  if (n == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == LLP_BF16)
    hipLaunchKernelGGL(mul_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, s, n, (const bf16_t*)a, (const bf16_t*)b,
                       (bf16_t*)out);
  else
    hipLaunchKernelGGL(mul_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, n, (const float*)a, (const float*)b,
                       (float*)out);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_row_scale(int dtype, int64_t rows, int64_t cols, const void* z, const float* sc, void* out,
                             void* stream) {
  LLP_CHECK_ARG((rows * cols == 0) || (z && sc && out), "llp_row_scale: null pointer");
  if (rows * cols == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == LLP_BF16)
    hipLaunchKernelGGL(row_scale_kernel<bf16_t>, dim3(grid_for(rows * cols)), dim3(256), 0, s, rows, cols,
                       (const bf16_t*)z, sc, (bf16_t*)out);
  else
    hipLaunchKernelGGL(row_scale_kernel<float>, dim3(grid_for(rows * cols)), dim3(256), 0, s, rows, cols,
                       (const float*)z, sc, (float*)out);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_sigmoid_bwd(int64_t n, const float* gprob, const float* prob, float* out, void* stream) {
  LLP_CHECK_ARG(gprob && prob && out, "llp_sigmoid_bwd: null pointer");
  if (n == 0) return LLP_OK;
  hipLaunchKernelGGL(sigmoid_bwd_kernel, dim3(ceil_div_u(n, 256)), dim3(256), 0, (hipStream_t)stream, n, gprob, prob,
                     out);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}
