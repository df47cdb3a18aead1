// Sparse-input first student layer: nn.Linear(F, H) over bag-of-words node features
// (src/models.py:48, the MLP student's first layer on x; coauthor-physics' 8,415 binary keyword
// features are ~0.5 % nonzero, ~40 per node).  x is constant over training, so the engine keeps
// it once as CSR (rows = nodes) and, per student slice, CSC (rows = features); the first layer
// then gathers rows of the bf16 transposed weight shadow Wt [F, H] (L2 / MALL resident, 4.3 MB
// at the physics shape) instead of streaming the dense [N, 8,448] bf16 x through MFMA tiles
// whose products are 99.5 % zero.
//
//   forward   Y[r, :]  = act(sum_{k in row r} val[k] * Wt[col[k], :] + bias)      (f32 sums)
//   backward  dW[o, f] (+)= sum_{k in column f} val[k] * dY[row[k], o]            (f32 sums)
//
// Both sum in a fixed order (interleaved streams of the index order, then a butterfly; below):
// deterministic, equal to the dense GEMM's f32 sums up to their order.  The forward's epilogue is the GEMMs': bias add,
// bf16 round (RNE), ReLU by the sign bit, the ReLU bit mask (bit i of byte c = column 8c + i
// nonzero) that the ReLU-backward GEMM of the next layer reads.  HBM: the CSR / CSC indices
// (4 B per nonzero, +4 with values), Y or dW once; the gathered rows come from cache.
#include "llp_common.h"
#include "llp_hip.h"

namespace {

// Both kernels read 16 B per lane (8 bf16 or 4 f32 values: E = 16 / sizeof(T)) and split a row
// of the gathered matrix into column slices: a workgroup works on one slice, chosen by blockIdx
// % slices.  Workgroups go to the 8 XCDs round-robin (blockIdx % 8), so each XCD only ever
// gathers its own slices' columns: half of W^T (2.15 MB at 8,415 x 256 bf16) or a quarter of dY
// stays resident in that XCD's 4 MB L2, where the whole 4.3 MB W^T would not.  Within a wave,
// lanes are (stream, E-column chunk): the streams take interleaved nonzeros (k = first + stream +
// streams * i) so that a row with few nonzeros still has many gathers in flight, and they are
// summed in a fixed butterfly.  The f32 instantiation (round 6) serves the fp32 engine, whose
// arithmetic is the reference's own: the same order of sums, f32 rows in and out.

template <typename T>
struct Vec16 {
  static constexpr int E = 16 / sizeof(T);
};

__device__ __forceinline__ void fma16(float* acc, uint4 w, float v, bf16_t) {
  acc[0] = fmaf(v, __uint_as_float(w.x << 16), acc[0]);
  acc[1] = fmaf(v, __uint_as_float(w.x & 0xFFFF0000u), acc[1]);
  acc[2] = fmaf(v, __uint_as_float(w.y << 16), acc[2]);
  acc[3] = fmaf(v, __uint_as_float(w.y & 0xFFFF0000u), acc[3]);
  acc[4] = fmaf(v, __uint_as_float(w.z << 16), acc[4]);
  acc[5] = fmaf(v, __uint_as_float(w.z & 0xFFFF0000u), acc[5]);
  acc[6] = fmaf(v, __uint_as_float(w.w << 16), acc[6]);
  acc[7] = fmaf(v, __uint_as_float(w.w & 0xFFFF0000u), acc[7]);
}
__device__ __forceinline__ void fma16(float* acc, uint4 w, float v, float) {
  acc[0] = fmaf(v, __uint_as_float(w.x), acc[0]);
  acc[1] = fmaf(v, __uint_as_float(w.y), acc[1]);
  acc[2] = fmaf(v, __uint_as_float(w.z), acc[2]);
  acc[3] = fmaf(v, __uint_as_float(w.w), acc[3]);
}

__device__ __forceinline__ uint16_t relu_bf(uint16_t b) { return (b & 0x8000u) ? (uint16_t)0 : b; }

// sum of `streams` nonzero streams of [first, last): stream s (this lane's) takes first + s,
// first + s + streams, ..; U gathers of 16 B each in flight
template <int U, typename T>
__device__ __forceinline__ void gather_sum(float* acc, const int32_t* __restrict__ idx, const float* __restrict__ val,
                                           const T* __restrict__ M, int64_t ldm, int64_t col, bool live,
                                           int32_t first, int32_t last, int s, int streams) {
  constexpr int E = Vec16<T>::E;
#pragma unroll
  for (int i = 0; i < E; ++i) acc[i] = 0.f;
  int32_t k = first + s;
  const int64_t colc = live ? col : 0;
  for (; k + streams * (U - 1) < last; k += streams * U) {
    uint4 g[U];
    float v[U];
    int32_t r[U];
#ifndef LLP_SPMM_INTERLEAVED
    // all U indices (and values) first, then the U row loads: interleaved per u, each row load
    // waited for the previous one (the vector-memory counter is in order, and the next index was
    // issued behind it), so one row was in flight per lane instead of U (round 6)
    // (no branch between the loads: a dead lane reads its row's column 0 and adds nothing, and
    // the values' presence is uniform)
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = idx[k + streams * u];
    if (val) {
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = val[k + streams * u];
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = 1.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) g[u] = *reinterpret_cast<const uint4*>(M + (int64_t)r[u] * ldm + colc);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (live) fma16(acc, g[u], v[u], T());
    continue;
#else
#pragma unroll
    for (int u = 0; u < U; ++u) {
      r[u] = idx[k + streams * u];
      v[u] = val ? val[k + streams * u] : 1.f;
      g[u] = live ? *reinterpret_cast<const uint4*>(M + (int64_t)r[u] * ldm + col) : make_uint4(0u, 0u, 0u, 0u);
    }
#endif
#pragma unroll
    for (int u = 0; u < U; ++u) fma16(acc, g[u], v[u], T());
  }
  for (; k < last; k += streams) {
    const int64_t r = idx[k];
    const float v = val ? val[k] : 1.f;
    if (live) fma16(acc, *reinterpret_cast<const uint4*>(M + r * ldm + col), v, T());
  }
}

// forward: slices of 16 E columns (16 lanes x E); one row per wave, 4 streams of its nonzeros;
// four rows per workgroup.  Workgroup b: slice b % S, rows 4 (b / S) ..
template <typename T>
__global__ __launch_bounds__(256) void spmm_rows_kernel(int64_t rows, int64_t row0, int64_t H, int S,
                                                        const int32_t* __restrict__ rowptr,
                                                        const int32_t* __restrict__ colidx,
                                                        const float* __restrict__ val, const T* __restrict__ Wt,
                                                        int64_t ldw, const float* __restrict__ bias, int relu,
                                                        T* __restrict__ Y, int64_t ldy,
                                                        uint8_t* __restrict__ mask, int64_t ld_mask) {
  constexpr int E = Vec16<T>::E;
  const int slice = blockIdx.x % S;
  const int64_t r = (int64_t)(blockIdx.x / S) * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int lane = threadIdx.x & 63, st = lane >> 4, cl = lane & 15;
  const int64_t col = (int64_t)slice * (16 * E) + E * cl;
  const bool live = col < H;
  float acc[E];
  gather_sum<4>(acc, colidx, val, Wt, ldw, col, live, rowptr[row0 + r], rowptr[row0 + r + 1], st, 4);
#pragma unroll
  for (int i = 0; i < E; ++i) {   // ((s0 + s1) + (s2 + s3))
    acc[i] += __shfl_xor(acc[i], 16, 64);
    acc[i] += __shfl_xor(acc[i], 32, 64);
  }
  if (st != 0 || !live) return;
  if constexpr (sizeof(T) == 2) {
    uint32_t byte = 0, w[4];
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      uint16_t b0 = f2bf(acc[i] + (bias ? bias[col + i] : 0.f));
      uint16_t b1 = f2bf(acc[i + 1] + (bias ? bias[col + i + 1] : 0.f));
      if (relu) { b0 = relu_bf(b0); b1 = relu_bf(b1); }
      byte |= (b0 ? 1u : 0u) << i | (b1 ? 1u : 0u) << (i + 1);
      w[i / 2] = (uint32_t)b0 | ((uint32_t)b1 << 16);
    }
    *reinterpret_cast<uint4*>(Y + r * ldy + col) = make_uint4(w[0], w[1], w[2], w[3]);
    if (mask) mask[r * ld_mask + col / 8] = (uint8_t)byte;
  } else {
    float y[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      y[i] = acc[i] + (bias ? bias[col + i] : 0.f);
      if (relu) y[i] = y[i] < 0.f ? 0.f : y[i];   // torch.relu: a NaN stays NaN (the f32 GEMM epilogue's rule)
    }
    *reinterpret_cast<float4_t*>(Y + r * ldy + col) = float4_t{y[0], y[1], y[2], y[3]};
  }
}

// backward: slices of 8 E columns (8 lanes x E), features in the order perm (most nonzeros
// first).  The first n_heavy features (>= LLP_SPMM_HEAVY_NNZ nonzeros) take a workgroup each,
// every wave a contiguous quarter of the nonzeros; the rest take a wave each, four per
// workgroup.  A wave sums 8 interleaved streams; order: the butterfly
// (((s0+s1)+(s2+s3))+((s4+s5)+(s6+s7))), then for a heavy feature ((q0+q1)+(q2+q3)).
// Workgroup b: slice b % S, work item b / S.
constexpr int SPMM_HEAVY_NNZ = 128;

template <typename T>
__global__ __launch_bounds__(256) void spmm_tn_kernel(int64_t F, int64_t H, int S, const int32_t* __restrict__ colptr,
                                                      const int32_t* __restrict__ rowidx,
                                                      const float* __restrict__ val, const int32_t* __restrict__ perm,
                                                      int64_t n_heavy, const T* __restrict__ dY, int64_t ldy,
                                                      float* __restrict__ dW, int64_t ldw, int accumulate) {
  constexpr int E = Vec16<T>::E;
  constexpr int BW_COLS = 8 * E;
  __shared__ float part[4][BW_COLS];
  const int slice = blockIdx.x % S;
  const int64_t item = blockIdx.x / S;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, st = lane >> 3, cl = lane & 7;
  const int64_t col = (int64_t)slice * BW_COLS + E * cl;
  const bool live = col < H;
  const bool heavy = item < n_heavy;
  const int64_t fi = heavy ? item : n_heavy + 4 * (item - n_heavy) + wv;
  if (fi >= F) return;   // light workgroups only: their waves never meet at a barrier
  const int64_t f = perm[fi];
  const int32_t kb = colptr[f], n = colptr[f + 1] - kb;
  const int32_t first = heavy ? kb + (int32_t)((int64_t)n * wv / 4) : kb;
  const int32_t last = heavy ? kb + (int32_t)((int64_t)n * (wv + 1) / 4) : kb + n;
  float acc[E];
  gather_sum<4>(acc, rowidx, val, dY, ldy, col, live, first, last, st, 8);
#pragma unroll
  for (int i = 0; i < E; ++i) {
    acc[i] += __shfl_xor(acc[i], 8, 64);
    acc[i] += __shfl_xor(acc[i], 16, 64);
    acc[i] += __shfl_xor(acc[i], 32, 64);
  }
  if (!heavy) {   // this wave's feature, its BW_COLS columns: lanes 0..7 of stream 0 hold them
    if (st == 0 && live) {
#pragma unroll
      for (int i = 0; i < E; ++i) {
        float* dst = dW + (col + i) * ldw + f;
        *dst = accumulate ? *dst + acc[i] : acc[i];
      }
    }
    return;
  }
  if (st == 0) {
#pragma unroll
    for (int i = 0; i < E; ++i) part[wv][E * cl + i] = acc[i];
  }
  __syncthreads();
  if (threadIdx.x < BW_COLS) {
    const int64_t o = (int64_t)slice * BW_COLS + threadIdx.x;
    if (o < H) {
      const int c = threadIdx.x;
      const float x = (part[0][c] + part[1][c]) + (part[2][c] + part[3][c]);
      float* dst = dW + o * ldw + f;
      *dst = accumulate ? *dst + x : x;
    }
  }
}

}  // namespace

extern "C" int llp_spmm_rows_dt(int dtype, int64_t rows, int64_t row0, int64_t H, const int32_t* rowptr,
                                const int32_t* colidx, const float* val, const void* Wt, int64_t ldw,
                                const float* bias, int act, void* Y, int64_t ldy, void* mask_out, int64_t ld_mask,
                                void* stream) {
  LLP_CHECK_ARG(dtype == LLP_BF16 || dtype == LLP_F32, "llp_spmm_rows: dtype must be BF16 or F32");
  const int E = dtype == LLP_BF16 ? 8 : 4;
  LLP_CHECK_ARG(rows >= 0 && row0 >= 0 && H > 0 && H <= 4096 && H % 8 == 0,
                "llp_spmm_rows: rows >= 0, row0 >= 0, H in [8, 4096] with H %% 8 == 0 (rows=%lld row0=%lld H=%lld)",
                (long long)rows, (long long)row0, (long long)H);
  LLP_CHECK_ARG(act == LLP_ACT_NONE || act == LLP_ACT_RELU, "llp_spmm_rows: act must be NONE or RELU");
  LLP_CHECK_ARG(!mask_out || act == LLP_ACT_RELU, "llp_spmm_rows: a ReLU mask needs act RELU");
  LLP_CHECK_ARG(!mask_out || dtype == LLP_BF16, "llp_spmm_rows: the ReLU bit mask is written by the bf16 form only");
  if (rows == 0) return LLP_OK;
  LLP_CHECK_ARG(rowptr && colidx && Wt && Y && (!mask_out || ld_mask >= H / 8), "llp_spmm_rows: null pointer / ld_mask");
  LLP_CHECK_ARG((uintptr_t)Wt % 16 == 0 && ldw % E == 0 && ldw >= H && (uintptr_t)Y % 16 == 0 && ldy % E == 0 &&
                    ldy >= H,
                "llp_spmm_rows: Wt and Y need 16-B aligned rows (ldw, ldy multiples of 16 B, >= H)");
  const int cols = 16 * E;
  const int S = (int)((H + cols - 1) / cols);
  const int64_t blocks = ((rows + 3) / 4) * S;
  LLP_CHECK_ARG(blocks < (1ll << 31), "llp_spmm_rows: too many rows");
  const int relu = act == LLP_ACT_RELU ? 1 : 0;
  if (dtype == LLP_BF16)
    hipLaunchKernelGGL(spmm_rows_kernel<bf16_t>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, rows, row0,
                       H, S, rowptr, colidx, val, (const bf16_t*)Wt, ldw, bias, relu, (bf16_t*)Y, ldy,
                       (uint8_t*)mask_out, ld_mask);
  else
    hipLaunchKernelGGL(spmm_rows_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, rows, row0,
                       H, S, rowptr, colidx, val, (const float*)Wt, ldw, bias, relu, (float*)Y, ldy, nullptr,
                       (int64_t)0);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_spmm_rows(int64_t rows, int64_t row0, int64_t H, const int32_t* rowptr, const int32_t* colidx,
                             const float* val, const void* Wt, int64_t ldw, const float* bias, int act, void* Y,
                             int64_t ldy, void* mask_out, int64_t ld_mask, void* stream) {
  return llp_spmm_rows_dt(LLP_BF16, rows, row0, H, rowptr, colidx, val, Wt, ldw, bias, act, Y, ldy, mask_out, ld_mask,
                          stream);
}

extern "C" int llp_spmm_heavy_nnz(void) { return SPMM_HEAVY_NNZ; }

extern "C" int llp_spmm_tn_dt(int dtype, int64_t F, int64_t H, const int32_t* colptr, const int32_t* rowidx,
                              const float* val, const int32_t* perm, int64_t n_heavy, const void* dY, int64_t ldy,
                              float* dW, int64_t ldw, int accumulate, void* stream) {
  LLP_CHECK_ARG(dtype == LLP_BF16 || dtype == LLP_F32, "llp_spmm_tn: dtype must be BF16 or F32");
  const int E = dtype == LLP_BF16 ? 8 : 4;
  LLP_CHECK_ARG(F >= 0 && H > 0 && H <= 4096 && H % 8 == 0,
                "llp_spmm_tn: F >= 0, H in [8, 4096] with H %% 8 == 0 (F=%lld H=%lld)", (long long)F, (long long)H);
  if (F == 0) return LLP_OK;
  LLP_CHECK_ARG(colptr && rowidx && perm && dY && dW && ldw >= F, "llp_spmm_tn: null pointer / ldw < F");
  LLP_CHECK_ARG(n_heavy >= 0 && n_heavy <= F, "llp_spmm_tn: n_heavy %lld not in [0, F]", (long long)n_heavy);
  LLP_CHECK_ARG((uintptr_t)dY % 16 == 0 && ldy % E == 0 && ldy >= H, "llp_spmm_tn: dY needs 16-B aligned rows");
  const int cols = 8 * E;
  const int S = (int)((H + cols - 1) / cols);
  const int64_t items = n_heavy + (F - n_heavy + 3) / 4;
  LLP_CHECK_ARG(items * S < (1ll << 31), "llp_spmm_tn: too many features");
  if (dtype == LLP_BF16)
    hipLaunchKernelGGL(spmm_tn_kernel<bf16_t>, dim3((unsigned)(items * S)), dim3(256), 0, (hipStream_t)stream, F, H, S,
                       colptr, rowidx, val, perm, n_heavy, (const bf16_t*)dY, ldy, dW, ldw, accumulate);
  else
    hipLaunchKernelGGL(spmm_tn_kernel<float>, dim3((unsigned)(items * S)), dim3(256), 0, (hipStream_t)stream, F, H, S,
                       colptr, rowidx, val, perm, n_heavy, (const float*)dY, ldy, dW, ldw, accumulate);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_spmm_tn(int64_t F, int64_t H, const int32_t* colptr, const int32_t* rowidx, const float* val,
                           const int32_t* perm, int64_t n_heavy, const void* dY, int64_t ldy, float* dW, int64_t ldw,
                           int accumulate, void* stream) {
  return llp_spmm_tn_dt(LLP_BF16, F, H, colptr, rowidx, val, perm, n_heavy, dY, ldy, dW, ldw, accumulate, stream);
}
