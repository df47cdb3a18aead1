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
// Both sum in index order (CSR: ascending feature, CSC: ascending row): deterministic, equal to
// the dense GEMM's f32 sums up to their order.  The forward's epilogue is the GEMMs': bias add,
// bf16 round (RNE), ReLU by the sign bit, the ReLU bit mask (bit i of byte c = column 8c + i
// nonzero) that the ReLU-backward GEMM of the next layer reads.  HBM: the CSR / CSC indices
// (4 B per nonzero, +4 with values), Y or dW once; the gathered rows come from cache.
#include "llp_common.h"
#include "llp_hip.h"

namespace {

constexpr int SP_UNROLL = 8;   // nonzeros whose gathers are in flight together

__device__ __forceinline__ void bf4_fma(float* acc, uint2 w, float v) {
  acc[0] = fmaf(v, __uint_as_float(w.x << 16), acc[0]);
  acc[1] = fmaf(v, __uint_as_float(w.x & 0xFFFF0000u), acc[1]);
  acc[2] = fmaf(v, __uint_as_float(w.y << 16), acc[2]);
  acc[3] = fmaf(v, __uint_as_float(w.y & 0xFFFF0000u), acc[3]);
}

__device__ __forceinline__ uint16_t relu_bf(uint16_t b) { return (b & 0x8000u) ? (uint16_t)0 : b; }

// One wave per row; lane l holds columns 4l + 256j (j < J).  Four rows per workgroup.
template <int J>
__global__ __launch_bounds__(256) void spmm_rows_kernel(int64_t rows, int64_t row0, int64_t H,
                                                        const int32_t* __restrict__ rowptr,
                                                        const int32_t* __restrict__ colidx,
                                                        const float* __restrict__ val, const bf16_t* __restrict__ Wt,
                                                        int64_t ldw, const float* __restrict__ bias, int relu,
                                                        bf16_t* __restrict__ Y, int64_t ldy,
                                                        uint8_t* __restrict__ mask, int64_t ld_mask) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int lane = threadIdx.x & 63;
  const int32_t k0 = rowptr[row0 + r], k1 = rowptr[row0 + r + 1];
  float acc[J][4];
#pragma unroll
  for (int j = 0; j < J; ++j) acc[j][0] = acc[j][1] = acc[j][2] = acc[j][3] = 0.f;
  bool live[J];
#pragma unroll
  for (int j = 0; j < J; ++j) live[j] = 4 * lane + 256 * j < H;
  int32_t k = k0;
  for (; k + SP_UNROLL <= k1; k += SP_UNROLL) {
    uint2 w[SP_UNROLL][J];
    float v[SP_UNROLL];
#pragma unroll
    for (int u = 0; u < SP_UNROLL; ++u) {
      const int64_t c = colidx[k + u];
      v[u] = val ? val[k + u] : 1.f;
#pragma unroll
      for (int j = 0; j < J; ++j)
        w[u][j] = live[j] ? *reinterpret_cast<const uint2*>(Wt + c * ldw + 4 * lane + 256 * j) : make_uint2(0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < SP_UNROLL; ++u)
#pragma unroll
      for (int j = 0; j < J; ++j) bf4_fma(acc[j], w[u][j], v[u]);
  }
  for (; k < k1; ++k) {
    const int64_t c = colidx[k];
    const float v = val ? val[k] : 1.f;
#pragma unroll
    for (int j = 0; j < J; ++j)
      if (live[j]) bf4_fma(acc[j], *reinterpret_cast<const uint2*>(Wt + c * ldw + 4 * lane + 256 * j), v);
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int64_t col = 4 * lane + 256 * j;
    uint32_t nib = 0;
    if (live[j]) {
      uint16_t b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        b[i] = f2bf(acc[j][i] + (bias ? bias[col + i] : 0.f));
        if (relu) b[i] = relu_bf(b[i]);
        nib |= (b[i] ? 1u : 0u) << i;
      }
      *reinterpret_cast<uint2*>(Y + r * ldy + col) =
          make_uint2((uint32_t)b[0] | ((uint32_t)b[1] << 16), (uint32_t)b[2] | ((uint32_t)b[3] << 16));
    }
    if (mask) {   // byte col / 8: this (even) lane's four columns and the next lane's
      const uint32_t hi = __shfl_xor(nib, 1, 64);
      if (live[j] && !(lane & 1)) mask[r * ld_mask + col / 8] = (uint8_t)(nib | (hi << 4));
    }
  }
}

// Eight features per workgroup, one wave per two of them (features 2w, 2w+1 of the group, one
// after the other); lane l holds outputs 4l + 256j (j < J).  The eight f32 columns meet in LDS
// and leave as 32-B runs of dW's rows.
constexpr int TN_FB = 8;

template <int J>
__global__ __launch_bounds__(256) void spmm_tn_kernel(int64_t F, int64_t H, const int32_t* __restrict__ colptr,
                                                      const int32_t* __restrict__ rowidx,
                                                      const float* __restrict__ val, const bf16_t* __restrict__ dY,
                                                      int64_t ldy, float* __restrict__ dW, int64_t ldw,
                                                      int accumulate) {
  __shared__ float tile[TN_FB][256 * J + 1];
  const int64_t f0 = (int64_t)blockIdx.x * TN_FB;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  bool live[J];
#pragma unroll
  for (int j = 0; j < J; ++j) live[j] = 4 * lane + 256 * j < H;
#pragma unroll
  for (int q = 0; q < TN_FB / 4; ++q) {
    const int fi = wv * (TN_FB / 4) + q;
    const int64_t f = f0 + fi;
    float acc[J][4];
#pragma unroll
    for (int j = 0; j < J; ++j) acc[j][0] = acc[j][1] = acc[j][2] = acc[j][3] = 0.f;
    if (f < F) {
      const int32_t k1 = colptr[f + 1];
      int32_t k = colptr[f];
      for (; k + SP_UNROLL <= k1; k += SP_UNROLL) {
        uint2 g[SP_UNROLL][J];
        float v[SP_UNROLL];
#pragma unroll
        for (int u = 0; u < SP_UNROLL; ++u) {
          const int64_t r = rowidx[k + u];
          v[u] = val ? val[k + u] : 1.f;
#pragma unroll
          for (int j = 0; j < J; ++j)
            g[u][j] = live[j] ? *reinterpret_cast<const uint2*>(dY + r * ldy + 4 * lane + 256 * j) : make_uint2(0u, 0u);
        }
#pragma unroll
        for (int u = 0; u < SP_UNROLL; ++u)
#pragma unroll
          for (int j = 0; j < J; ++j) bf4_fma(acc[j], g[u][j], v[u]);
      }
      for (; k < k1; ++k) {
        const int64_t r = rowidx[k];
        const float v = val ? val[k] : 1.f;
#pragma unroll
        for (int j = 0; j < J; ++j)
          if (live[j]) bf4_fma(acc[j], *reinterpret_cast<const uint2*>(dY + r * ldy + 4 * lane + 256 * j), v);
      }
    }
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) tile[fi][4 * lane + 256 * j + i] = acc[j][i];
  }
  __syncthreads();
  // thread t: output rows o = t, t + 256, ..; its TN_FB features' columns f0 .. f0+7
  for (int64_t o = threadIdx.x; o < H; o += 256) {
    float* dst = dW + o * ldw + f0;
#pragma unroll
    for (int fi = 0; fi < TN_FB; ++fi) {
      if (f0 + fi >= F) break;
      const float x = tile[fi][o];
      dst[fi] = accumulate ? dst[fi] + x : x;
    }
  }
}

template <int J>
void launch_rows(int64_t rows, int64_t row0, int64_t H, const int32_t* rowptr, const int32_t* colidx, const float* val,
                 const bf16_t* Wt, int64_t ldw, const float* bias, int relu, bf16_t* Y, int64_t ldy, uint8_t* mask,
                 int64_t ld_mask, hipStream_t s) {
  hipLaunchKernelGGL(spmm_rows_kernel<J>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, rows, row0, H, rowptr,
                     colidx, val, Wt, ldw, bias, relu, Y, ldy, mask, ld_mask);
}

template <int J>
void launch_tn(int64_t F, int64_t H, const int32_t* colptr, const int32_t* rowidx, const float* val, const bf16_t* dY,
               int64_t ldy, float* dW, int64_t ldw, int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(spmm_tn_kernel<J>, dim3((unsigned)((F + TN_FB - 1) / TN_FB)), dim3(256), 0, s, F, H, colptr,
                     rowidx, val, dY, ldy, dW, ldw, accumulate);
}

}  // namespace

extern "C" int llp_spmm_rows(int64_t rows, int64_t row0, int64_t H, const int32_t* rowptr, const int32_t* colidx,
                             const float* val, const void* Wt, int64_t ldw, const float* bias, int act, void* Y,
                             int64_t ldy, void* mask_out, int64_t ld_mask, void* stream) {
  LLP_CHECK_ARG(rows >= 0 && row0 >= 0 && H > 0 && H <= 1024 && H % 8 == 0,
                "llp_spmm_rows: rows >= 0, row0 >= 0, H in [8, 1024] with H %% 8 == 0 (rows=%lld row0=%lld H=%lld)",
                (long long)rows, (long long)row0, (long long)H);
  LLP_CHECK_ARG(act == LLP_ACT_NONE || act == LLP_ACT_RELU, "llp_spmm_rows: act must be NONE or RELU");
  LLP_CHECK_ARG(!mask_out || act == LLP_ACT_RELU, "llp_spmm_rows: a ReLU mask needs act RELU");
  if (rows == 0) return LLP_OK;
  LLP_CHECK_ARG(rowptr && colidx && Wt && Y && (!mask_out || ld_mask >= H / 8), "llp_spmm_rows: null pointer / ld_mask");
  LLP_CHECK_ARG((uintptr_t)Wt % 8 == 0 && ldw % 4 == 0 && ldw >= H && (uintptr_t)Y % 8 == 0 && ldy % 4 == 0 && ldy >= H,
                "llp_spmm_rows: Wt and Y need 8-B aligned rows (ldw, ldy multiples of 4, >= H)");
  hipStream_t s = (hipStream_t)stream;
  const bf16_t* w = (const bf16_t*)Wt;
  bf16_t* y = (bf16_t*)Y;
  uint8_t* m = (uint8_t*)mask_out;
  const int relu = act == LLP_ACT_RELU;
  switch ((H + 255) / 256) {
    case 1: launch_rows<1>(rows, row0, H, rowptr, colidx, val, w, ldw, bias, relu, y, ldy, m, ld_mask, s); break;
    case 2: launch_rows<2>(rows, row0, H, rowptr, colidx, val, w, ldw, bias, relu, y, ldy, m, ld_mask, s); break;
    case 3: launch_rows<3>(rows, row0, H, rowptr, colidx, val, w, ldw, bias, relu, y, ldy, m, ld_mask, s); break;
    default: launch_rows<4>(rows, row0, H, rowptr, colidx, val, w, ldw, bias, relu, y, ldy, m, ld_mask, s); break;
  }
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_spmm_tn(int64_t F, int64_t H, const int32_t* colptr, const int32_t* rowidx, const float* val,
                           const void* dY, int64_t ldy, float* dW, int64_t ldw, int accumulate, void* stream) {
  LLP_CHECK_ARG(F >= 0 && H > 0 && H <= 1024 && H % 4 == 0,
                "llp_spmm_tn: F >= 0, H in [4, 1024] with H %% 4 == 0 (F=%lld H=%lld)", (long long)F, (long long)H);
  if (F == 0) return LLP_OK;
  LLP_CHECK_ARG(colptr && rowidx && dY && dW && ldw >= F, "llp_spmm_tn: null pointer / ldw < F");
  LLP_CHECK_ARG((uintptr_t)dY % 8 == 0 && ldy % 4 == 0 && ldy >= H, "llp_spmm_tn: dY needs 8-B aligned rows");
  hipStream_t s = (hipStream_t)stream;
  const bf16_t* g = (const bf16_t*)dY;
  switch ((H + 255) / 256) {
    case 1: launch_tn<1>(F, H, colptr, rowidx, val, g, ldy, dW, ldw, accumulate, s); break;
    case 2: launch_tn<2>(F, H, colptr, rowidx, val, g, ldy, dW, ldw, accumulate, s); break;
    case 3: launch_tn<3>(F, H, colptr, rowidx, val, g, ldy, dW, ldw, accumulate, s); break;
    default: launch_tn<4>(F, H, colptr, rowidx, val, g, ldy, dW, ldw, accumulate, s); break;
  }
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}
