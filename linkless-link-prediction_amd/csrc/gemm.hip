// MFMA GEMMs for the LLP distillation step (gfx950).
//
//   llp_gemm_nt : C[m,n] = epi(alpha * sum_k A[m,k] B[n,k])   forward / data-grad
//   llp_gemm_tn : C[p,q] = sum_m A[m,p] B[m,q]                weight-grad (split-m slabs)
//
// Operands are llp_operand rows: plain, gathered (idx) or Hadamard of two
// gathered rows — the row gather x[this_target] (src/main.py:95-96) and the
// predictor input x_i*x_j (src/models.py:140) happen while staging, never in HBM.
//
// Tiles: 128x128 per 256-thread workgroup (4 waves, 2x2, 64x64 per wave),
// BK = 128 bytes of K per row (64 bf16 / 32 f32), register-staged double
// buffering into one LDS array, XOR-swizzled 16-B chunks.
//   bf16: v_mfma_f32_16x16x32_bf16, fragments by ds_read_b128 (NT) or
//         ds_read_b64_tr_b16 transposed reads (TN).
//   f32 : v_mfma_f32_16x16x4_f32 (exact f32 fma chain), fragments by
//         ds_read_b128 with a k-permutation shared by both operands (NT) or
//         ds_read_b32 (TN).
#include "llp_common.h"

int llp_gemm_nt_bf16_256(const llp_operand* A, const llp_operand* B, int64_t M, int64_t N, int64_t K, void* C,
                         int64_t ldc, const float* bias, int act, const void* aux, int64_t ld_aux, float alpha,
                         float drop_p, uint32_t drop_thresh, float drop_scale, uint64_t drop_seed,
                         const int64_t* drop_ctr, int64_t drop_stream, const float* head_w, float* head_part,
                         uint8_t* mask_out, const uint8_t* mask_in, int64_t ld_mask, hipStream_t s);
int llp_gemm_nt_bf16_splitk(const llp_operand* A, const llp_operand* B, int64_t M, int64_t N, int64_t K, void* C,
                            int64_t ldc, const float* bias, int relu, uint8_t* mask_out, int64_t ld_mask, int S,
                            float* slab, hipStream_t s);
int llp_cu_count();
int64_t llp_gemm_tn_256_splits(int64_t M, int64_t P, int64_t Q);
int llp_gemm_tn_bf16_256(const llp_operand* A, const llp_operand* B, int64_t M, int64_t P, int64_t Q, float* ws,
                         float* ws_colsum, int64_t splits, hipStream_t s);

namespace {

constexpr int BM = 128;
constexpr int BN = 128;
constexpr int NTHREADS = 256;

struct Op {
  const char* ptr;
  const int32_t* idx;
  const char* ptr2;
  const int32_t* idx2;
  int64_t ld;   // elements
  int64_t ld2;
};

struct NTParams {
  Op A, B;
  int64_t M, N, K;
  void* C;
  int64_t ldc;
  int c_bf16;
  const float* bias;
  int act;
  const void* aux;
  int64_t ld_aux;
  int aux_bf16;
  float alpha;
  float drop_p;          // 0 = no dropout
  uint32_t drop_thresh;  // llp::drop_code(p): keep iff drop_keep(..) (llp_common.h)
  float drop_scale;      // 1 / (1 - p)
  uint64_t drop_seed;
  const int64_t* drop_ctr;
  int64_t drop_stream;
  const int32_t* m_dev;  // device row count (llp_operand.rows_dev) or NULL
  int64_t ngroups;       // column groups walked one after another (nt_groups): B panel per XCD's L2
};

struct TNParams {
  Op A, B;
  int64_t M, P, Q;
  int64_t mchunk;
  int64_t splits;
  float* ws;  // [splits][P][Q]
  const int32_t* m_dev;  // device row count: M and mchunk are re-derived from it
};

// min(M, *m_dev) (M when m_dev is NULL)
__device__ __forceinline__ int64_t rows_live(int64_t M, const int32_t* m_dev) {
  if (!m_dev) return M;
  const int64_t c = *m_dev;
  return c < M ? (c > 0 ? c : 0) : M;
}

template <typename T>
struct Traits;
template <>
struct Traits<float> {
  static constexpr int ELEMS = 4;
};
template <>
struct Traits<bf16_t> {
  static constexpr int ELEMS = 8;
};

__device__ __forceinline__ float ld_elem(const float* p) { return *p; }
__device__ __forceinline__ float ld_elem(const bf16_t* p) { return bf2f(*p); }

__device__ __forceinline__ uint4 mul_chunk(uint4 a, uint4 b, float*) {
  uint4 r;
  r.x = __float_as_uint(__uint_as_float(a.x) * __uint_as_float(b.x));
  r.y = __float_as_uint(__uint_as_float(a.y) * __uint_as_float(b.y));
  r.z = __float_as_uint(__uint_as_float(a.z) * __uint_as_float(b.z));
  r.w = __float_as_uint(__uint_as_float(a.w) * __uint_as_float(b.w));
  return r;
}
__device__ __forceinline__ uint32_t mul_bf2(uint32_t a, uint32_t b) {
  const float a0 = __uint_as_float(a << 16), a1 = __uint_as_float(a & 0xFFFF0000u);
  const float b0 = __uint_as_float(b << 16), b1 = __uint_as_float(b & 0xFFFF0000u);
  return (uint32_t)f2bf(a0 * b0) | ((uint32_t)f2bf(a1 * b1) << 16);
}
__device__ __forceinline__ uint4 mul_chunk(uint4 a, uint4 b, bf16_t*) {
  return make_uint4(mul_bf2(a.x, b.x), mul_bf2(a.y, b.y), mul_bf2(a.z, b.z), mul_bf2(a.w, b.w));
}

// Load ELEMS consecutive elements [k0, k0+ELEMS) of a resolved row (p0 [, p1]).
// Elements at k >= K read as 0.  `valid` = row in range.
template <typename T, bool VEC>
__device__ __forceinline__ uint4 load_chunk(const T* p0, const T* p1, int64_t k0, int64_t K, bool valid) {
  constexpr int E = Traits<T>::ELEMS;
  uint4 r = make_uint4(0, 0, 0, 0);
  if (!valid) return r;
  if (VEC) {
    if (k0 < K) {
      r = *reinterpret_cast<const uint4*>(p0 + k0);
      if (p1) r = mul_chunk(r, *reinterpret_cast<const uint4*>(p1 + k0), (T*)nullptr);
    }
  } else {
    T v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      T x = T(0);
      if (k0 + e < K) {
        x = p0[k0 + e];
        if (p1) {
          if constexpr (sizeof(T) == 4) {
            x = x * p1[k0 + e];
          } else {
            x = f2bf(bf2f(x) * bf2f(p1[k0 + e]));
          }
        }
      }
      v[e] = x;
    }
    r = *reinterpret_cast<uint4*>(v);
  }
  return r;
}

template <typename T>
__device__ __forceinline__ const T* row_ptr(const Op& op, int64_t r) {
  const int64_t pr = op.idx ? (int64_t)op.idx[r] : r;
  return reinterpret_cast<const T*>(op.ptr) + pr * op.ld;
}
template <typename T>
__device__ __forceinline__ const T* row_ptr2(const Op& op, int64_t r) {
  if (!op.ptr2) return nullptr;
  const int64_t pr = op.idx2 ? (int64_t)op.idx2[r] : r;
  return reinterpret_cast<const T*>(op.ptr2) + pr * op.ld2;
}

// Bijective XCD-aware remap (cdna_hip_programming.md T1): blocks that share an
// XCD (same bid % 8) get a contiguous range of logical tiles.
__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nwg) {
  if (nwg < 8) return bid;
  const int64_t q = nwg / 8, r = nwg % 8;
  const int64_t xcd = bid % 8, loc = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// ============================================================== NT kernel
// NW waves per 128 x 128 tile: 4 (2 x 2, 64 x 64 per wave) or 8 (2 x 4, 64 x 32 per wave: four
// waves per SIMD at two workgroups per CU, to cover each other's K-tile boundary)
// BNT: the tile's width (128, or 256 for the f32 wide form: each wave 64 x 64, the A row panel
// re-read from L2 half as often; LDS 96 KB, one workgroup per CU).
template <typename T, bool VEC, int NW = 4, int BNT = BN>
__global__ __launch_bounds__(64 * NW, BNT == BN ? 2 : 1) void gemm_nt_kernel(NTParams p) {
  constexpr int E = Traits<T>::ELEMS;
  constexpr int BK = 8 * E;  // 8 chunks of 16 B per row
  constexpr int NT = 64 * NW, WN = NW / 2, WC = BNT / WN, JN = WC / 16, SI = (BM * 8) / NT, SIB = (BNT * 8) / NT;
  __shared__ uint4 smem[2 * (BM + BNT) * 8];
  uint4* sA0 = smem;
  uint4* sB0 = smem + BM * 8;
  const int buf_stride = (BM + BNT) * 8;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  p.M = rows_live(p.M, p.m_dev);
  const int64_t tilesN = (p.N + BNT - 1) / BNT;
  const int64_t tilesM = (p.M + BM - 1) / BM;
  if ((int64_t)blockIdx.x >= tilesM * tilesN) return;
  const int64_t lt = xcd_remap(blockIdx.x, tilesM * tilesN);
  // column group outermost (ngroups divides tilesN): the XCDs that take a group hold only its
  // slice of B in L2 while the row panels stream past (f32 B of 4 MB thrashed a 4 MB L2 with
  // the A panels: 3.4x A re-reads, profiles/r04_fp32_pmc_dominant.json)
  const int64_t tnG = tilesN / p.ngroups, per = tilesM * tnG;
  const int64_t grp = lt / per, rem = lt % per;
  const int64_t tm = rem / tnG, tn = grp * tnG + rem % tnG;
  const int64_t m0 = tm * BM, n0 = tn * BNT;

  // staging assignment: chunk c = tid + NT*i -> row (tid>>3) + (NT/8)*i, kc = tid&7
  const int kc = tid & 7;
  const T* pa[SI];
  const T* pa2[SI];
  const T* pb[SIB];
  const T* pb2[SIB];
  bool va[SI], vb[SIB];
#pragma unroll
  for (int i = 0; i < SI; ++i) {
    const int r = (tid >> 3) + (NT / 8) * i;
    int64_t gm = m0 + r;
    va[i] = gm < p.M;
    gm = va[i] ? gm : (p.M - 1);
    pa[i] = row_ptr<T>(p.A, gm);
    pa2[i] = row_ptr2<T>(p.A, gm);
  }
#pragma unroll
  for (int i = 0; i < SIB; ++i) {
    const int r = (tid >> 3) + (NT / 8) * i;
    int64_t gn = n0 + r;
    vb[i] = gn < p.N;
    gn = vb[i] ? gn : (p.N - 1);
    pb[i] = row_ptr<T>(p.B, gn);
    pb2[i] = row_ptr2<T>(p.B, gn);
  }

  uint4 ra[SI], rb[SIB];
  auto gload = [&](int64_t kt) {
    const int64_t k0 = kt * BK + kc * E;
#pragma unroll
    for (int i = 0; i < SI; ++i) ra[i] = load_chunk<T, VEC>(pa[i], pa2[i], k0, p.K, va[i]);
#pragma unroll
    for (int i = 0; i < SIB; ++i) rb[i] = load_chunk<T, VEC>(pb[i], pb2[i], k0, p.K, vb[i]);
  };
  auto lstore = [&](int buf) {
    uint4* sA = sA0 + buf * buf_stride;
    uint4* sB = sB0 + buf * buf_stride;
#pragma unroll
    for (int i = 0; i < SI; ++i) {
      const int r = (tid >> 3) + (NT / 8) * i;
      sA[r * 8 + (kc ^ (r & 7))] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < SIB; ++i) {
      const int r = (tid >> 3) + (NT / 8) * i;
      sB[r * 8 + (kc ^ (r & 7))] = rb[i];
    }
  };

  float4_t acc[4][JN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

  const int64_t nk = (p.K + BK - 1) / BK;
  gload(0);
  lstore(0);
  __syncthreads();

  const int g = lane >> 4, li = lane & 15;
  for (int64_t kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const uint4* sA = sA0 + buf * buf_stride;
    const uint4* sB = sB0 + buf * buf_stride;
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        short8 af[4], bfr[JN];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = wm * 64 + i * 16 + li;
          uint4 v = sA[r * 8 + ((g + 4 * s) ^ (r & 7))];
          af[i] = *reinterpret_cast<short8*>(&v);
        }
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int c = wn * WC + j * 16 + li;
          uint4 w = sB[c * 8 + ((g + 4 * s) ^ (c & 7))];
          bfr[j] = *reinterpret_cast<short8*>(&w);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < JN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        float4_t af[4], bfr[JN];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = wm * 64 + i * 16 + li;
          uint4 v = sA[r * 8 + ((kb * 4 + g) ^ (r & 7))];
          af[i] = *reinterpret_cast<float4_t*>(&v);
        }
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int c = wn * WC + j * 16 + li;
          uint4 w = sB[c * 8 + ((kb * 4 + g) ^ (c & 7))];
          bfr[j] = *reinterpret_cast<float4_t*>(&w);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < JN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][t], bfr[j][t], acc[i][j], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) lstore(buf ^ 1);
    __syncthreads();
  }

  // epilogue: acc[i][j][r] -> row m0 + wm*64 + i*16 + g*4 + r, col n0 + wn*WC + j*16 + li
  const uint64_t dstream = p.drop_p > 0.f ? (uint64_t)(LLP_STREAMS_PER_STEP * (*p.drop_ctr) + p.drop_stream) : 0;
#pragma unroll
  for (int j = 0; j < JN; ++j) {
    const int64_t col = n0 + wn * WC + j * 16 + li;
    if (col >= p.N) continue;
    const float bias = p.bias ? p.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 64 + i * 16 + g * 4 + r;
        if (row >= p.M) continue;
        float v = p.alpha * acc[i][j][r] + bias;
        if (p.act == LLP_ACT_RELU) {
          // f32: torch.relu's NaN propagation (fmaxf would give 0); bf16 output: the 256-tile
          // epilogues' sign-bit rule, so every bf16 kernel agrees
          v = p.c_bf16 ? (__float_as_int(v) < 0 ? 0.f : v) : (v < 0.f ? 0.f : v);
        } else if (p.act == LLP_ACT_RELU_BWD) {
          const float a = p.aux_bf16 ? bf2f(reinterpret_cast<const bf16_t*>(p.aux)[row * p.ld_aux + col])
                                     : reinterpret_cast<const float*>(p.aux)[row * p.ld_aux + col];
          v = a > 0.f ? v : 0.f;
        }
        if (p.drop_p > 0.f) {
          v = drop_keep(p.drop_thresh, p.drop_seed, dstream, row, col, p.N) ? v * p.drop_scale : 0.f;
        }
        if (p.c_bf16)
          reinterpret_cast<bf16_t*>(p.C)[row * p.ldc + col] = f2bf(v);
        else
          reinterpret_cast<float*>(p.C)[row * p.ldc + col] = v;
      }
    }
  }
}

// ============================================================== TN kernel
// C[p,q] = sum_m A[m,p] B[m,q]; block (tile, split z) writes ws[z][P][Q].
// bf16: BKm = 64 rows of m per step; LDS image [m][128 cols] (256 B rows),
//       swizzle ch ^ (((row&3)<<2) | ((row>>2)&3))  (T10 image (b)),
//       fragments via ds_read_b64_tr_b16.
// f32 : BKm = 32; LDS image [m][128 + 16 pad] floats; ds_read_b32.
__device__ __forceinline__ int tr_swz(int row, int ch) { return ch ^ (((row & 3) << 2) | ((row >> 2) & 3)); }

template <typename T, bool VEC, int NW = 4>
__global__ __launch_bounds__(64 * NW, 2) void gemm_tn_kernel(TNParams p) {
  constexpr int E = Traits<T>::ELEMS;
  constexpr bool BF = sizeof(T) == 2;
  static_assert(!BF || NW == 4, "the bf16 TN fragment path is written for four waves");
  constexpr int NT = 64 * NW, WN = NW / 2, WC = BN / WN, JN = WC / 16;
  constexpr int BKM = BF ? 64 : 32;
  constexpr int CPR = BF ? 16 : 32;               // 16-B chunks per 128-col row
  constexpr int ROWU4 = BF ? 16 : 36;             // uint4 per LDS row (f32 padded by 16 floats)
  constexpr int TILE_U4 = BKM * ROWU4;
  __shared__ uint4 smem[2 * 2 * TILE_U4];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wp = wave / WN, wq = wave % WN;
  const int64_t tilesQ = (p.Q + BN - 1) / BN;
  const int64_t tilesP = (p.P + BM - 1) / BM;
  const int64_t ntile = tilesP * tilesQ;
  const int64_t splits = p.splits;
  const int64_t lt = xcd_remap(blockIdx.x, ntile * splits);
  // bf16: the splits of one tile are adjacent in logical order (tile = lt / splits); f32: the
  // tiles of one split are (z = lt / ntile), so the workgroups an XCD runs together read the
  // same m rows of A and B (one HBM read, served from L2 to every tile of the split)
#ifdef LLP_NO_L2_ORDER   // A/B build: the f32 splits adjacent too (tools/gpu_call.sh fp32-ab)
  const int64_t tile = lt / splits, z = lt % splits;
#else
  const int64_t tile = BF ? lt / splits : lt % ntile, z = BF ? lt % splits : lt / ntile;
#endif
  const int64_t tp = tile / tilesQ, tq = tile % tilesQ;
  const int64_t p0 = tp * BM, q0 = tq * BN;
  if (p.m_dev) {   // live rows from the device count; the grid (splits) is the host M's
    p.M = rows_live(p.M, p.m_dev);
    const int64_t mc = (p.M + splits - 1) / splits;
    p.mchunk = mc > 0 ? (mc + BKM - 1) / BKM * BKM : BKM;
  }
  const int64_t mbeg = z * p.mchunk;
  const int64_t mend = min(p.M, mbeg + p.mchunk);

  // staging: chunk c = tid + NT*i -> m row c / CPR, chunk (c % CPR)
  constexpr int ROWS_PER_PASS = NT / CPR;  // 16 (bf16) or 8 / 16 (f32, 4 / 8 waves)
  constexpr int SI = BKM * CPR / NT;
  const int cc = tid % CPR;
  const int rr = tid / CPR;

  uint4 ra[SI], rb[SI];
  auto gload = [&](int64_t mt) {
#pragma unroll
    for (int i = 0; i < SI; ++i) {
      const int64_t m = mt + rr + ROWS_PER_PASS * i;
      const bool v = m < mend;
      const int64_t mm = v ? m : mbeg;
      const T* a0 = row_ptr<T>(p.A, mm);
      const T* a1 = row_ptr2<T>(p.A, mm);
      const T* b0 = row_ptr<T>(p.B, mm);
      const T* b1 = row_ptr2<T>(p.B, mm);
      // columns beyond P / Q read 0 (k-bound = P / Q on the column axis)
      ra[i] = load_chunk<T, VEC>(a0 + p0, a1 ? a1 + p0 : nullptr, (int64_t)cc * E, p.P - p0, v);
      rb[i] = load_chunk<T, VEC>(b0 + q0, b1 ? b1 + q0 : nullptr, (int64_t)cc * E, p.Q - q0, v);
    }
  };
  auto lstore = [&](int buf) {
    uint4* sA = smem + buf * 2 * TILE_U4;
    uint4* sB = sA + TILE_U4;
#pragma unroll
    for (int i = 0; i < SI; ++i) {
      const int r = rr + ROWS_PER_PASS * i;
      const int ch = BF ? tr_swz(r, cc) : cc;
      sA[r * ROWU4 + ch] = ra[i];
      sB[r * ROWU4 + ch] = rb[i];
    }
  };

  float4_t acc[4][JN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

  if (mbeg < mend) {
    const int64_t nsteps = (mend - mbeg + BKM - 1) / BKM;
    gload(mbeg);
    lstore(0);
    __syncthreads();
    const int g = lane >> 4, li = lane & 15;
    for (int64_t st = 0; st < nsteps; ++st) {
      const int buf = st & 1;
      if (st + 1 < nsteps) gload(mbeg + (st + 1) * BKM);
      const uint4* sA = smem + buf * 2 * TILE_U4;
      const uint4* sB = sA + TILE_U4;
      if constexpr (BF) {
        typedef __attribute__((address_space(3))) short4_t lds_s4;
        const int q4 = li >> 2, pp = li & 3;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          short8 af[4], bfr[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int col = wp * 64 + i * 16 + 4 * pp;
            const int colb = wq * 64 + i * 16 + 4 * pp;
#pragma unroll
            for (int hlf = 0; hlf < 2; ++hlf) {
              const int row = s * 32 + 8 * g + 4 * hlf + q4;
              const int offa = row * 256 + 16 * tr_swz(row, col >> 3) + 8 * ((col >> 2) & 1);
              const int offb = row * 256 + 16 * tr_swz(row, colb >> 3) + 8 * ((colb >> 2) & 1);
              short4_t ta = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                  (lds_s4*)((__attribute__((address_space(3))) char*)((__attribute__((address_space(3))) uint4*)sA) + offa));
              short4_t tb = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                  (lds_s4*)((__attribute__((address_space(3))) char*)((__attribute__((address_space(3))) uint4*)sB) + offb));
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                af[i][4 * hlf + e] = ta[e];
                bfr[i][4 * hlf + e] = tb[e];
              }
            }
          }
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < JN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
      } else {
        const float* fA = reinterpret_cast<const float*>(sA);
        const float* fB = reinterpret_cast<const float*>(sB);
#pragma unroll
        for (int t = 0; t < BKM / 4; ++t) {
          const int row = 4 * t + g;
          float af[4], bfr[JN];
#pragma unroll
          for (int i = 0; i < 4; ++i) af[i] = fA[row * (ROWU4 * 4) + wp * 64 + i * 16 + li];
#pragma unroll
          for (int j = 0; j < JN; ++j) bfr[j] = fB[row * (ROWU4 * 4) + wq * WC + j * 16 + li];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < JN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
      }
      if (st + 1 < nsteps) lstore(buf ^ 1);
      __syncthreads();
    }
  }
  // slab store: ws[z][row][col]
  const int g = lane >> 4, li = lane & 15;
  float* out = p.ws + z * p.P * p.Q;
#pragma unroll
  for (int j = 0; j < JN; ++j) {
    const int64_t col = q0 + wq * WC + j * 16 + li;
    if (col >= p.Q) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = p0 + wp * 64 + i * 16 + g * 4 + r;
        if (row < p.P) out[row * p.Q + col] = acc[i][j][r];
      }
  }
}

// Columns c >= qs go to C2 (column c - qs, row stride ldc2): one weight-gradient GEMM over a
// K-concatenated operand written straight into two modules' gradients.
__global__ void slab_reduce_kernel(const float* __restrict__ ws, int64_t splits, int64_t P, int64_t Q,
                                   float* __restrict__ C, int64_t ldc, int accumulate, int64_t qs,
                                   float* __restrict__ C2, int64_t ldc2) {
  const int64_t n = P * Q;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int64_t z = 0; z < splits; ++z) s += ws[z * n + e];
    const int64_t r = e / Q, c = e % Q;
    float* dst = c < qs ? C + r * ldc + c : C2 + r * ldc2 + (c - qs);
    *dst = accumulate ? *dst + s : s;
  }
}

// Vector form: C[p][q..q+3] (+)= sum_z ws[z][p][q..q+3] for Q % 4 == 0.  A block
// is 64 float4 columns x 4 slab groups (group g sums z in [g*S/4, (g+1)*S/4)
// with 8 loads in flight per thread); the group sums are added in group order
// through LDS: a fixed order, so the result is deterministic.  The scalar
// kernel above keeps one load in flight per thread and is latency-bound at
// large S (the teacher's TN splits, S = 128).
constexpr int SR_G = 4, SR_L = 256 / SR_G;
struct SlabJob {           // C[e4 / Q4][(e4 % Q4) * 4 ..] (+)= sum_z ws[z][e4], e4 < n4
  const float4* ws; int64_t S, n4, Q4; float* C; int64_t ldc;
  int64_t Q4s; float* C2; int64_t ldc2;   // float4 columns >= Q4s go to C2 (column - Q4s); Q4s = Q4: none
};
// One launch can carry two jobs (the weight slabs and the bias-gradient slabs of a TN
// GEMM): blocks [0, nblk0) take job 0, the rest job 1.
__global__ __launch_bounds__(256) void slab_reduce_v4_kernel(SlabJob j0, SlabJob j1, int64_t nblk0, int accumulate) {
  __shared__ float4 part[SR_G][SR_L];
  const bool second = (int64_t)blockIdx.x >= nblk0;
  const SlabJob& j = second ? j1 : j0;
  const float4* __restrict__ ws = j.ws;
  const int64_t S = j.S, n4 = j.n4;
  const int lane = threadIdx.x % SR_L, g = threadIdx.x / SR_L;
  const int64_t e4 = ((int64_t)blockIdx.x - (second ? nblk0 : 0)) * SR_L + lane;
  const int64_t z1 = (g + 1) * S / SR_G;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e4 < n4) {
    int64_t z = g * S / SR_G;
    for (; z + 8 <= z1; z += 8) {
      float4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = ws[(z + k) * n4 + e4];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w;
      }
    }
    for (; z < z1; ++z) {
      const float4 v = ws[z * n4 + e4];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  part[g][lane] = acc;
  __syncthreads();
  if (g != 0 || e4 >= n4) return;
  float4 t = part[0][lane];
#pragma unroll
  for (int k = 1; k < SR_G; ++k) {
    const float4 v = part[k][lane];
    t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
  }
  const int64_t row = e4 / j.Q4, q4 = e4 % j.Q4;
  float4* dst = reinterpret_cast<float4*>(q4 < j.Q4s ? j.C + row * j.ldc + q4 * 4 : j.C2 + row * j.ldc2 + (q4 - j.Q4s) * 4);
  if (accumulate) {
    const float4 o = *dst;
    t.x += o.x; t.y += o.y; t.z += o.z; t.w += o.w;
  }
  *dst = t;
}

// C (+)= sum of the S slabs [S][P][Q] (f32), deterministic; with C2, in the same
// launch when both take the vector form, also C2 (+)= sum of the S slabs [S][P2] at ws2
// (a TN GEMM's bias-gradient column sums).
// C (+)= ... for columns < qs, Cq (row stride ldq) for columns >= qs (qs < 0: Q, no split).
void slab_reduce(const float* ws, int64_t S, int64_t P, int64_t Q, float* C, int64_t ldc, int accumulate,
                 hipStream_t s, const float* ws2 = nullptr, int64_t P2 = 0, float* C2 = nullptr, int64_t qs = -1,
                 float* Cq = nullptr, int64_t ldq = 0) {
  const int64_t n = P * Q;
  if (qs < 0 || qs >= Q || !Cq) {
    qs = Q;
    Cq = C;
    ldq = ldc;
  }
  auto vec_ok = [](const float* w, int64_t q, const float* c, int64_t ld) {
    return q % 4 == 0 && ld % 4 == 0 && (uintptr_t)c % 16 == 0 && (uintptr_t)w % 16 == 0;
  };
  const bool v1 = n > 0 && vec_ok(ws, Q, C, ldc) && qs % 4 == 0 && vec_ok(ws, Q, Cq, ldq);
  const bool two = C2 && P2 > 0;
  const bool v2 = two && vec_ok(ws2, P2, C2, P2);
  if (v1) {
    SlabJob j0{reinterpret_cast<const float4*>(ws), S, n / 4, Q / 4, C, ldc, qs / 4, Cq, ldq};
    SlabJob j1 = j0;
    const int64_t nb0 = ceil_div_u(n / 4, SR_L);
    int64_t nb = nb0;
    if (v2) {
      j1 = SlabJob{reinterpret_cast<const float4*>(ws2), S, P2 / 4, P2 / 4, C2, P2, P2 / 4, C2, P2};
      nb += ceil_div_u(P2 / 4, SR_L);
    }
    hipLaunchKernelGGL(slab_reduce_v4_kernel, dim3((unsigned)nb), dim3(256), 0, s, j0, j1, nb0, accumulate);
  } else if (n > 0) {
    const unsigned nb = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(slab_reduce_kernel, dim3(nb), dim3(256), 0, s, ws, S, P, Q, C, ldc, accumulate, qs, Cq, ldq);
  }
  if (two && !(v1 && v2)) slab_reduce(ws2, S, (int64_t)1, P2, C2, P2, accumulate, s);
}

Op to_op(const llp_operand* o) {
  Op r;
  r.ptr = reinterpret_cast<const char*>(o->ptr);
  r.idx = o->idx;
  r.ptr2 = reinterpret_cast<const char*>(o->ptr2);
  r.idx2 = o->idx2;
  r.ld = o->ld;
  r.ld2 = o->ptr2 ? o->ld2 : 0;
  return r;
}

bool aligned_op(const llp_operand* o, int esize, int64_t extent_mult) {
  auto al = [&](const void* p, int64_t ld) {
    return ((uintptr_t)p % 16 == 0) && ((ld * esize) % 16 == 0);
  };
  bool ok = al(o->ptr, o->ld);
  if (o->ptr2) ok = ok && al(o->ptr2, o->ld2);
  return ok && (extent_mult % (16 / esize) == 0);
}

int64_t tn_splits(int dtype, int64_t M, int64_t P, int64_t Q) {
  const int64_t tiles = ((P + BM - 1) / BM) * ((Q + BN - 1) / BN);
  const int64_t bkm = dtype == LLP_BF16 ? 64 : 32;
  const int64_t wave = 4 * (int64_t)llp_cu_count();   // whole waves (4 blocks per CU): no sliver of a round
  int64_t splits = tiles >= wave ? 1 : wave / tiles;
  const int64_t maxs = (M + bkm * 8 - 1) / (bkm * 8);  // at least 8 m-steps per split
  if (splits > maxs) splits = maxs;
  if (splits < 1) splits = 1;
  return splits;
}

}  // namespace

// Column groups of the 128x128 NT kernel's tile walk: B (N x K) split into groups of at most
// 2 MB, half an XCD's 4 MB L2, when the row panels are many (each group then re-reads A once).
static int64_t nt_groups_w(int64_t N, int64_t K, int es, int64_t tilesM, int64_t bn) {
  const int64_t tilesN = (N + bn - 1) / bn;
  int64_t g = 1;
  while (g * 2 <= tilesN && tilesN % (g * 2) == 0 && N * K * es / g > (2ll << 20) && tilesM >= 64) g *= 2;
  return g;
}
static int64_t nt_groups(int64_t N, int64_t K, int es, int64_t tilesM) {
  const int64_t tilesN = (N + BN - 1) / BN;
  int64_t g = 1;
#ifdef LLP_NO_L2_ORDER   // A/B build: one group, the round-3 walk
  return g;
#endif
  while (g * 2 <= tilesN && tilesN % (g * 2) == 0 && N * K * es / g > (2ll << 20) && tilesM >= 64) g *= 2;
  return g;
}

int64_t llp_gemm_tn_f32_256_splits(int64_t M, int64_t P, int64_t Q);
int llp_gemm_tn_f32_256(const llp_operand* A, const llp_operand* B, int64_t M, int64_t P, int64_t Q, float* ws,
                        float* ws_colsum, int64_t splits, hipStream_t s);
int llp_gemm_nt_f32_256(const llp_operand* A, const llp_operand* B, int64_t M, int64_t N, int64_t K, float* C,
                        int64_t ldc, const float* bias, int act, const float* aux, int64_t ld_aux, float alpha,
                        hipStream_t s, const float* head_w = nullptr, float* head_part = nullptr);

extern "C" int llp_gemm_nt(int dtype, int64_t M, int64_t N, int64_t K, const llp_operand* A,
                           const llp_operand* B, void* C, int64_t ldc, int c_dtype, const float* bias,
                           int act, const void* aux, int64_t ld_aux, int aux_dtype, float alpha,
                           const llp_dropout* dropout, void* stream) {
  LLP_CHECK_ARG(A && B && (C || M == 0 || N == 0), "llp_gemm_nt: null operand");   // empty C: null (torch)
  LLP_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "llp_gemm_nt: negative size");
  LLP_CHECK_ARG(dtype == LLP_F32 || dtype == LLP_BF16, "llp_gemm_nt: bad dtype %d", dtype);
  LLP_CHECK_ARG(act != LLP_ACT_RELU_BWD || aux, "llp_gemm_nt: RELU_BWD needs aux");
  const bool mask = aux && aux_dtype == LLP_MASK;
  LLP_CHECK_ARG(!mask || act == LLP_ACT_RELU || act == LLP_ACT_RELU_BWD,
                "llp_gemm_nt: a bit-mask aux goes with RELU (written) or RELU_BWD (read)");
  if (M == 0 || N == 0) return LLP_OK;
  NTParams p;
  p.A = to_op(A);
  p.B = to_op(B);
  p.M = M; p.N = N; p.K = K;
  p.m_dev = A->rows_dev;
  p.C = C; p.ldc = ldc; p.c_bf16 = c_dtype == LLP_BF16;
  p.bias = bias; p.act = act; p.aux = aux; p.ld_aux = ld_aux; p.aux_bf16 = aux_dtype == LLP_BF16;
  p.alpha = alpha;
  p.drop_p = 0.f;
  p.drop_thresh = 0;
  p.drop_scale = 1.f;
  p.drop_seed = 0;
  p.drop_ctr = nullptr;
  p.drop_stream = 0;
  if (dropout && dropout->p > 0.f) {
    LLP_CHECK_ARG(dropout->p < 1.f && dropout->step_ctr, "llp_gemm_nt: dropout p in (0,1) needs step_ctr");
    p.drop_p = dropout->p;
    p.drop_thresh = llp::drop_code(dropout->p);
    p.drop_scale = 1.f / (1.f - dropout->p);
    p.drop_seed = dropout->seed;
    p.drop_ctr = dropout->step_ctr;
    p.drop_stream = dropout->stream_offset;
  }
  const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  LLP_CHECK_ARG(tiles < (1ll << 31), "llp_gemm_nt: too many tiles");
  hipStream_t s = (hipStream_t)stream;
  // Large-tile bf16 kernel (gemm256.hip) whenever the layout allows it.  (Round 5 measured the
  // 128 x 128 kernel for launches of <= 64 such tiles -- the physics student's 31-tile rank shard --
  // and it was slower: DESIGN.md 4.5.)
  auto a16 = [](const void* q, int64_t ld) { return ((uintptr_t)q % 16 == 0) && ((ld * 2) % 16 == 0); };
  if (dtype == LLP_BF16 && c_dtype == LLP_BF16 && K > 0 && K % 64 == 0 && N % 8 == 0 && !B->ptr2 &&
      a16(A->ptr, A->ld) && (!A->ptr2 || a16(A->ptr2, A->ld2)) && a16(B->ptr, B->ld) && a16(C, ldc) &&
      (act != LLP_ACT_RELU_BWD || mask || (aux_dtype == LLP_BF16 && a16(aux, ld_aux))) &&
      (!mask || (N % 32 == 0 && ld_aux % 4 == 0 && (uintptr_t)aux % 4 == 0))) {
    uint8_t* mask_out = mask && act == LLP_ACT_RELU ? (uint8_t*)aux : nullptr;
    const uint8_t* mask_in = mask && act == LLP_ACT_RELU_BWD ? (const uint8_t*)aux : nullptr;
    const int rc = llp_gemm_nt_bf16_256(A, B, M, N, K, C, ldc, bias, act, mask ? nullptr : aux, ld_aux, alpha,
                                        p.drop_p, p.drop_thresh, p.drop_scale, p.drop_seed, p.drop_ctr,
                                        p.drop_stream, nullptr, nullptr, mask_out, mask_in, ld_aux, s);
    if (rc != 0) return llp::set_error(rc, "llp_gemm_nt (256 tile): %s", hipGetErrorString((hipError_t)rc));
    return LLP_OK;
  }
  LLP_CHECK_ARG(!mask, "llp_gemm_nt: bit-mask aux needs the bf16 256-tile path (bf16 in/out, K %% 64 == 0, "
                       "N %% 32 == 0, 16-byte aligned operands)");
  const int es = dtype == LLP_BF16 ? 2 : 4;
  const bool vec = aligned_op(A, es, K) && aligned_op(B, es, K);
  p.ngroups = nt_groups(N, K, es, (M + BM - 1) / BM);
  dim3 grid((unsigned)tiles);
  if (dtype == LLP_BF16) {
    llp::note_kernel(vec ? "gemm_nt_kernel<bf16, vec> (128x128)" : "gemm_nt_kernel<bf16> (128x128)");
    if (vec) hipLaunchKernelGGL((gemm_nt_kernel<bf16_t, true>), grid, dim3(NTHREADS), 0, s, p);
    else hipLaunchKernelGGL((gemm_nt_kernel<bf16_t, false>), grid, dim3(NTHREADS), 0, s, p);
  } else {
#ifndef LLP_F32_NO_PP8
    // the persistent 256 x 256 LDS-DMA f32 kernel (gemm256_f32.hip) for plain aligned operands,
    // N % 256 == 0, K % 64 == 0, more than one wave of tiles, no dropout
    auto a16f = [](const void* q, int64_t ld) { return ((uintptr_t)q % 16 == 0) && (ld % 4 == 0); };
    const int64_t tiles256 = ((M + 255) / 256) * (N / 256);
    if (c_dtype == LLP_F32 && p.drop_p == 0.f && N % 256 == 0 && K > 0 && K % 64 == 0 && tiles256 > 256 &&
        !A->idx && !A->ptr2 && !B->idx && !B->ptr2 && a16f(A->ptr, A->ld) && a16f(B->ptr, B->ld) && a16f(C, ldc) &&
        (!bias || (uintptr_t)bias % 16 == 0) &&
        (act == LLP_ACT_RELU || act == LLP_ACT_NONE ||
         (act == LLP_ACT_RELU_BWD && aux_dtype == LLP_F32 && a16f(aux, ld_aux)))) {
      llp::note_kernel("gemm_nt_f32_pp8p (persistent 256x256, LDS-DMA, v_mfma_f32_16x16x4_f32)");
      const int rc = llp_gemm_nt_f32_256(A, B, M, N, K, (float*)C, ldc, bias, act, (const float*)aux, ld_aux, alpha, s);
      if (rc != 0) return llp::set_error(rc, "llp_gemm_nt (f32 256 tile): %s", hipGetErrorString((hipError_t)rc));
      return LLP_OK;
    }
#endif
    // eight waves per f32 tile (four per SIMD): 105.3 -> 97.5 ms per fp32 collab step, dominant
    // launch 4.28 -> 3.86 ms (profiles/r04_fp32_8w_ab.jsonl); bf16 keeps four (its 256 path rules)
#ifdef LLP_F32_NT_WIDE   // A/B build: 128 x 256 f32 tiles on LLP_F32_NT_WIDE (8 or 16) waves
    if (vec && N % 256 == 0) {
      NTParams pw = p;
      pw.ngroups = nt_groups_w(N, K, es, (M + BM - 1) / BM, 256);
      llp::note_kernel("gemm_nt_kernel<f32, vec, wide waves, 128x256> (v_mfma_f32_16x16x4_f32)");
      hipLaunchKernelGGL((gemm_nt_kernel<float, true, LLP_F32_NT_WIDE, 256>),
                         dim3((unsigned)(((M + BM - 1) / BM) * (N / 256))), dim3(64 * LLP_F32_NT_WIDE), 0, s, pw);
      LLP_LAUNCH_CHECK();
      return LLP_OK;
    }
#endif
    llp::note_kernel(vec ? "gemm_nt_kernel<f32, vec, 8 waves> (128x128, v_mfma_f32_16x16x4_f32)"
                         : "gemm_nt_kernel<f32, 8 waves> (128x128, v_mfma_f32_16x16x4_f32)");
    if (vec) hipLaunchKernelGGL((gemm_nt_kernel<float, true, 8>), grid, dim3(512), 0, s, p);
    else hipLaunchKernelGGL((gemm_nt_kernel<float, false, 8>), grid, dim3(512), 0, s, p);
  }
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

// Split-K plan: worth it when the 256x256 tiles fill under ~5/8 of the CUs and K is long.
// S = CUs / tiles (one wave of workgroups), at least 8 K-tiles per split, at most 16 slabs.
extern "C" int llp_gemm_nt_splitk_plan(int64_t M, int64_t N, int64_t K) {
#ifdef LLP_NO_SPLITK   // A/B build: never split
  return 1;
#endif
  if (M <= 0 || N <= 0 || N % 256 != 0 || K <= 0 || K % 64 != 0) return 1;
  const int64_t tiles = ((M + 255) / 256) * (N / 256), nkt = K / 64;
  const int64_t cus = llp_cu_count();
  if (tiles * 8 > cus * 5 || nkt < 16) return 1;
  int64_t S = cus / tiles;
  if (S > nkt / 8) S = nkt / 8;
  if (S > 16) S = 16;
  return S < 2 ? 1 : (int)S;
}

extern "C" int64_t llp_gemm_nt_splitk_ws_bytes(int64_t M, int64_t N, int splits) {
  return (int64_t)(splits > 0 ? splits : 0) * M * N * (int64_t)sizeof(float);
}

extern "C" int llp_gemm_nt_splitk(int64_t M, int64_t N, int64_t K, const llp_operand* A, const llp_operand* B, void* C,
                                  int64_t ldc, const float* bias, int act, void* mask_out, int64_t ld_mask, int splits,
                                  void* workspace, int64_t workspace_bytes, void* stream) {
  LLP_CHECK_ARG(A && B && (M == 0 || (C && workspace)), "llp_gemm_nt_splitk: null pointer");
  LLP_CHECK_ARG(act == LLP_ACT_NONE || act == LLP_ACT_RELU, "llp_gemm_nt_splitk: act must be NONE or RELU");
  LLP_CHECK_ARG(!mask_out || act == LLP_ACT_RELU, "llp_gemm_nt_splitk: a ReLU mask needs act RELU");
  LLP_CHECK_ARG(splits >= 1 && splits <= 64, "llp_gemm_nt_splitk: splits %d not in 1..64", splits);
  LLP_CHECK_ARG(M >= 0 && N % 256 == 0 && N > 0 && K % 64 == 0 && K / 64 >= splits,
                "llp_gemm_nt_splitk: needs N %% 256 == 0, K %% 64 == 0, K/64 >= splits (M=%lld N=%lld K=%lld S=%d)",
                (long long)M, (long long)N, (long long)K, splits);
  auto a16 = [](const void* q, int64_t ld) { return ((uintptr_t)q % 16 == 0) && ((ld * 2) % 16 == 0); };
  LLP_CHECK_ARG(!A->idx && !A->ptr2 && !A->rows_dev && !B->idx && !B->ptr2 && a16(A->ptr, A->ld) &&
                    a16(B->ptr, B->ld) && a16(C, ldc) && (!bias || (uintptr_t)bias % 16 == 0),
                "llp_gemm_nt_splitk: plain 16-B aligned bf16 operands and C, 16-B aligned bias");
  LLP_CHECK_ARG(workspace_bytes >= llp_gemm_nt_splitk_ws_bytes(M, N, splits) && (uintptr_t)workspace % 16 == 0,
                "llp_gemm_nt_splitk: workspace too small or misaligned");
  if (M == 0) return LLP_OK;
  const int rc = llp_gemm_nt_bf16_splitk(A, B, M, N, K, C, ldc, bias, act == LLP_ACT_RELU ? 1 : 0, (uint8_t*)mask_out,
                                         ld_mask, splits, (float*)workspace, (hipStream_t)stream);
  if (rc != 0) return llp::set_error(rc, "llp_gemm_nt_splitk: %s", hipGetErrorString((hipError_t)rc));
  return LLP_OK;
}

namespace {
__global__ void head_finish_kernel(int64_t parts, int64_t M, const float* __restrict__ part, const float* __restrict__ b,
                                   float* __restrict__ logit, float* __restrict__ prob) {
  const int64_t m = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (m >= M) return;
  float s = b ? b[0] : 0.f;
  for (int64_t t = 0; t < parts; ++t) s += part[t * M + m];   // fixed order: deterministic
  if (logit) logit[m] = s;
  if (prob) prob[m] = 1.f / (1.f + expf(-s));
}
}  // namespace

extern "C" int64_t llp_gemm_nt_head_parts(int64_t N) { return (N + 255) / 256; }

extern "C" int llp_gemm_nt_head(int64_t M, int64_t N, int64_t K, const llp_operand* A, const llp_operand* B, void* C,
                                int64_t ldc, const float* bias, int act, float alpha, const llp_dropout* dropout,
                                const float* head_w, float* head_part, void* stream) {
  LLP_CHECK_ARG(A && B && head_w && (head_part || M == 0), "llp_gemm_nt_head: null pointer");
  LLP_CHECK_ARG(act == LLP_ACT_NONE || act == LLP_ACT_RELU, "llp_gemm_nt_head: act must be NONE or RELU");
  auto a16 = [](const void* q, int64_t ld) { return ((uintptr_t)q % 16 == 0) && ((ld * 2) % 16 == 0); };
  LLP_CHECK_ARG(K > 0 && K % 64 == 0 && N % 8 == 0 && !A->ptr2 && !B->ptr2 && a16(A->ptr, A->ld) && a16(B->ptr, B->ld) &&
                    (!C || a16(C, ldc)),
                "llp_gemm_nt_head: needs bf16 rows of 16-B multiples, K %% 64 == 0, N %% 8 == 0, plain operands");
  if (M == 0) return LLP_OK;
  float dp = 0.f, ds = 1.f;
  uint32_t dth = 0;
  uint64_t dseed = 0;
  const int64_t* dctr = nullptr;
  int64_t dstr = 0;
  if (dropout && dropout->p > 0.f) {
    LLP_CHECK_ARG(dropout->p < 1.f && dropout->step_ctr, "llp_gemm_nt_head: dropout p in (0,1) needs step_ctr");
    dp = dropout->p;
    dth = llp::drop_code(dropout->p);
    ds = 1.f / (1.f - dropout->p);
    dseed = dropout->seed;
    dctr = dropout->step_ctr;
    dstr = dropout->stream_offset;
  }
  const int rc = llp_gemm_nt_bf16_256(A, B, M, N, K, C, ldc, bias, act, nullptr, 0, alpha, dp, dth, ds, dseed, dctr,
                                      dstr, head_w, head_part, nullptr, nullptr, 0, (hipStream_t)stream);
  if (rc != 0) return llp::set_error(rc, "llp_gemm_nt_head: %s", hipGetErrorString((hipError_t)rc));
  return LLP_OK;
}

// f32 operands: the persistent f32 kernel's F32_HEAD epilogue (gemm256_f32.hip), ReLU + head partials
// head_part[N / 256][M]; C (the hidden activations the head backward reads) is stored too.
extern "C" int llp_gemm_nt_head_f32(int64_t M, int64_t N, int64_t K, const llp_operand* A, const llp_operand* B,
                                    float* C, int64_t ldc, const float* bias, const float* head_w, float* head_part,
                                    void* stream) {
  LLP_CHECK_ARG(A && B && C && head_w && (head_part || M == 0), "llp_gemm_nt_head_f32: null pointer");
  auto a16f = [](const void* q, int64_t ld) { return ((uintptr_t)q % 16 == 0) && (ld % 4 == 0); };
  LLP_CHECK_ARG(K > 0 && K % 64 == 0 && N % 256 == 0 && !A->idx && !A->ptr2 && !B->idx && !B->ptr2 &&
                    a16f(A->ptr, A->ld) && a16f(B->ptr, B->ld) && a16f(C, ldc) && (uintptr_t)head_w % 16 == 0 &&
                    (!bias || (uintptr_t)bias % 16 == 0),
                "llp_gemm_nt_head_f32: needs plain 16-B aligned f32 operands, K %% 64 == 0, N %% 256 == 0");
  if (M == 0) return LLP_OK;
  llp::note_kernel("gemm_nt_f32_pp8p<F32_HEAD> (persistent 256x256, head fused)");
  const int rc = llp_gemm_nt_f32_256(A, B, M, N, K, C, ldc, bias, LLP_ACT_RELU, nullptr, 0, 1.f, (hipStream_t)stream,
                                     head_w, head_part);
  if (rc != 0) return llp::set_error(rc, "llp_gemm_nt_head_f32: %s", hipGetErrorString((hipError_t)rc));
  return LLP_OK;
}

extern "C" int llp_head_finish(int64_t parts, int64_t M, const float* part, const float* b, float* logit, float* prob,
                               void* stream) {
  LLP_CHECK_ARG(part || M == 0, "llp_head_finish: null part");
  if (M == 0) return LLP_OK;
  hipLaunchKernelGGL(head_finish_kernel, dim3(ceil_div_u(M, 256)), dim3(256), 0, (hipStream_t)stream, parts, M, part,
                     b, logit, prob);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int64_t llp_colsum_workspace_bytes(int64_t M, int64_t N);
extern "C" int llp_colsum(int dtype, int64_t M, int64_t N, const void* Y, int64_t ldy, float* out, int accumulate,
                          void* workspace, int64_t workspace_bytes, void* stream);
namespace llp {
int colsum_rows_dev(int dtype, int64_t M, int64_t N, const void* Y, int64_t ldy, float* out, int accumulate,
                    void* workspace, int64_t workspace_bytes, const int32_t* m_dev, void* stream);
}

// workspace = [weight slabs: splits*P*Q f32][column-sum region]
static int64_t tn_colsum_region(int dtype, int64_t M, int64_t P) {
  int64_t r = llp_colsum_workspace_bytes(M, P);
  if (dtype == LLP_BF16) r = std::max(r, llp_gemm_tn_256_splits(M, P, 256) * P * (int64_t)sizeof(float));
  else r = std::max(r, llp_gemm_tn_f32_256_splits(M, P, 256) * P * (int64_t)sizeof(float));
  return r;
}

// the contraction rows' device count: A's, else B's
static const int32_t* tn_rows_dev(const llp_operand* A, const llp_operand* B) {
  return A->rows_dev ? A->rows_dev : B->rows_dev;
}

extern "C" int64_t llp_gemm_tn_workspace_bytes(int dtype, int64_t M, int64_t P, int64_t Q) {
  int64_t s = tn_splits(dtype, M, P, Q);
  if (dtype == LLP_BF16) s = std::max(s, llp_gemm_tn_256_splits(M, P, Q));
  else s = std::max(s, llp_gemm_tn_f32_256_splits(M, P, Q));
  return s * P * Q * (int64_t)sizeof(float) + tn_colsum_region(dtype, M, P);
}

static int gemm_tn_impl(int dtype, int64_t M, int64_t P, int64_t Q, const llp_operand* A, const llp_operand* B,
                        float* C, int64_t ldc, int64_t qs, float* Cq, int64_t ldq, int accumulate, float* colsum_a,
                        void* workspace, int64_t workspace_bytes, void* stream) {
  LLP_CHECK_ARG(A && B && C, "llp_gemm_tn: null operand");
  LLP_CHECK_ARG(dtype == LLP_F32 || dtype == LLP_BF16, "llp_gemm_tn: bad dtype %d", dtype);
  LLP_CHECK_ARG(!colsum_a || (!A->idx && !A->ptr2), "llp_gemm_tn: colsum_a needs a plain A operand");
  if (P == 0 || Q == 0) return LLP_OK;
  if (workspace_bytes < llp_gemm_tn_workspace_bytes(dtype, M, P, Q) || !workspace)
    return llp::set_error(LLP_E_WORKSPACE, "llp_gemm_tn: workspace %lld < %lld", (long long)workspace_bytes,
                          (long long)llp_gemm_tn_workspace_bytes(dtype, M, P, Q));
  hipStream_t s = (hipStream_t)stream;
  auto a16 = [](const void* q, int64_t ld) { return ((uintptr_t)q % 16 == 0) && ((ld * 2) % 16 == 0); };
  if (dtype == LLP_BF16 && P % 8 == 0 && Q % 8 == 0 && !A->ptr2 && !B->ptr2 && a16(A->ptr, A->ld) &&
      a16(B->ptr, B->ld)) {
    // large-tile glds kernel (gemm256_tn.hip), bias gradient fused
    const int64_t sp = llp_gemm_tn_256_splits(M, P, Q);
    float* ws = reinterpret_cast<float*>(workspace);
    float* wcs = colsum_a ? ws + sp * P * Q : nullptr;
    const int rc = llp_gemm_tn_bf16_256(A, B, M, P, Q, ws, wcs, sp, s);
    if (rc != 0) return llp::set_error(rc, "llp_gemm_tn (256 tile): %s", hipGetErrorString((hipError_t)rc));
    // weight slabs and the [sp][P] column-sum slabs in one launch
    slab_reduce(ws, sp, P, Q, C, ldc, accumulate, s, wcs, colsum_a ? P : 0, colsum_a, qs, Cq, ldq);
    LLP_LAUNCH_CHECK();
    return LLP_OK;
  }
#ifndef LLP_F32_NO_PP8
  auto a16f = [](const void* q, int64_t ld) { return ((uintptr_t)q % 16 == 0) && (ld % 4 == 0); };
  // (Q <= 128 would leave half of every 256-wide tile's MFMAs on padding: the 128-tile kernel below
  // is faster there, 582 vs 930 us on the collab student's first layer, 225k x 1024 x 128)
  if (dtype == LLP_F32 && P % 4 == 0 && Q % 4 == 0 && Q > 128 && !A->idx && !A->ptr2 && !B->idx && !B->ptr2 &&
      a16f(A->ptr, A->ld) && a16f(B->ptr, B->ld)) {
    // the f32 256-tile LDS-DMA kernel (gemm256_tn_f32.hip), bias gradient fused
    const int64_t sp = llp_gemm_tn_f32_256_splits(M, P, Q);
    float* ws = reinterpret_cast<float*>(workspace);
    float* wcs = colsum_a ? ws + sp * P * Q : nullptr;
    const int rc = llp_gemm_tn_f32_256(A, B, M, P, Q, ws, wcs, sp, s);
    if (rc != 0) return llp::set_error(rc, "llp_gemm_tn (f32 256 tile): %s", hipGetErrorString((hipError_t)rc));
    slab_reduce(ws, sp, P, Q, C, ldc, accumulate, s, wcs, colsum_a ? P : 0, colsum_a, qs, Cq, ldq);
    LLP_LAUNCH_CHECK();
    return LLP_OK;
  }
#endif
  const int64_t splits = tn_splits(dtype, M, P, Q);
  if (colsum_a) {
    char* region = reinterpret_cast<char*>(workspace) + splits * P * Q * (int64_t)sizeof(float);
    const int rc = llp::colsum_rows_dev(dtype, M, P, A->ptr, A->ld, colsum_a, accumulate, region,
                                        tn_colsum_region(dtype, M, P), tn_rows_dev(A, B), stream);
    if (rc != 0) return rc;
  }
  TNParams p;
  p.A = to_op(A);
  p.B = to_op(B);
  p.M = M; p.P = P; p.Q = Q;
  p.m_dev = tn_rows_dev(A, B);
  const int64_t bkm = dtype == LLP_BF16 ? 64 : 32;
  int64_t mchunk = (M + splits - 1) / splits;
  mchunk = (mchunk + bkm - 1) / bkm * bkm;
  p.mchunk = mchunk > 0 ? mchunk : bkm;
  p.ws = reinterpret_cast<float*>(workspace);
  const int64_t tiles = ((P + BM - 1) / BM) * ((Q + BN - 1) / BN);
  const int es = dtype == LLP_BF16 ? 2 : 4;
  const bool vec = aligned_op(A, es, P) && aligned_op(B, es, Q);
  p.splits = splits;
  TNParams pp = p;
  dim3 g2((unsigned)(tiles * splits));
  if (dtype == LLP_BF16) {
    if (vec) hipLaunchKernelGGL((gemm_tn_kernel<bf16_t, true>), g2, dim3(NTHREADS), 0, s, pp);
    else hipLaunchKernelGGL((gemm_tn_kernel<bf16_t, false>), g2, dim3(NTHREADS), 0, s, pp);
  } else {
    // eight waves per f32 tile, as the f32 NT kernel: fp32 collab step 97.3 -> 95.3 ms
    // (profiles/r04_fp32_tn8w_ab.jsonl)
    if (vec) hipLaunchKernelGGL((gemm_tn_kernel<float, true, 8>), g2, dim3(512), 0, s, pp);
    else hipLaunchKernelGGL((gemm_tn_kernel<float, false, 8>), g2, dim3(512), 0, s, pp);
  }
  LLP_LAUNCH_CHECK();
  slab_reduce(reinterpret_cast<const float*>(workspace), splits, P, Q, C, ldc, accumulate, s, nullptr, 0, nullptr, qs,
              Cq, ldq);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_gemm_tn(int dtype, int64_t M, int64_t P, int64_t Q, const llp_operand* A,
                           const llp_operand* B, float* C, int64_t ldc, int accumulate, float* colsum_a,
                           void* workspace, int64_t workspace_bytes, void* stream) {
  return gemm_tn_impl(dtype, M, P, Q, A, B, C, ldc, -1, nullptr, 0, accumulate, colsum_a, workspace, workspace_bytes,
                      stream);
}

extern "C" int llp_gemm_tn_split(int dtype, int64_t M, int64_t P, int64_t Q, const llp_operand* A,
                                 const llp_operand* B, float* C, int64_t ldc, int64_t q_split, float* C2,
                                 int64_t ldc2, int accumulate, float* colsum_a, void* workspace,
                                 int64_t workspace_bytes, void* stream) {
  LLP_CHECK_ARG(C2 && q_split > 0 && q_split < Q, "llp_gemm_tn_split: bad split %lld of %lld columns",
                (long long)q_split, (long long)Q);
  return gemm_tn_impl(dtype, M, P, Q, A, B, C, ldc, q_split, C2, ldc2, accumulate, colsum_a, workspace,
                      workspace_bytes, stream);
}
