// Large-tile bf16 MFMA GEMM (NT form) for the LLP hot path — the kernel that
// carries the student MLP / LinkPredictor / teacher-predictor Linear layers
// (src/models.py:48,143,146) and their data-gradients.
//
//   C[m, n] = epi(alpha * sum_k A[m, k] * B[n, k])      bf16 in, f32 accumulate, bf16 out
//
// Geometry: 256 x 256 output tile per 512-thread workgroup (8 waves as 2 (m) x
// 4 (n), 128 x 64 per wave), BK = 64, one workgroup per CU (128 KiB of LDS
// double-buffered stages).  Staging: global_load_lds_dwordx4 (per-lane source
// address = gathered row, XOR-swizzled 16-B chunks, lane-linear LDS image) for
// plain / gathered operands; register staging (two loads, multiply, ds_write)
// when A is a Hadamard product x_i * x_j (src/models.py:140).
// MFMA roles are swapped (weights = MFMA A operand, activations = MFMA B
// operand) so that a lane's accumulator holds 4 CONSECUTIVE output columns of
// one output row: the epilogue (bias, ReLU, dropout) runs in registers, the
// tile is staged row-major through LDS and written with 16-byte coalesced
// stores; the ReLU-backward mask (aux) is read with the same 16-byte pattern.
#include "llp_common.h"

#include <type_traits>

#ifdef LLP_GEMM_STAMPS
// Diagnostic build (tools/gemm_stamps.py): per workgroup of the pp8 kernel, lane 0 of wave 0
// records s_memtime (shader clock) and s_memrealtime (100 MHz) at entry, after the prologue's
// first K-tile, after the main loop and at exit; read back by llp_debug_gemm_stamps.
constexpr int STAMP_MAX = 1 << 16;
__device__ unsigned long long g_llp_stamps[STAMP_MAX * 8];
#define LLP_STAMP(slot)                                                                          \
  do {                                                                                           \
    if (tid == 0 && blockIdx.x < STAMP_MAX) {                                                    \
      g_llp_stamps[blockIdx.x * 8 + 2 * (slot)] = __builtin_amdgcn_s_memtime();                  \
      g_llp_stamps[blockIdx.x * 8 + 2 * (slot) + 1] = __builtin_amdgcn_s_memrealtime();          \
    }                                                                                            \
  } while (0)
#else
#define LLP_STAMP(slot) \
  do {                  \
  } while (0)
#endif

namespace {

constexpr int TM = 256, TN = 256, TK = 64;
constexpr int NT2 = 512;
constexpr int STAGE_U4 = (TM + TN) * 8;          // uint4 per stage (A then B), 64 KiB
constexpr int EPI_ROW_U4 = TN / 8 + 1;           // 16-B chunks per staged C row (+1 pad)
constexpr int SMEM_U4_LOOP = 2 * STAGE_U4;       // 128 KiB
constexpr int SMEM_U4_EPI = TM * EPI_ROW_U4;     // 132 KiB
constexpr int SMEM_U4 = SMEM_U4_LOOP > SMEM_U4_EPI ? SMEM_U4_LOOP : SMEM_U4_EPI;

struct P256 {
  const bf16_t* A;  const int32_t* ia;  const bf16_t* A2; const int32_t* ia2; int64_t lda, lda2;
  const bf16_t* B;  const int32_t* ib;  int64_t ldb;
  int64_t M, N, K;
  bf16_t* C; int64_t ldc;
  const float* bias;
  int act;
  const bf16_t* aux; int64_t ld_aux;
  float alpha;
  float drop_p; uint32_t drop_thresh; float drop_scale; uint64_t drop_seed; const int64_t* drop_ctr;
  int64_t drop_stream;
  // fused Linear(N, 1) head (LinkPredictor's last layer, src/models.py:146):
  // head_part[tn][m] = sum over this tile's columns of y[m, n] * head_w[n]
  const float* head_w;
  float* head_part;
  // ReLU mask as bits (bit c%8 of byte c/8 of row r at +r*ld_mask): written by a
  // RELU forward (mask_out), read by RELU_BWD instead of the bf16 aux (mask_in)
  uint8_t* mask_out;
  const uint8_t* mask_in;
  int64_t ld_mask;
  // device row count (llp_operand.rows_dev): M = min(M, *m_dev) at run time;
  // the grid and head_part's row stride (head_ld) stay the host M
  const int32_t* m_dev;
  int64_t head_ld;
  int nt_store;   // epilogue stores with the non-temporal hint
  int lean_epi;   // pp8 mode kernels: lean epilogue on full tiles
};

typedef __attribute__((address_space(3))) void lds_void;

// hp + v . w over four columns in a fixed fma order
template <typename W4>
__device__ __forceinline__ float head_dot4(float hp, const float (&v)[4], const W4& w) {
  return fmaf(v[3], w[3], fmaf(v[2], w[2], fmaf(v[1], w[1], fmaf(v[0], w[0], hp))));
}

// byte of quad lane 0 | byte of lane 1 << 8 | lane 2 << 16 | lane 3 << 24, valid in
// lane 0 of every 4-lane quad.  Two DPP quad_perm moves (VALU) instead of three
// ds_bpermute round trips through the LDS pipe, whose latency every mask store
// waited for.  All 64 lanes must be active.
__device__ __forceinline__ uint32_t quad_pack_bytes(uint32_t byte) {
  const uint32_t t = byte | ((uint32_t)__builtin_amdgcn_mov_dpp((int)byte, 0xB1, 0xF, 0xF, false) << 8);   // [1,0,3,2]
  return t | ((uint32_t)__builtin_amdgcn_mov_dpp((int)t, 0x4E, 0xF, 0xF, false) << 16);                    // [2,3,0,1]
}

__device__ __forceinline__ int64_t xcd_remap2(int64_t bid, int64_t nwg) {
  if (nwg < 8) return bid;
  const int64_t q = nwg / 8, r = nwg % 8;
  const int64_t xcd = bid % 8, loc = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// This block's output tile.  Applies the device row count first (p.M shrinks to
// min(M, *m_dev)); the grid is sized for the host M, and blocks past the live
// tiles return before touching memory.  The live tiles are remapped as a
// contiguous range per XCD, as without a count.
__device__ __forceinline__ bool tile_256(P256& p, int64_t& m0, int64_t& n0) {
  if (p.m_dev) {
    const int64_t c = *p.m_dev;
    p.M = c < p.M ? (c > 0 ? c : 0) : p.M;
  }
  const int64_t tilesN = (p.N + TN - 1) / TN;
  const int64_t tilesM = (p.M + TM - 1) / TM;
  const int64_t nt = tilesM * tilesN;
  if ((int64_t)blockIdx.x >= nt) return false;
  const int64_t lt = xcd_remap2(blockIdx.x, nt);
  m0 = (lt / tilesN) * TM;
  n0 = (lt % tilesN) * TN;
  return true;
}

// Tile of this block on the HOST grid when the row count is device-resident
// (q64 kernel): m-tiles are dealt to XCDs round-robin (XCD x = blockIdx % 8
// takes m-tiles x, x+8, ..., each with its tilesN n-tiles in consecutive
// blocks), so the tiles past the live row count, which are the highest
// m-tiles, are spread over all eight XCDs instead of idling the last one.
// Needs no device value: the prologue is issued before the count is waited on.
// The grid is ceil(tilesM / 8) * 8 * tilesN blocks (llp_gemm_nt_bf16_256).
__device__ __forceinline__ bool tile_256_host_interleaved(const P256& p, int64_t& m0, int64_t& n0) {
  const int64_t tilesN = (p.N + TN - 1) / TN;
  const int64_t tilesM = (p.M + TM - 1) / TM;
  const int64_t xcd = blockIdx.x % 8, loc = blockIdx.x / 8;
  const int64_t mt = (loc / tilesN) * 8 + xcd;
  m0 = mt * TM;
  n0 = (loc % tilesN) * TN;
  return mt < tilesM;
}

__device__ __forceinline__ uint32_t mulbf2(uint32_t a, uint32_t b) {
  const float a0 = __uint_as_float(a << 16), a1 = __uint_as_float(a & 0xFFFF0000u);
  const float b0 = __uint_as_float(b << 16), b1 = __uint_as_float(b & 0xFFFF0000u);
  return (uint32_t)f2bf(a0 * b0) | ((uint32_t)f2bf(a1 * b1) << 16);
}

template <bool HADA>
__global__ __launch_bounds__(NT2) void gemm_nt_bf16_256(P256 p) {
  __shared__ __attribute__((aligned(16))) uint4 smem[SMEM_U4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  int64_t m0, n0;
  if (!tile_256(p, m0, n0)) return;

  // ---------------- staging addresses
  // glds: wave w stages rows [32w, 32w+32) of A and of B: 4 instructions each,
  // instruction i covers rows 32w + 8i + (lane>>3), physical chunk lane&7.
  const int srow0 = 32 * w + (lane >> 3);
  const int pch = lane & 7;
  const bf16_t* ga[4];
  const bf16_t* gb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = srow0 + 8 * i;
    const int lc = pch ^ (r & 7);                      // logical chunk stored at physical pch
    int64_t m = m0 + r;
    m = m < p.M ? m : p.M - 1;
    const int64_t pm = p.ia ? (int64_t)p.ia[m] : m;
    ga[i] = p.A + pm * p.lda + lc * 8;
    int64_t n = n0 + r;
    n = n < p.N ? n : p.N - 1;
    const int64_t pn = p.ib ? (int64_t)p.ib[n] : n;
    gb[i] = p.B + pn * p.ldb + lc * 8;
  }
  // register staging of a Hadamard A: thread t owns chunks t + 512*i (i < 4):
  // row (t>>3) + 64 i, logical chunk t & 7.
  const bf16_t* ha[4];
  const bf16_t* ha2[4];
  if (HADA) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int64_t m = m0 + (tid >> 3) + 64 * i;
      m = m < p.M ? m : p.M - 1;
      ha[i] = p.A + (p.ia ? (int64_t)p.ia[m] : m) * p.lda + (tid & 7) * 8;
      ha2[i] = p.A2 + (p.ia2 ? (int64_t)p.ia2[m] : m) * p.lda2 + (tid & 7) * 8;
    }
  }
  uint4 hr[4], hr2[4];

  auto stage_glds = [&](int buf, int64_t kt) {
    uint4* sA = smem + buf * STAGE_U4;
    uint4* sB = sA + TM * 8;
    const int64_t koff = kt * TK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (!HADA)
        __builtin_amdgcn_global_load_lds((const void*)(ga[i] + koff), (lds_void*)(sA + (32 * w + 8 * i) * 8), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(gb[i] + koff), (lds_void*)(sB + (32 * w + 8 * i) * 8), 16, 0, 0);
    }
  };
  auto hada_load = [&](int64_t kt) {
    const int64_t koff = kt * TK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      hr[i] = *reinterpret_cast<const uint4*>(ha[i] + koff);
      hr2[i] = *reinterpret_cast<const uint4*>(ha2[i] + koff);
    }
  };
  auto hada_store = [&](int buf) {
    uint4* sA = smem + buf * STAGE_U4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (tid >> 3) + 64 * i, c = tid & 7;
      uint4 v;
      v.x = mulbf2(hr[i].x, hr2[i].x); v.y = mulbf2(hr[i].y, hr2[i].y);
      v.z = mulbf2(hr[i].z, hr2[i].z); v.w = mulbf2(hr[i].w, hr2[i].w);
      sA[r * 8 + (c ^ (r & 7))] = v;
    }
  };

  // ---------------- main loop
  const int wm = w >> 2, wn = w & 3;
  float4_t acc[4][8];   // [n-tile jn][m-tile im]: rows n = 16 jn + 4 g + r, col m = 16 im + li
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = float4_t{0.f, 0.f, 0.f, 0.f};

  const int64_t nk = p.K / TK;
  if (HADA) hada_load(0);
  stage_glds(0, 0);
  if (HADA) hada_store(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int64_t kt = 0; kt < nk; ++kt) {
    const int buf = (int)(kt & 1);
    const bool more = kt + 1 < nk;
    if (more) {
      if (HADA) hada_load(kt + 1);
      stage_glds(buf ^ 1, kt + 1);
    }
    const uint4* sA = smem + buf * STAGE_U4;
    const uint4* sB = sA + TM * 8;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      short8 fw[4], fx[8];
#pragma unroll
      for (int jn = 0; jn < 4; ++jn) {
        const int r = wn * 64 + jn * 16 + li;
        uint4 v = sB[r * 8 + ((g + 4 * s) ^ (r & 7))];
        fw[jn] = *reinterpret_cast<short8*>(&v);
      }
#pragma unroll
      for (int im = 0; im < 8; ++im) {
        const int r = wm * 128 + im * 16 + li;
        uint4 v = sA[r * 8 + ((g + 4 * s) ^ (r & 7))];
        fx[im] = *reinterpret_cast<short8*>(&v);
      }
#pragma unroll
      for (int jn = 0; jn < 4; ++jn)
#pragma unroll
        for (int im = 0; im < 8; ++im)
          acc[jn][im] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[jn], fx[im], acc[jn][im], 0, 0, 0);
    }
    if (more && HADA) hada_store(buf ^ 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---------------- epilogue in registers: alpha, bias, ReLU, dropout
  const uint64_t dstream = p.drop_p > 0.f ? (uint64_t)(LLP_STREAMS_PER_STEP * (*p.drop_ctr) + p.drop_stream) : 0;
  uint4* stg = smem;   // staged C tile: row-major [256][EPI_ROW_U4] uint4
  // keep flags of this thread's 16 columns per row (one or two Philox blocks, drop_keep16)
  uint32_t kb[8];
#pragma unroll
  for (int im = 0; im < 8; ++im)
    kb[im] = p.drop_p > 0.f ? drop_keep16(p.drop_thresh, p.drop_seed, dstream, m0 + wm * 128 + im * 16 + li,
                                          n0 + wn * 64 + g * 4, p.N)
                            : 0u;
#pragma unroll
  for (int jn = 0; jn < 4; ++jn) {
    const int nl = wn * 64 + jn * 16 + g * 4;          // local column of element r = 0
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (p.bias) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = (n0 + nl + r < p.N) ? p.bias[n0 + nl + r] : 0.f;
    }
#pragma unroll
    for (int im = 0; im < 8; ++im) {
      const int ml = wm * 128 + im * 16 + li;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = p.alpha * acc[jn][im][r] + bv[r];
        if (p.act == LLP_ACT_RELU) v[r] = __float_as_int(v[r]) < 0 ? 0.f : v[r];   // the lean epilogues' sign rule
      }
      if (p.drop_p > 0.f) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (kb[im] >> (4 * jn + r)) & 1u ? v[r] * p.drop_scale : 0.f;
      }
      const uint32_t lo = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      const uint32_t hi = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      uint2* dst = reinterpret_cast<uint2*>(stg + ml * EPI_ROW_U4) + (nl >> 2);
      *dst = make_uint2(lo, hi);
    }
  }
  __syncthreads();
  // ---------------- coalesced write-out (+ ReLU-backward mask from aux)
  const int chunks_per_row = TN / 8;   // 32
#pragma unroll 4
  for (int q = tid; q < TM * chunks_per_row; q += NT2) {
    const int rl = q / chunks_per_row, c = q % chunks_per_row;
    const int64_t row = m0 + rl, col = n0 + c * 8;
    if (row >= p.M || col >= p.N) continue;
    uint4 v = stg[rl * EPI_ROW_U4 + c];
    if (p.act == LLP_ACT_RELU_BWD) {
      const uint4 a = *reinterpret_cast<const uint4*>(p.aux + row * p.ld_aux + col);
      const uint32_t av[4] = {a.x, a.y, a.z, a.w};
      uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool k0 = __uint_as_float(av[e] << 16) > 0.f;
        const bool k1 = __uint_as_float(av[e] & 0xFFFF0000u) > 0.f;
        vv[e] = (k0 ? (vv[e] & 0xFFFFu) : 0u) | (k1 ? (vv[e] & 0xFFFF0000u) : 0u);
      }
      v = make_uint4(vv[0], vv[1], vv[2], vv[3]);
    }
    *reinterpret_cast<uint4*>(p.C + row * p.ldc + col) = v;
  }
}

// ---------------------------------------------------------------------------
// LDS-DMA helpers of the pipelined kernels.  64-B image rows: 16-B chunk swizzle
// phys = logical ^ ((row >> 2) & 2) is conflict-free for ds_read_b128 fragment reads of
// 16 consecutive rows (checked against the four 16-lane bank groups of ds_read_b128).
// global_load_lds_dwordx4 issued from inline asm: hipcc's waitcnt pass then does
// not see the LDS-DMA and does not put s_waitcnt vmcnt(0) in front of every
// ds_read of the ring (it cannot prove the reads do not alias the DMA).  The
// kernel owns the counting: a counted s_waitcnt vmcnt + s_barrier before a stage is read.
__device__ __forceinline__ void glds16(const void* gptr, uint32_t lds_addr_uniform) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gptr),
               "s"(lds_addr_uniform)
               : "memory", "m0");
}
// SADDR form: a wave-uniform 64-bit base in SGPRs plus a per-lane 32-bit byte offset
__device__ __forceinline__ void glds16_s(uint32_t voff, const void* sbase, uint32_t lds_addr_uniform) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase),
               "s"(lds_addr_uniform)
               : "memory", "m0");
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) void*)p);
}

// Shared epilogue of the 256x256 kernels: alpha, bias, ReLU, dropout, fused
// Linear(N,1) head partials, LDS-staged coalesced store (+ReLU-bwd mask).
// smem must hold SMEM_U4_EPI uint4 + 4 KiB at smem + head_off_u4.
// Epilogue specialisations (compile-time flags instead of run-time branches per element):
// EPI_ANY reads everything from P256; EPI_FWD_RELU / EPI_FWD_NONE: alpha 1, optional bias and
// ReLU mask out, no dropout / head / aux; EPI_BWD_MASK: ReLU backward through a bit mask, alpha,
// no bias / dropout / head.  The host picks the mode (epi_mode_of).
constexpr int EPI_ANY = 0, EPI_FWD_RELU = 1, EPI_FWD_NONE = 2, EPI_BWD_MASK = 3, EPI_HEAD_RELU = 4;
// EPI_HEAD_RELU with the head dot taken from the staged bf16 outputs in the lean
// epilogue's second phase (pp8 / pp8p; epilogue_lean_head; the host's default)
constexpr int EPI_HEAD_LEAN = 5;
// split-K partial (pp8 only): workgroup (tile, blockIdx.y = s) sums K-tiles
// [nkt*s/S, nkt*(s+1)/S) and stores its raw f32 accumulators to slab s at
// head_part + s*M*N (row stride N); splitk_reduce_kernel applies the epilogue
constexpr int EPI_PARTIAL = 6;
// ReLU + dropout forward (pp8p only): EPI_FWD_RELU's epilogue with the keep draws
// (drop_keep16, one or two Philox blocks per thread row) applied before the bf16 rounding,
// and the ReLU mask of the dropped outputs; the values and bits of epilogue_t's dropout
constexpr int EPI_FWD_DROP = 7;
// EPI_HEAD_LEAN with dropout before the rounding, as EPI_FWD_DROP (pp8p only; the head dot is
// over the staged dropped outputs, the lean head's rule)
constexpr int EPI_HEAD_DROP = 8;

// MASK_LDS (TMv 256, NTHR 512 only): the ReLU-backward bit mask of the tile (256 rows x
// 32 bytes) is read with ONE 16-byte load per thread into LDS at smem + head_off_u4 + 256
// (512 uint4 past the head partials; the caller's LDS must hold them) and each store
// iteration takes its byte from there, instead of 16 one-byte global loads per thread.
template <int TMv, int NTHR, int MODE = EPI_ANY, bool MASK_LDS = false>
__device__ __forceinline__ void epilogue_t(const P256& p, float4_t (&acc)[4][8], uint4* smem, int head_off_u4,
                                           int64_t m0, int64_t n0, int tid, int wm, int wn, int g, int li) {
  static_assert(!MASK_LDS || (TMv == 256 && NTHR == 512 && TN == 256), "MASK_LDS: one 16-B mask piece per thread");
  const bool relu = MODE == EPI_FWD_RELU || MODE == EPI_HEAD_RELU || (MODE == EPI_ANY && p.act == LLP_ACT_RELU);
  const bool drop = MODE == EPI_ANY && p.drop_p > 0.f;
  const bool headw = MODE == EPI_HEAD_RELU || (MODE == EPI_ANY && p.head_w);
  const bool rbwd = MODE == EPI_BWD_MASK || (MODE == EPI_ANY && p.act == LLP_ACT_RELU_BWD);
  const bool fwd = MODE == EPI_FWD_RELU || MODE == EPI_FWD_NONE || MODE == EPI_HEAD_RELU;
  const float alpha = fwd ? 1.f : p.alpha;
  const float* bias = MODE == EPI_BWD_MASK ? nullptr : p.bias;
  const uint64_t dstream = drop ? (uint64_t)(LLP_STREAMS_PER_STEP * (*p.drop_ctr) + p.drop_stream) : 0;
  // ReLU-backward bit mask: this thread's 16 bytes (one per store below) are loaded
  // first, so their latency hides under the staging work instead of under each store
  constexpr int chunks_per_row = TN / 8;
  constexpr int ITERS = TMv * chunks_per_row / NTHR;
  const bool mask_rd = rbwd && (MODE == EPI_BWD_MASK || p.mask_in);
  uint32_t mb[ITERS];
  const uint8_t* mask_lds = reinterpret_cast<const uint8_t*>(smem + head_off_u4 + 256);
  if (MASK_LDS && mask_rd) {
    // row tid/2 of the tile, bytes 16*(tid&1) .. +15 (columns n0 + 128*(tid&1) ..)
    const int64_t row = m0 + (tid >> 1);
    const int64_t cb = (n0 >> 3) + 16 * (tid & 1);
    const uint8_t* src = p.mask_in + row * p.ld_mask + cb;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (row < p.M) {
      if (8 * (cb + 16) <= p.N && ((uintptr_t)src & 15) == 0) {
        v = *reinterpret_cast<const uint4*>(src);
      } else {
        uint8_t b[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) b[e] = 8 * (cb + e) < p.N ? src[e] : (uint8_t)0;
        v = *reinterpret_cast<const uint4*>(b);
      }
    }
    reinterpret_cast<uint4*>(smem + head_off_u4 + 256)[tid] = v;   // read after the barrier below
  } else if (mask_rd) {
#pragma unroll
    for (int i = 0; i < ITERS; ++i) {
      const int q = tid + i * NTHR;
      const int64_t row = m0 + q / chunks_per_row, col = n0 + (q % chunks_per_row) * 8;
      mb[i] = (row < p.M && col < p.N) ? (uint32_t)p.mask_in[row * p.ld_mask + (col >> 3)] : 0u;
    }
  }
  uint4* stg = smem;
  float hp[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // keep flags of this thread's 16 columns per row (one or two Philox blocks, drop_keep16)
  uint32_t kb[8];
#pragma unroll
  for (int im = 0; im < 8; ++im)
    kb[im] = drop ? drop_keep16(p.drop_thresh, p.drop_seed, dstream, m0 + wm * 128 + im * 16 + li,
                                n0 + wn * 64 + g * 4, p.N)
                  : 0u;
#pragma unroll
  for (int jn = 0; jn < 4; ++jn) {
    const int nl = wn * 64 + jn * 16 + g * 4;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    float hw[4] = {0.f, 0.f, 0.f, 0.f};
    if (bias) {
      if (MODE != EPI_ANY && n0 + nl + 3 < p.N && ((uintptr_t)bias & 15) == 0) {
        const float4_t b4 = *reinterpret_cast<const float4_t*>(bias + n0 + nl);
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = b4[r];
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = (n0 + nl + r < p.N) ? bias[n0 + nl + r] : 0.f;
      }
    }
    if (headw) {
#pragma unroll
      for (int r = 0; r < 4; ++r) hw[r] = (n0 + nl + r < p.N) ? p.head_w[n0 + nl + r] : 0.f;
    }
#pragma unroll
    for (int im = 0; im < 8; ++im) {
      const int ml = wm * 128 + im * 16 + li;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = fwd ? acc[jn][im][r] + bv[r] : alpha * acc[jn][im][r] + bv[r];
        // sign-bit ReLU, the lean epilogue's packed int16 max on the rounded pair: x if its sign
        // bit is clear (a +NaN stays NaN), else 0 (-0 and -NaN too), so the two agree on every input
        if (relu) v[r] = __float_as_int(v[r]) < 0 ? 0.f : v[r];
      }
      if (drop) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (kb[im] >> (4 * jn + r)) & 1u ? v[r] * p.drop_scale : 0.f;
      }
      // explicit fma order: the head partial is bit-identical across kernel variants
      if (headw) hp[im] = head_dot4(hp[im], v, hw);
      const uint32_t lo = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      const uint32_t hi = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      uint2* dst = reinterpret_cast<uint2*>(stg + ml * EPI_ROW_U4) + (nl >> 2);
      *dst = make_uint2(lo, hi);
    }
  }
  if (headw) {
    float* part = reinterpret_cast<float*>(smem + head_off_u4);   // [4 wn][TMv rows]
#pragma unroll
    for (int im = 0; im < 8; ++im) {
      float v = hp[im];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (g == 0) part[wn * TMv + wm * 128 + im * 16 + li] = v;
    }
  }
  __syncthreads();
  if (headw && tid < TMv && m0 + tid < p.M) {
    const float* part = reinterpret_cast<const float*>(smem + head_off_u4);
    const float s = part[tid] + part[TMv + tid] + part[2 * TMv + tid] + part[3 * TMv + tid];
    p.head_part[(n0 / TN) * p.head_ld + m0 + tid] = s;
  }
  if (!p.C) return;
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int q = tid + i * NTHR;
    const int rl = q / chunks_per_row, c = q % chunks_per_row;
    const int64_t row = m0 + rl, col = n0 + c * 8;
    const bool ok = row < p.M && col < p.N;
    uint4 v = stg[rl * EPI_ROW_U4 + c];
    if (rbwd) {
      uint32_t vv[4] = {v.x, v.y, v.z, v.w};
      if (mask_rd) {
        const uint32_t bits = MASK_LDS ? (uint32_t)mask_lds[rl * 32 + c] : mb[i];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          vv[e] = ((bits >> (2 * e)) & 1u ? (vv[e] & 0xFFFFu) : 0u) | ((bits >> (2 * e + 1)) & 1u ? (vv[e] & 0xFFFF0000u) : 0u);
      } else if (MODE == EPI_ANY && ok) {
        const uint4 a = *reinterpret_cast<const uint4*>(p.aux + row * p.ld_aux + col);
        const uint32_t av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool k0 = __uint_as_float(av[e] << 16) > 0.f;
          const bool k1 = __uint_as_float(av[e] & 0xFFFF0000u) > 0.f;
          vv[e] = (k0 ? (vv[e] & 0xFFFFu) : 0u) | (k1 ? (vv[e] & 0xFFFF0000u) : 0u);
        }
      }
      v = make_uint4(vv[0], vv[1], vv[2], vv[3]);
    }
    if (ok) {
      if (p.nt_store) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 vv = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(vv, reinterpret_cast<u32x4*>(p.C + row * p.ldc + col));
      } else {
        *reinterpret_cast<uint4*>(p.C + row * p.ldc + col) = v;
      }
    }
    if ((MODE == EPI_ANY || MODE == EPI_FWD_RELU || MODE == EPI_FWD_NONE) && p.mask_out) {
      // bit e of this chunk's byte = (bf16 output e > 0), the test RELU_BWD applies;
      // four consecutive lanes (one row, 32 columns) pack one 32-bit word
      const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
      uint32_t byte = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        byte |= (__uint_as_float(vw[e] << 16) > 0.f ? 1u : 0u) << (2 * e);
        byte |= (__uint_as_float(vw[e] & 0xFFFF0000u) > 0.f ? 1u : 0u) << (2 * e + 1);
      }
      const uint32_t word = quad_pack_bytes(byte);
      if ((q & 3) == 0 && ok) *reinterpret_cast<uint32_t*>(p.mask_out + row * p.ld_mask + (col >> 3)) = word;
    }
  }
}

template <int MODE = EPI_ANY, bool MASK_LDS = false>
__device__ __forceinline__ void epilogue_256(const P256& p, float4_t (&acc)[4][8], uint4* smem, int head_off_u4,
                                             int64_t m0, int64_t n0, int tid, int wm, int wn, int g, int li) {
  epilogue_t<TM, NT2, MODE, MASK_LDS>(p, acc, smem, head_off_u4, m0, n0, tid, wm, wn, g, li);
}

// ---------------------------------------------------------------------------
// K64 quadrant-phase variant: full 128-byte lines per DMA piece.
// A K-tile of 64 (A and B images [256 rows][128 B], 64 KiB) is consumed in 4
// phases; phase p computes one quadrant (m-half mh, n-half nh) of every wave's
// 128 x 64 output over K = 64 (16 MFMAs), in the order (0,0) (0,1) (1,1) (1,0)
// so each phase re-reads only one operand half.  The DMA of the next K-tile is
// cut into the same halves — chunk 0 = A rows with row%128 < 64, 1 = B rows
// with row%64 < 32, 2 = B rows with row%64 >= 32, 3 = the other A rows — and
// chunk j of tile t+1 is issued in phase j of tile t (2 x 1 KiB pieces per
// wave, 8 rows x 128 B each).  Two K-tile buffers.  RAW: before the barrier of
// the phase that first reads a chunk (phases 0, 0, 1, 2), a counted vmcnt
// leaves exactly the younger pieces in flight.  WAR: chunk j is re-filled 2-4
// phases after its last read (drained by lgkmcnt inside that phase).
__device__ __forceinline__ int q64_row(int chunk, int cr) {
  // chunk-row cr in [0,128) -> tile row
  switch (chunk) {
    case 0: return (cr & 63) + 128 * (cr >> 6);
    case 3: return (cr & 63) + 128 * (cr >> 6) + 64;
    case 1: return (cr & 31) + 64 * (cr >> 5);
    default: return (cr & 31) + 64 * (cr >> 5) + 32;
  }
}

// bias (or head weights) of 16 columns c0 .. c0 + 15, four per float4 (0 past N)
__device__ __forceinline__ void load_cols16(const float* v, int64_t N, int64_t c0, float4_t (&out)[4]) {
  // columns c0 + 16 jn + 0..3 of v (v null -> 0); c0 % 4 == 0
#pragma unroll
  for (int jn = 0; jn < 4; ++jn) {
    const int64_t c = c0 + 16 * jn;
    if (v && c + 3 < N && ((uintptr_t)v & 15) == 0) {
      out[jn] = *reinterpret_cast<const float4_t*>(v + c);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) out[jn][r] = (v && c + r < N) ? v[c + r] : 0.f;
    }
  }
}

// ---------------------------------------------------------------------------
// Lean epilogue of the pp8 kernel for FULL 256 x 256 tiles of the per-call modes
// EPI_FWD_RELU / EPI_FWD_NONE / EPI_BWD_MASK (same values and bits as epilogue_t).
// epilogue_t spends ~1,450 VALU per wave on a ReLU-forward tile (per-element
// bias loads and f32 ReLU, 64-bit store addressing and bounds tests per store,
// per-bit mask compares); here:
//  * bias from registers loaded before the main loop, packed f32 adds (v_pk_add /
//    v_pk_fma as before), ReLU AFTER rounding as a packed int16 max on the bf16
//    pair: the sign-bit rule of epilogue_t (x if the sign bit is clear, else 0), so
//    the two epilogues agree on every input, NaNs included (+NaN stays NaN; -NaN
//    becomes 0 where torch.relu would keep it);
//  * LDS staging at per-thread bases + compile-time offsets;
//  * stores from a uniform tile-corner base (SGPRs, advanced per 16 rows) plus one
//    32-bit lane offset, no bounds tests;
//  * ReLU mask byte of 8 non-negative bf16: nonzero tests as packed u16 min(x, 1),
//    three shift-ors and a fold (11 VALU instead of ~35).
template <int MODE>
__device__ __forceinline__ bool lean_tile_ok(const P256& p, int64_t m0, int64_t n0) {
  if (!p.lean_epi || m0 + TM > p.M || n0 + TN > p.N || (p.ldc & 7) || ((uintptr_t)p.C & 15)) return false;
  if (MODE == EPI_FWD_RELU && p.mask_out && ((p.ld_mask & 3) || ((uintptr_t)p.mask_out & 3))) return false;
  if (MODE == EPI_BWD_MASK && ((p.ld_mask & 15) || ((uintptr_t)p.mask_in & 15))) return false;
  return true;
}

typedef float float2_t __attribute__((ext_vector_type(2)));
typedef short short2_t __attribute__((ext_vector_type(2)));
typedef unsigned short ushort2_t __attribute__((ext_vector_type(2)));

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_bf16(float2_t v) {   // one v_cvt_pk_bf16_f32 (RNE, as f2bf)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}
__device__ __forceinline__ uint32_t relu_pk_bf16(uint32_t x) {   // v_pk_max_i16(x, 0)
  const short2_t r = __builtin_elementwise_max(__builtin_bit_cast(short2_t, x), (short2_t){0, 0});
  return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint32_t nz_pk_u16(uint32_t x, uint32_t ones) {   // v_pk_min_u16(x, 1): 1 per nonzero half
  uint32_t r;   // (asm: hipcc turns the builtin min into per-half compares and selects)
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(x), "v"(ones));
  return r;
}

// 0xFFFF where bit B of `bits` is set | 0xFFFF0000 where bit B+1 is: two sign-extended
// one-bit fields and a bitfield insert (hipcc makes ~10 VALU of the plain expression)
template <int B>
__device__ __forceinline__ uint32_t half_mask(uint32_t bits, uint32_t lo16) {   // lo16 = 0xFFFF (SGPR)
  uint32_t lo, hi;
  asm("v_bfe_i32 %0, %2, %3, 1\n\t"
      "v_bfe_i32 %1, %2, %4, 1\n\t"
      "v_bfi_b32 %0, %5, %0, %1"
      : "=&v"(lo), "=&v"(hi)
      : "v"(bits), "i"(B), "i"(B + 1), "s"(lo16));
  return lo;
}

template <int MODE>
__device__ __forceinline__ void epilogue_lean(const P256& p, float4_t (&acc)[4][8], const float4_t (&bvec)[4],
                                              uint4* smem, int64_t m0, int64_t n0, int tid, int wm, int wn, int g,
                                              int li) {
  constexpr bool RELU = MODE == EPI_FWD_RELU;
  constexpr bool BWD = MODE == EPI_BWD_MASK;
  constexpr int ROWB = EPI_ROW_U4 * 16;   // bytes per staged row
  uint8_t* mlds = reinterpret_cast<uint8_t*>(smem + SMEM_U4_EPI + 256);
  if (BWD) {   // the tile's 256 x 32 mask bytes: one 16-B piece per thread (row tid/2, half tid&1)
    const uint8_t* src = p.mask_in + (m0 + (tid >> 1)) * p.ld_mask + (n0 >> 3) + 16 * (tid & 1);
    reinterpret_cast<uint4*>(mlds)[tid] = *reinterpret_cast<const uint4*>(src);
  }
  // phase 1: row wm*128 + im*16 + li, columns wn*64 + jn*16 + g*4 .. +3
  char* sb = reinterpret_cast<char*>(smem) + (wm * 128 + li) * ROWB + (wn * 64 + g * 4) * 2;
  const float2_t al = {p.alpha, p.alpha}, z2 = {0.f, 0.f};
#pragma unroll
  for (int jn = 0; jn < 4; ++jn) {
    const float2_t b01 = {bvec[jn][0], bvec[jn][1]}, b23 = {bvec[jn][2], bvec[jn][3]};
#pragma unroll
    for (int im = 0; im < 8; ++im) {
      float2_t v01 = {acc[jn][im][0], acc[jn][im][1]}, v23 = {acc[jn][im][2], acc[jn][im][3]};
      if (BWD) {   // alpha * acc + 0 (v_pk_fma, as epilogue_t)
        v01 = __builtin_elementwise_fma(v01, al, z2);
        v23 = __builtin_elementwise_fma(v23, al, z2);
      } else {   // acc + bias (zeros without a bias, as epilogue_t adds)
        v01 = v01 + b01;
        v23 = v23 + b23;
      }
      uint32_t lo = pk_bf16(v01), hi = pk_bf16(v23);
      if (RELU) { lo = relu_pk_bf16(lo); hi = relu_pk_bf16(hi); }
      *reinterpret_cast<uint2*>(sb + im * 16 * ROWB + jn * 32) = make_uint2(lo, hi);
    }
  }
  __syncthreads();
  // phase 2: chunk (row rl0 + 16 i, 16-B column chunk c) per iteration
  const int rl0 = tid >> 5, c = tid & 31;
  const char* rb = reinterpret_cast<const char*>(smem) + rl0 * ROWB + c * 16;
  char* cbase = reinterpret_cast<char*>(p.C + m0 * p.ldc + n0);
  const uint32_t toff = (uint32_t)((rl0 * p.ldc + c * 8) * 2);
  const int64_t cstep = 16 * p.ldc * 2;
  const bool mo = RELU && p.mask_out;
  char* mbase = mo ? reinterpret_cast<char*>(p.mask_out + m0 * p.ld_mask + (n0 >> 3)) : nullptr;
  const uint32_t moff = (uint32_t)(rl0 * p.ld_mask + c);
  const int64_t mstep = 16 * p.ld_mask;
  const uint32_t ones = 0x00010001u;
  const uint32_t lo16 = __builtin_amdgcn_readfirstlane(0xFFFFu);
  auto run = [&](auto NTS) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      uint4 v = *reinterpret_cast<const uint4*>(rb + i * 16 * ROWB);
      if (BWD) {
        const uint32_t bits = mlds[(rl0 + 16 * i) * 32 + c];
        v.x &= half_mask<0>(bits, lo16);
        v.y &= half_mask<2>(bits, lo16);
        v.z &= half_mask<4>(bits, lo16);
        v.w &= half_mask<6>(bits, lo16);
      }
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 sv = {v.x, v.y, v.z, v.w};
      u32x4* dst = reinterpret_cast<u32x4*>(cbase + i * cstep + toff);
      if constexpr (decltype(NTS)::value) __builtin_nontemporal_store(sv, dst);
      else *dst = sv;
      if (RELU) {
        if (mo) {
          const uint32_t u = nz_pk_u16(v.x, ones) | (nz_pk_u16(v.y, ones) << 2) | (nz_pk_u16(v.z, ones) << 4) |
                             (nz_pk_u16(v.w, ones) << 6);
          const uint32_t word = quad_pack_bytes((u | (u >> 15)) & 0xFFu);
          if ((c & 3) == 0) *reinterpret_cast<uint32_t*>(mbase + i * mstep + moff) = word;
        }
      }
    }
  };
  if (p.nt_store) run(std::true_type{});
  else run(std::false_type{});
}

// Lean epilogue of the fused Linear(N,1) head (EPI_HEAD_LEAN, opt-in): phase 1 as
// EPI_FWD_RELU (bias, bf16 rounding, packed ReLU, LDS staging); phase 2 reads each
// staged 16-B chunk once for the optional store of C AND the head dot of its 8
// columns (head weights in 8 registers per thread), so the per-element f32 dot of
// epilogue_t (4 fma per accumulator quad + 16 cross-lane adds per tile row) goes.
// The dot is taken over the ROUNDED bf16 outputs (the values the head backward reads
// back), in a fixed order: 8 fma per chunk, quad sums by DPP ([1,0,3,2] then
// [2,3,0,1]), the row's 8 quad partials summed in column order -- deterministic, but
// not bit-identical to EPI_HEAD_RELU's f32 dot (differences of bf16 rounding size).
// Runs on EVERY tile (no generic fallback in the kernel, which made it spill): the host
// launches it only for N % 256 == 0, 16-B aligned head weights and C rows; rows past M
// (the last m-tile, or a device row count) are neither stored nor summed.
__device__ __forceinline__ float dpp_quad_sum(float d) {
  d += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(d), 0xB1, 0xF, 0xF, false));   // [1,0,3,2]
  return d + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(d), 0x4E, 0xF, 0xF, false));   // [2,3,0,1]
}

__device__ __forceinline__ void epilogue_lean_head(const P256& p, float4_t (&acc)[4][8], uint4* smem, int64_t m0,
                                                   int64_t n0, int tid, int wm, int wn, int g, int li) {
  constexpr int ROWB = EPI_ROW_U4 * 16;
  const int rl0 = tid >> 5, c = tid & 31;
  // this thread's 8 head weights (columns n0 + 8c ..), issued first: their latency
  // hides under phase 1
  const float4_t hw0 = *reinterpret_cast<const float4_t*>(p.head_w + n0 + 8 * c);
  const float4_t hw1 = *reinterpret_cast<const float4_t*>(p.head_w + n0 + 8 * c + 4);
  float4_t bl[4];
  load_cols16(p.bias, p.N, n0 + wn * 64 + g * 4, bl);
  char* sb = reinterpret_cast<char*>(smem) + (wm * 128 + li) * ROWB + (wn * 64 + g * 4) * 2;
#pragma unroll
  for (int jn = 0; jn < 4; ++jn) {
    const float2_t b01 = {bl[jn][0], bl[jn][1]}, b23 = {bl[jn][2], bl[jn][3]};
#pragma unroll
    for (int im = 0; im < 8; ++im) {
      const float2_t v01 = float2_t{acc[jn][im][0], acc[jn][im][1]} + b01;
      const float2_t v23 = float2_t{acc[jn][im][2], acc[jn][im][3]} + b23;
      *reinterpret_cast<uint2*>(sb + im * 16 * ROWB + jn * 32) =
          make_uint2(relu_pk_bf16(pk_bf16(v01)), relu_pk_bf16(pk_bf16(v23)));
    }
  }
  __syncthreads();
  // phase 2: chunk (row rl0 + 16 i, columns 8c .. 8c+7); quad partials to LDS past the
  // staging, [256 rows][8 quads] floats (8 KiB of the 12 KiB the kernel reserves there)
  float* part = reinterpret_cast<float*>(smem + SMEM_U4_EPI);
  const char* rb = reinterpret_cast<const char*>(smem) + rl0 * ROWB + c * 16;
  const bool st = p.C != nullptr;
  char* cbase = st ? reinterpret_cast<char*>(p.C + m0 * p.ldc + n0) : nullptr;
  const uint32_t toff = st ? (uint32_t)((rl0 * p.ldc + c * 8) * 2) : 0u;
  const int64_t cstep = st ? 16 * p.ldc * 2 : 0;
  const int64_t rows = p.M - m0;   // live rows of this tile (>= 1)
  auto run = [&](auto NTS) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint4 v = *reinterpret_cast<const uint4*>(rb + i * 16 * ROWB);
      if (st && rl0 + 16 * i < rows) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 sv = {v.x, v.y, v.z, v.w};
        u32x4* dst = reinterpret_cast<u32x4*>(cbase + i * cstep + toff);
        if constexpr (decltype(NTS)::value) __builtin_nontemporal_store(sv, dst);
        else *dst = sv;
      }
      float d = __uint_as_float(v.x << 16) * hw0[0];
      d = fmaf(__uint_as_float(v.x & 0xFFFF0000u), hw0[1], d);
      d = fmaf(__uint_as_float(v.y << 16), hw0[2], d);
      d = fmaf(__uint_as_float(v.y & 0xFFFF0000u), hw0[3], d);
      d = fmaf(__uint_as_float(v.z << 16), hw1[0], d);
      d = fmaf(__uint_as_float(v.z & 0xFFFF0000u), hw1[1], d);
      d = fmaf(__uint_as_float(v.w << 16), hw1[2], d);
      d = fmaf(__uint_as_float(v.w & 0xFFFF0000u), hw1[3], d);
      d = dpp_quad_sum(d);
      if ((c & 3) == 0) part[(rl0 + 16 * i) * 8 + (c >> 2)] = d;
    }
  };
  if (p.nt_store) run(std::true_type{});
  else run(std::false_type{});
  __syncthreads();
  if (tid < TM && tid < rows) {
    const float4_t a = *reinterpret_cast<const float4_t*>(part + tid * 8);
    const float4_t b = *reinterpret_cast<const float4_t*>(part + tid * 8 + 4);
    p.head_part[(n0 / TN) * p.head_ld + m0 + tid] = ((a[0] + a[1]) + (a[2] + a[3])) + ((b[0] + b[1]) + (b[2] + b[3]));
  }
}

// ---------------------------------------------------------------------------
// Ping-pong variant of the q64 loop (cdna_hip_programming.md §5 "The 256²
// 8-phase template"): every quadrant phase is a LOAD segment (counted vmcnt,
// the phase's ds_reads, its DMA chunk of the next K-tile), a barrier, an MFMA
// segment (lgkmcnt(0), 16 MFMAs at s_setprio 1) and a second barrier.  Waves
// 4-7 (rows 128-255) run one barrier behind waves 0-3, so on every SIMD one
// wave's MFMA segment coincides with its partner's LOAD segment and the two
// never compete for the matrix pipe.  Same chunks, quadrant order, MFMA
// operands and per-accumulator k order as q64 (bit-identical outputs).
//
// Chunk j of K-tile t+1 is issued in phase j of tile t.  With the groups one
// barrier apart, the data a phase reads must be waited for (each wave's counted
// vmcnt) in the PREVIOUS phase's LOAD segment, so the barriers ending both
// groups' segments of that phase order it before every reader: chunks 0, 1 in
// phase 3 of the previous tile, chunk 2 in phase 0, chunk 3 in phase 1.  WAR:
// chunk j's refill (phase j of tile t+1) comes 4-5 phases after its last read.
template <int MODE>
__global__ __launch_bounds__(NT2) void gemm_nt_bf16_pp8(P256 p) {
  constexpr int IMG_U4 = 256 * 8;
  constexpr int TILE_U4 = 2 * IMG_U4;
  // staging + head partials (256 uint4) + the ReLU-backward mask tile (512 uint4, MASK_LDS)
  constexpr int SM_U4 = 2 * TILE_U4 > SMEM_U4_EPI + 768 ? 2 * TILE_U4 : SMEM_U4_EPI + 768;
  __shared__ __attribute__((aligned(16))) uint4 smem[SM_U4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  LLP_STAMP(0);
  int64_t m0, n0;
  const bool dyn = p.m_dev != nullptr;
  const int32_t mlive = dyn ? *p.m_dev : 0;
  if (dyn ? !tile_256_host_interleaved(p, m0, n0) : !tile_256(p, m0, n0)) return;
  if constexpr (MODE == EPI_PARTIAL) {   // this workgroup's K range and slab
    const int64_t nkt = p.K / TK, S = gridDim.y, sk = blockIdx.y;
    const int64_t k0 = nkt * sk / S, k1 = nkt * (sk + 1) / S;
    p.A += k0 * TK;
    p.B += k0 * TK;
    p.K = (k1 - k0) * TK;
    p.head_part += sk * p.M * p.N;
  }

  const bf16_t* src[4][2];
  int dst_row[4][2];
  const int wu = __builtin_amdgcn_readfirstlane(w);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row0 = q64_row(j, 16 * wu + 8 * i);
      dst_row[j][i] = row0;
      const int r = row0 + (lane >> 3);
      const int lc = (lane & 7) ^ (r & 7);
      if (j == 0 || j == 3) {
        int64_t m = m0 + r;
        m = m < p.M ? m : p.M - 1;
        src[j][i] = p.A + (p.ia ? (int64_t)p.ia[m] : m) * p.lda + lc * 8;
      } else {
        int64_t n = n0 + r;
        n = n < p.N ? n : p.N - 1;
        src[j][i] = p.B + (p.ib ? (int64_t)p.ib[n] : n) * p.ldb + lc * 8;
      }
    }
  const uint32_t lds0 = lds_u32(smem);
  auto issue_chunk = [&](int j, int64_t kt) {
    const uint32_t base = lds0 + (uint32_t)((kt & 1) * TILE_U4 * 16) + ((j == 0 || j == 3) ? 0u : IMG_U4 * 16u);
    const int64_t koff = kt * TK;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      glds16(src[j][i] + koff, __builtin_amdgcn_readfirstlane(base + (uint32_t)(dst_row[j][i] * 128)));
  };

  const int wm = w >> 2, wn = w & 3;
  float4_t bvec[4];     // bias of the lane's 16 epilogue columns, loaded under the main loop
  // lean epilogue modes (the fused-head mode measured slower: its bias and head weights
  // in registers make the kernel spill)
  constexpr bool LEAN = MODE == EPI_FWD_RELU || MODE == EPI_FWD_NONE || MODE == EPI_BWD_MASK;
  if (LEAN && MODE != EPI_BWD_MASK) load_cols16(p.bias, p.N, n0 + wn * 64 + g * 4, bvec);
  else if (LEAN) bvec[0] = bvec[1] = bvec[2] = bvec[3] = float4_t{0.f, 0.f, 0.f, 0.f};
  float4_t acc[4][8];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = float4_t{0.f, 0.f, 0.f, 0.f};

  const int64_t nk = p.K / TK;
  short8 fa[2][4];
  short8 fb[2][2][2];
  auto read_a = [&](const uint4* sA, int mh) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int im = 0; im < 4; ++im) {
        const int r = wm * 128 + mh * 64 + im * 16 + li;
        uint4 v = sA[r * 8 + ((kh * 4 + g) ^ (r & 7))];
        fa[kh][im] = *reinterpret_cast<short8*>(&v);
      }
  };
  auto read_b = [&](const uint4* sB, int nh) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int jn = 0; jn < 2; ++jn) {
        const int r = wn * 64 + nh * 32 + jn * 16 + li;
        uint4 v = sB[r * 8 + ((kh * 4 + g) ^ (r & 7))];
        fb[nh][kh][jn] = *reinterpret_cast<short8*>(&v);
      }
  };
  auto mfma_q = [&](int mh, int nh) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int jn = 0; jn < 2; ++jn)
#pragma unroll
        for (int im = 0; im < 4; ++im)
          acc[nh * 2 + jn][mh * 4 + im] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[nh][kh][jn], fa[kh][im], acc[nh * 2 + jn][mh * 4 + im], 0,
                                                      0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: the whole of K-tile 0; chunks 0 and 1 (phase 0) landed for every wave
#pragma unroll
  for (int j = 0; j < 4; ++j) issue_chunk(j, 0);
  if (dyn) {
    p.M = mlive < p.M ? (mlive > 0 ? mlive : 0) : p.M;
    if (m0 >= p.M) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      return;
    }
  }
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  barrier();
  LLP_STAMP(1);
  const bool grp1 = wu >= 4;
  if (grp1) barrier();          // waves 4-7: one barrier behind from here on
  for (int64_t kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    const uint4* sA = smem + (int)(kt & 1) * TILE_U4;
    const uint4* sB = sA + IMG_U4;
    // phase 0, quadrant (0,0): wait chunk 2 of this tile (read in phase 1); younger: chunk 3
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    read_a(sA, 0);
    read_b(sB, 0);
    if (more) issue_chunk(0, kt + 1);
    barrier();
    mfma_q(0, 0);
    barrier();
    // phase 1, (0,1): wait chunk 3 (read in phase 2); younger: chunk 0 of the next tile
    if (more) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    read_b(sB, 1);
    if (more) issue_chunk(1, kt + 1);
    barrier();
    mfma_q(0, 1);
    barrier();
    // phase 2, (1,1): nothing to wait for
    read_a(sA, 1);
    if (more) issue_chunk(2, kt + 1);
    barrier();
    mfma_q(1, 1);
    barrier();
    // phase 3, (1,0): operands in registers; wait chunks 0, 1 of the next tile; younger: chunk 2
    if (more) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    if (more) issue_chunk(3, kt + 1);
    barrier();
    mfma_q(1, 0);
    barrier();
  }
  if (!grp1) barrier();         // waves 0-3 match the other half's barrier count
  LLP_STAMP(2);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if constexpr (MODE == EPI_PARTIAL) {   // raw accumulators: lane (li, g) holds row im*16 + li, columns jn*16 + g*4 ..
#pragma unroll
    for (int im = 0; im < 8; ++im) {
      const int64_t row = m0 + wm * 128 + im * 16 + li;
      if (row < p.M) {
        float* dst = p.head_part + row * p.N + n0 + wn * 64 + g * 4;
#pragma unroll
        for (int jn = 0; jn < 4; ++jn) *reinterpret_cast<float4_t*>(dst + jn * 16) = acc[jn][im];
      }
    }
    return;
  } else if constexpr (MODE == EPI_HEAD_LEAN) {   // every tile (the host checked the shapes)
    __syncthreads();
    epilogue_lean_head(p, acc, smem, m0, n0, tid, wm, wn, g, li);
    return;
  } else {
    if constexpr (LEAN) {
      if (lean_tile_ok<MODE>(p, m0, n0)) {
        __syncthreads();
        epilogue_lean<MODE>(p, acc, bvec, smem, m0, n0, tid, wm, wn, g, li);
        LLP_STAMP(3);
        return;
      }
    }
    __syncthreads();
    epilogue_256<MODE, true>(p, acc, smem, SMEM_U4_EPI, m0, n0, tid, wm, wn, g, li);
  }
}

}  // namespace

namespace {

// ---------------------------------------------------------------------------
// Persistent form of pp8 for the lean modes (EPI_FWD_RELU / EPI_FWD_NONE / EPI_BWD_MASK,
// plain operands, K % 128 == 0).  In pp8 every 256 x 256 tile pays a prologue (its first
// K-tile's DMA, nothing to overlap it with) and an epilogue (LDS staging + 128 KB of
// stores) on top of the main loop: tools/gemm_stamps.py measured 6.6k + 8.4k of 58.8k
// cycles per tile at the dominant shape (26 %).  Here one workgroup per CU walks its
// tiles (t = blockIdx.x, + gridDim.x, ...; the tile map of tile_256_host_interleaved),
// and the last K-tile of a tile issues the NEXT tile's first K-tile into buffer 0, exactly
// as it would issue its own next K-tile (same phases, same counted waits: WAR-safe for
// the same reason), so that DMA lands during the epilogue.  The epilogue (the lean one of
// pp8, with row guards for a partial last m-tile; the host admits only shapes it takes)
// therefore must not touch buffer 0: it stages the C tile in two 128-row halves in
// [64 KB, 131 KB), and
// the bias and the ReLU-backward mask tile come into LDS by DMA at the tile's start (an
// ordinary load would make hipcc drain every DMA in flight, vmcnt(0), at its first use),
// and all its barriers are raw s_barrier + lgkmcnt waits (a __syncthreads() would drain
// the prefetch too).  Before the next tile's loop a counted vmcnt leaves only the
// epilogue's stores in flight.  Per tile the MFMAs, their operands and their order are
// pp8's, and the lean epilogue's values are epilogue_t's: outputs are bit-identical.
constexpr int PP_STAGE_U4 = 128 * EPI_ROW_U4;          // one 128-row half of the staged C tile
template <int MODE>
__global__ __launch_bounds__(NT2) void gemm_nt_bf16_pp8p(P256 p) {
  static_assert(MODE == EPI_FWD_RELU || MODE == EPI_FWD_NONE || MODE == EPI_BWD_MASK || MODE == EPI_HEAD_LEAN ||
                    MODE == EPI_FWD_DROP || MODE == EPI_HEAD_DROP,
                "lean modes only");
  constexpr bool DROP = MODE == EPI_FWD_DROP || MODE == EPI_HEAD_DROP;
  constexpr bool RELU = MODE == EPI_FWD_RELU || MODE == EPI_FWD_DROP;   // (the ReLU bit mask out)
  constexpr bool BWD = MODE == EPI_BWD_MASK;
  constexpr bool HEAD = MODE == EPI_HEAD_LEAN || MODE == EPI_HEAD_DROP;
  constexpr int IMG_U4 = 256 * 8;
  constexpr int TILE_U4 = 2 * IMG_U4;
  constexpr int STG = TILE_U4;                          // staging half: [64 KB, 64 KB + 66 KB)
  constexpr int MLDS = STG + PP_STAGE_U4;               // ReLU-backward mask tile: 256 x 32 B (head: quad partials)
  constexpr int BLDS = MLDS + 512;                      // bias of the tile's 256 columns: 1 KB
  constexpr int HWLDS = BLDS + 64;                      // head weights of the tile's 256 columns: 1 KB
  constexpr int SM_A = HWLDS + 64;
  constexpr int SM_B = SMEM_U4_EPI + 768;               // epilogue_256 (partial tiles)
  constexpr int SM_U4 = SM_A > SM_B ? SM_A : SM_B;
  static_assert(SM_U4 * 16 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) uint4 smem[SM_U4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int wm = w >> 2, wn = w & 3;
  const bool grp1 = wu >= 4;
  const int64_t tilesN = (p.N + TN - 1) / TN;
  const int64_t tilesM_host = (p.M + TM - 1) / TM;
  // the map below deals m-tiles to XCDs in groups of 8, so its index space is the m-tile
  // count padded to a multiple of 8 (the padding's tiles are skipped) -- also without a
  // device row count
  const int64_t n_tiles = (tilesM_host + 7) / 8 * 8 * tilesN;
  int64_t M_live = p.M;
  if (p.m_dev) {
    const int64_t c = *p.m_dev;
    M_live = c < p.M ? (c > 0 ? c : 0) : p.M;
  }
  p.M = M_live;
  const int64_t tilesM = (M_live + TM - 1) / TM;
  // tile t -> (m0, n0): XCD t % 8 takes m-tiles t % 8, + 8, ..., each with its n-tiles
  auto tile_of = [&](int64_t t, int64_t& m0, int64_t& n0) -> bool {
    const int64_t xcd = t % 8, loc = t / 8;
    const int64_t mt = (loc / tilesN) * 8 + xcd;
    m0 = mt * TM;
    n0 = (loc % tilesN) * TN;
    return t < n_tiles && mt < tilesM;
  };
  // the first live tile at or after t on this workgroup's walk (t += gridDim.x); false past the end
  auto next_tile = [&](int64_t& t, int64_t& m0, int64_t& n0) -> bool {
    while (t < n_tiles && !tile_of(t, m0, n0)) t += gridDim.x;
    return t < n_tiles;
  };
  int64_t t = blockIdx.x, m0 = 0, n0 = 0;
  if (!next_tile(t, m0, n0)) return;
  // the dropout stream (a uniform load here, before any DMA is in flight)
  const uint64_t dstream = DROP ? (uint64_t)(LLP_STREAMS_PER_STEP * (*p.drop_ctr) + p.drop_stream) : 0;

  // DMA in SADDR form: a wave-uniform base (the tile's row panel at the K-tile) and a per-lane
  // 32-bit byte offset computed per piece: row q64_row(..) + lane / 8 of the tile, clamped to
  // the tile's last live row (lim), and 16-B chunk (lane % 8) ^ (lane / 8) -- the row's
  // swizzle, as q64_row(..) is a multiple of 8 (no offsets held across the loop)
  const int lr = lane >> 3, lc8 = ((lane & 7) ^ (lane >> 3)) * 8;
  const uint32_t lds0 = lds_u32(smem);
  auto issue_chunk = [&](int j, int buf, int64_t tm0, int64_t tn0, int64_t koff) {
    const bool isA = j == 0 || j == 3;
    const uint32_t base = lds0 + (uint32_t)(buf * TILE_U4 * 16) + (isA ? 0u : IMG_U4 * 16u);
    const bf16_t* sb = isA ? p.A + tm0 * p.lda + koff : p.B + tn0 * p.ldb + koff;
    const int lim = (int)(isA ? min((int64_t)255, p.M - 1 - tm0) : min((int64_t)255, p.N - 1 - tn0));
    const int64_t ld = isA ? p.lda : p.ldb;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row0 = q64_row(j, 16 * wu + 8 * i);
      const uint32_t voff = (uint32_t)((min(row0 + lr, lim) * (int)ld + lc8) * 2);
      glds16_s(voff, sb, __builtin_amdgcn_readfirstlane(base + (uint32_t)(row0 * 128)));
    }
  };
  short8 fa[2][4];
  short8 fb[2][2][2];
  float4_t acc[4][8];
  auto read_a = [&](const uint4* sA, int mh) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int im = 0; im < 4; ++im) {
        const int r = wm * 128 + mh * 64 + im * 16 + li;
        uint4 v = sA[r * 8 + ((kh * 4 + g) ^ (r & 7))];
        fa[kh][im] = *reinterpret_cast<short8*>(&v);
      }
  };
  auto read_b = [&](const uint4* sB, int nh) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int jn = 0; jn < 2; ++jn) {
        const int r = wn * 64 + nh * 32 + jn * 16 + li;
        uint4 v = sB[r * 8 + ((kh * 4 + g) ^ (r & 7))];
        fb[nh][kh][jn] = *reinterpret_cast<short8*>(&v);
      }
  };
  auto mfma_q = [&](int mh, int nh) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int jn = 0; jn < 2; ++jn)
#pragma unroll
        for (int im = 0; im < 4; ++im)
          acc[nh * 2 + jn][mh * 4 + im] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[nh][kh][jn], fa[kh][im], acc[nh * 2 + jn][mh * 4 + im], 0,
                                                      0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  const int64_t nk = p.K / TK;
  const uint32_t ones = 0x00010001u;
  const uint32_t lo16 = __builtin_amdgcn_readfirstlane(0xFFFFu);
  float* blds = reinterpret_cast<float*>(smem + BLDS);
  uint8_t* mlds = reinterpret_cast<uint8_t*>(smem + MLDS);

  // first tile: its K-tile 0 (all four chunks) into buffer 0
#pragma unroll
  for (int j = 0; j < 4; ++j) issue_chunk(j, 0, m0, n0, 0);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // chunks 0, 1 landed
  for (;;) {
    int64_t t_next = t + gridDim.x, m1 = 0, n1 = 0;
    const bool pf = next_tile(t_next, m1, n1);         // the next tile's K-tile 0 issued by this tile's last K-tile
    const int64_t rows = min((int64_t)TM, p.M - m0);  // live rows (the last m-tile may be partial)
    // this tile's bias and (ReLU backward) mask tile into LDS by DMA; older than its K-tile 1
    if (BWD) {
      const uint8_t* ms = p.mask_in + (m0 + min((int64_t)(tid >> 1), rows - 1)) * p.ld_mask + (n0 >> 3) + 16 * (tid & 1);
      glds16(ms, __builtin_amdgcn_readfirstlane(lds_u32(smem + MLDS) + (uint32_t)(wu * 1024)));
    } else {
      if (p.bias && wu == 0) glds16(p.bias + n0 + 4 * lane, __builtin_amdgcn_readfirstlane(lds_u32(smem + BLDS)));
      if (HEAD && wu == 1) glds16(p.head_w + n0 + 4 * lane, __builtin_amdgcn_readfirstlane(lds_u32(smem + HWLDS)));
    }
    barrier();
    if (grp1) barrier();          // waves 4-7: one barrier behind from here on
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) acc[a][b] = float4_t{0.f, 0.f, 0.f, 0.f};
    // one K-tile: 4 quadrant phases; `issue`: DMA chunk j of the K-tile at (tm0, tn0, koff)
    // into buffer nbuf in phase j (the next K-tile, or the next tile's K-tile 0)
    auto ktile = [&](int64_t kt, bool issue, int nbuf, int64_t tm0, int64_t tn0, int64_t koff) {
      const uint4* sA = smem + (int)(kt & 1) * TILE_U4;
      const uint4* sB = sA + IMG_U4;
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      read_a(sA, 0);
      read_b(sB, 0);
      if (issue) issue_chunk(0, nbuf, tm0, tn0, koff);
      barrier();
      mfma_q(0, 0);
      barrier();
      if (issue) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      read_b(sB, 1);
      if (issue) issue_chunk(1, nbuf, tm0, tn0, koff);
      barrier();
      mfma_q(0, 1);
      barrier();
      read_a(sA, 1);
      if (issue) issue_chunk(2, nbuf, tm0, tn0, koff);
      barrier();
      mfma_q(1, 1);
      barrier();
      if (issue) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      if (issue) issue_chunk(3, nbuf, tm0, tn0, koff);
      barrier();
      mfma_q(1, 0);
      barrier();
    };
    for (int64_t kt = 0; kt + 1 < nk; ++kt) ktile(kt, true, (int)((kt + 1) & 1), m0, n0, (kt + 1) * TK);
    // the last K-tile: the next tile's K-tile 0 into buffer 0 (nk is even) when prefetching
    ktile(nk - 1, pf, 0, m1, n1, 0);
    if (!grp1) barrier();         // waves 0-3 match the other half's barrier count
#ifdef LLP_DIAG_EPI_SKIP
    // diagnostic build (tools/gemm_epi_cost.py): no epilogue at all, the accumulators kept live
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) asm volatile("" ::"v"(acc[a][b]));
    if (!pf) return;
    t = t_next; m0 = m1; n0 = n1;
    continue;
#endif
    // ---- lean epilogue in two 128-row halves, staged in [64 KB, 130 KB): buffer 0 receives
    // the next tile's K-tile 0 meanwhile.  Its per-thread addresses derive from an opaque
    // copy of the thread id, so hipcc cannot hoist them above the main loop (where they
    // would hold ~12 VGPRs across it and push the kernel into scratch).
    int etid = tid;
    asm volatile("" : "+v"(etid));
    const int elane = etid & 63, ew = etid >> 6;
    const int eg = elane >> 4, eli = elane & 15, ewm = ew >> 2, ewn = ew & 3;
    constexpr int ROWB = EPI_ROW_U4 * 16;
    float4_t bl[4];
#pragma unroll
    for (int jn = 0; jn < 4; ++jn)
      bl[jn] = (!BWD && p.bias) ? *reinterpret_cast<const float4_t*>(blds + ewn * 64 + jn * 16 + eg * 4)
                                : float4_t{0.f, 0.f, 0.f, 0.f};
    const float2_t al = {p.alpha, p.alpha}, z2 = {0.f, 0.f};
    const int rl0 = etid >> 5, c = etid & 31;
    char* stg = reinterpret_cast<char*>(smem + STG);
    const bool st = !HEAD || p.C != nullptr;           // the head GEMM may store no C
#ifdef LLP_DIAG_EPI_ALIAS
    // diagnostic build (tools/gemm_epi_cost.py): every tile of this workgroup stores into the same
    // 64 rows x 256 columns (rows 64 * blockIdx.x ..; M >= 64 * grid), so its stores stay in L2 and
    // never reach HBM.  C and the mask hold garbage.
    char* cbase = st ? reinterpret_cast<char*>(p.C + (int64_t)blockIdx.x * 64 * p.ldc) : nullptr;
#else
    char* cbase = st ? reinterpret_cast<char*>(p.C + m0 * p.ldc + n0) : nullptr;
#endif
    float* part = reinterpret_cast<float*>(smem + MLDS);   // head: [256 rows][8 quads] partial dots
    float4_t hw0 = {0.f, 0.f, 0.f, 0.f}, hw1 = hw0;
    if (HEAD) {   // this thread's 8 head weights (columns n0 + 8c ..) for the head dot
      hw0 = *reinterpret_cast<const float4_t*>(reinterpret_cast<const float*>(smem + HWLDS) + 8 * (etid & 31));
      hw1 = *reinterpret_cast<const float4_t*>(reinterpret_cast<const float*>(smem + HWLDS) + 8 * (etid & 31) + 4);
    }
    const uint32_t toff = (uint32_t)((rl0 * p.ldc + c * 8) * 2);
    const int64_t cstep = 16 * p.ldc * 2;
    const bool mo = RELU && p.mask_out;
#ifdef LLP_DIAG_EPI_ALIAS
    char* mbase = mo ? reinterpret_cast<char*>(p.mask_out + (int64_t)blockIdx.x * 64 * p.ld_mask) : nullptr;
#else
    char* mbase = mo ? reinterpret_cast<char*>(p.mask_out + m0 * p.ld_mask + (n0 >> 3)) : nullptr;
#endif
    const uint32_t moff = (uint32_t)(rl0 * p.ld_mask + c);
    const int64_t mstep = 16 * p.ld_mask;
    // round h stages the tile's rows [64h, 64h + 64) and [128 + 64h, 128 + 64h + 64): every
    // wave converts half of its accumulators per round (staged row = group * 64 + local row),
    // so no wave group waits out the other's conversion
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      {   // phase 1: this wave's rows (4h + im') * 16 + li of its group's 128, im' < 4
        char* sb = stg + (ewm * 64 + eli) * ROWB + (ewn * 64 + eg * 4) * 2;
        if (DROP) {   // row by row: the keep flags of the row's 16 columns, then its 4 column quads
          const float dsc = p.drop_scale;
#pragma unroll
          for (int iq = 0; iq < 4; ++iq) {
            const int im = 4 * h + iq;
            const uint32_t kb = drop_keep16(p.drop_thresh, p.drop_seed, dstream, m0 + ewm * 128 + im * 16 + eli,
                                            n0 + ewn * 64 + eg * 4, p.N);
#pragma unroll
            for (int jn = 0; jn < 4; ++jn) {
              // before the rounding, as epilogue_t (the ReLU after it: same values and bits)
              float2_t v01 = float2_t{acc[jn][im][0], acc[jn][im][1]} + float2_t{bl[jn][0], bl[jn][1]};
              float2_t v23 = float2_t{acc[jn][im][2], acc[jn][im][3]} + float2_t{bl[jn][2], bl[jn][3]};
              const uint32_t k = kb >> (4 * jn);
              v01[0] = k & 1u ? v01[0] * dsc : 0.f;
              v01[1] = k & 2u ? v01[1] * dsc : 0.f;
              v23[0] = k & 4u ? v23[0] * dsc : 0.f;
              v23[1] = k & 8u ? v23[1] * dsc : 0.f;
              *reinterpret_cast<uint2*>(sb + iq * 16 * ROWB + jn * 32) =
                  make_uint2(relu_pk_bf16(pk_bf16(v01)), relu_pk_bf16(pk_bf16(v23)));
            }
          }
        } else
#pragma unroll
        for (int jn = 0; jn < 4; ++jn) {
          const float2_t b01 = {bl[jn][0], bl[jn][1]}, b23 = {bl[jn][2], bl[jn][3]};
#pragma unroll
          for (int iq = 0; iq < 4; ++iq) {
            const int im = 4 * h + iq;
            float2_t v01 = {acc[jn][im][0], acc[jn][im][1]}, v23 = {acc[jn][im][2], acc[jn][im][3]};
            if (BWD) {
              v01 = __builtin_elementwise_fma(v01, al, z2);
              v23 = __builtin_elementwise_fma(v23, al, z2);
            } else {
              v01 = v01 + b01;
              v23 = v23 + b23;
            }
            uint32_t lo = pk_bf16(v01), hi = pk_bf16(v23);
            if (RELU || HEAD) { lo = relu_pk_bf16(lo); hi = relu_pk_bf16(hi); }
            *reinterpret_cast<uint2*>(sb + iq * 16 * ROWB + jn * 32) = make_uint2(lo, hi);
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      barrier();
      // phase 2: all threads, staged rows rl0 + 16 i (i < 8) of this round
      const char* rb = stg + rl0 * ROWB + c * 16;
      auto run = [&](auto NTS) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          uint4 v = *reinterpret_cast<const uint4*>(rb + i * 16 * ROWB);
#ifdef LLP_DIAG_EPI_ALIAS
          const int ii = (i + 4 * h + (i >= 4 ? 4 : 0)) & 3;   // the aliased 64 rows
#else
          const int ii = i + 4 * h + (i >= 4 ? 4 : 0);   // 16-row group of the tile
#endif
          if (BWD) {
            const uint32_t bits = mlds[(rl0 + 16 * ii) * 32 + c];
            v.x &= half_mask<0>(bits, lo16);
            v.y &= half_mask<2>(bits, lo16);
            v.z &= half_mask<4>(bits, lo16);
            v.w &= half_mask<6>(bits, lo16);
          }
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 sv = {v.x, v.y, v.z, v.w};
          u32x4* dst = reinterpret_cast<u32x4*>(cbase + ii * cstep + toff);
          const bool live = rl0 + 16 * ii < rows;
#ifdef LLP_DIAG_EPI_NOSTORE
          // diagnostic build (tools/gemm_epi_cost.py): the staged values are read, not stored
          asm volatile("" ::"v"(sv), "v"(dst));
          (void)live;
#else
          if (live && st) {
            if constexpr (decltype(NTS)::value) __builtin_nontemporal_store(sv, dst);
            else *dst = sv;
          }
#endif
          if (RELU) {
            if (mo) {
              const uint32_t u = nz_pk_u16(v.x, ones) | (nz_pk_u16(v.y, ones) << 2) | (nz_pk_u16(v.z, ones) << 4) |
                                 (nz_pk_u16(v.w, ones) << 6);
              const uint32_t word = quad_pack_bytes((u | (u >> 15)) & 0xFFu);
              if ((c & 3) == 0 && live) *reinterpret_cast<uint32_t*>(mbase + ii * mstep + moff) = word;
            }
          }
          if (HEAD) {   // epilogue_lean_head's dot of the 8 rounded outputs, same order
            float d = __uint_as_float(v.x << 16) * hw0[0];
            d = fmaf(__uint_as_float(v.x & 0xFFFF0000u), hw0[1], d);
            d = fmaf(__uint_as_float(v.y << 16), hw0[2], d);
            d = fmaf(__uint_as_float(v.y & 0xFFFF0000u), hw0[3], d);
            d = fmaf(__uint_as_float(v.z << 16), hw1[0], d);
            d = fmaf(__uint_as_float(v.z & 0xFFFF0000u), hw1[1], d);
            d = fmaf(__uint_as_float(v.w << 16), hw1[2], d);
            d = fmaf(__uint_as_float(v.w & 0xFFFF0000u), hw1[3], d);
            d = dpp_quad_sum(d);
            if ((c & 3) == 0) part[(rl0 + 16 * ii) * 8 + (c >> 2)] = d;
          }
        }
      };
      if (p.nt_store) run(std::true_type{});
      else run(std::false_type{});
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      barrier();
    }
    if (HEAD && etid < rows) {   // the row's 8 quad partials in column order (epilogue_lean_head)
      const float4_t a = *reinterpret_cast<const float4_t*>(part + etid * 8);
      const float4_t b = *reinterpret_cast<const float4_t*>(part + etid * 8 + 4);
      p.head_part[(n0 / TN) * p.head_ld + m0 + etid] = ((a[0] + a[1]) + (a[2] + a[3])) + ((b[0] + b[1]) + (b[2] + b[3]));
    }
    if (!pf) return;
    // the next tile: its K-tile 0 was issued by this tile's last K-tile.  This wait only
    // bounds the stores in flight; correctness rests on the next tile's first K-tile wait
    // (vmcnt(2)), which the epilogue's stores and the bias / mask DMA, all younger than the
    // prefetch, can only make wait longer.  (Leaving a full tile's 16 stores per wave in
    // flight through the next tile's first two waits measured 1 % SLOWER on the collab
    // step, 3 interleaved rounds each: the stores then compete with that K-tile's DMA.)
    t = t_next; m0 = m1; n0 = n1;
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  }
}

// the epilogue specialisation a call can use (epilogue_t)
int epi_mode_of(const P256& p) {
  if (p.drop_p > 0.f) return EPI_ANY;
  if (p.head_w)
    return p.act == LLP_ACT_RELU && p.alpha == 1.f && !p.aux && !p.mask_in && !p.mask_out ? EPI_HEAD_RELU : EPI_ANY;
  if (!p.C) return EPI_ANY;
  if (p.act == LLP_ACT_RELU && p.alpha == 1.f && !p.aux && !p.mask_in) return EPI_FWD_RELU;
  if (p.act == LLP_ACT_NONE && p.alpha == 1.f && !p.aux && !p.mask_in && !p.mask_out) return EPI_FWD_NONE;
  if (p.act == LLP_ACT_RELU_BWD && p.mask_in && !p.bias && !p.mask_out) return EPI_BWD_MASK;
  return EPI_ANY;
}

// Split-K epilogue: thread (row, 8-column chunk) sums the S slabs in order (slab 0
// first), adds the bias, rounds to bf16 (RNE) and applies the lean epilogue's ReLU
// (sign-bit rule), stores 16 B of C and, with a mask, the chunk's ReLU bit byte
// (bit i = column 8c + i is nonzero).  Deterministic; the sum differs from the
// unsplit kernel's only in where the K-range partial sums are added.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(int64_t M, int64_t N, int S, const float* __restrict__ slab,
                                                            const float* __restrict__ bias, int relu,
                                                            bf16_t* __restrict__ C, int64_t ldc,
                                                            uint8_t* __restrict__ mask_out, int64_t ld_mask) {
  const int64_t cpr = N / 8;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= M * cpr) return;
  const int64_t row = i / cpr, c = i % cpr;
  const float* src = slab + row * N + c * 8;
  float4_t a = *reinterpret_cast<const float4_t*>(src), b = *reinterpret_cast<const float4_t*>(src + 4);
  for (int s = 1; s < S; ++s) {
    a += *reinterpret_cast<const float4_t*>(src + (int64_t)s * M * N);
    b += *reinterpret_cast<const float4_t*>(src + (int64_t)s * M * N + 4);
  }
  if (bias) {
    a += *reinterpret_cast<const float4_t*>(bias + c * 8);
    b += *reinterpret_cast<const float4_t*>(bias + c * 8 + 4);
  }
  uint32_t w0 = pk_bf16(float2_t{a[0], a[1]}), w1 = pk_bf16(float2_t{a[2], a[3]});
  uint32_t w2 = pk_bf16(float2_t{b[0], b[1]}), w3 = pk_bf16(float2_t{b[2], b[3]});
  if (relu) {
    w0 = relu_pk_bf16(w0); w1 = relu_pk_bf16(w1); w2 = relu_pk_bf16(w2); w3 = relu_pk_bf16(w3);
  }
  *reinterpret_cast<uint4*>(C + row * ldc + c * 8) = make_uint4(w0, w1, w2, w3);
  if (mask_out) {
    const uint32_t w[4] = {w0, w1, w2, w3};
    uint32_t byte = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      byte |= ((w[k] & 0xFFFFu) ? 1u : 0u) << (2 * k) | ((w[k] >> 16) ? 1u : 0u) << (2 * k + 1);
    mask_out[row * ld_mask + c] = (uint8_t)byte;
  }
}

}  // namespace

// CUs of the current device, queried once per device (a race only repeats the query)
int llp_cu_count() {
  static int cus_of[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  int cus = cus_of[dev];
  if (cus <= 0) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    cus_of[dev] = cus;
  }
  return cus;
}

// one workgroup per CU (the persistent kernel's grid)
static dim3 persistent_grid(int64_t tiles) {
  const int cus = llp_cu_count();
  return dim3((unsigned)(tiles < cus ? tiles : cus));
}

// Split-K bf16 GEMM (llp_gemm_nt_splitk, gemm.hip): pp8<EPI_PARTIAL> over (tiles, S)
// into f32 slabs, then splitk_reduce_kernel.  The caller checked the shapes.
int llp_gemm_nt_bf16_splitk(const llp_operand* A, const llp_operand* B, int64_t M, int64_t N, int64_t K, void* C,
                            int64_t ldc, const float* bias, int relu, uint8_t* mask_out, int64_t ld_mask, int S,
                            float* slab, hipStream_t s) {
  P256 p = {};
  p.A = (const bf16_t*)A->ptr; p.lda = A->ld;
  p.B = (const bf16_t*)B->ptr; p.ldb = B->ld;
  p.M = M; p.N = N; p.K = K;
  p.C = (bf16_t*)C; p.ldc = ldc;
  p.alpha = 1.f;
  p.head_part = slab;
  p.head_ld = M;
  const int64_t tiles = ((M + TM - 1) / TM) * (N / TN);
  hipLaunchKernelGGL(gemm_nt_bf16_pp8<EPI_PARTIAL>, dim3((unsigned)tiles, (unsigned)S), dim3(NT2), 0, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const int64_t n = M * (N / 8);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, M, N, S, slab, bias,
                     relu, (bf16_t*)C, ldc, mask_out, ld_mask);
  return (int)hipGetLastError();
}

// Called from llp_gemm_nt when the shapes allow it (gemm.hip).
int llp_gemm_nt_bf16_256(const llp_operand* A, const llp_operand* B, int64_t M, int64_t N, int64_t K, void* C,
                         int64_t ldc, const float* bias, int act, const void* aux, int64_t ld_aux, float alpha,
                         float drop_p, uint32_t drop_thresh, float drop_scale, uint64_t drop_seed,
                         const int64_t* drop_ctr, int64_t drop_stream, const float* head_w, float* head_part,
                         uint8_t* mask_out, const uint8_t* mask_in, int64_t ld_mask, hipStream_t s) {
  P256 p;
  p.head_w = head_w;
  p.head_part = head_part;
  p.mask_out = mask_out;
  p.mask_in = mask_in;
  p.ld_mask = ld_mask;
  if ((head_w || !C) && A->ptr2) return (int)hipErrorInvalidValue;   // fused head: pipelined kernel only
  p.A = (const bf16_t*)A->ptr; p.ia = A->idx; p.A2 = (const bf16_t*)A->ptr2; p.ia2 = A->idx2;
  p.lda = A->ld; p.lda2 = A->ptr2 ? A->ld2 : 0;
  p.B = (const bf16_t*)B->ptr; p.ib = B->idx; p.ldb = B->ld;
  p.M = M; p.N = N; p.K = K;
  p.m_dev = A->rows_dev;
  p.head_ld = M;
  p.nt_store = 1;   // non-temporal epilogue stores: +20 % on the write-bound K=128 layer, level at K=1024
  p.lean_epi = 1;
  p.C = (bf16_t*)C; p.ldc = ldc;
  p.bias = bias; p.act = act; p.aux = (const bf16_t*)aux; p.ld_aux = ld_aux; p.alpha = alpha;
  p.drop_p = drop_p; p.drop_thresh = drop_thresh; p.drop_scale = drop_scale; p.drop_seed = drop_seed;
  p.drop_ctr = drop_ctr; p.drop_stream = drop_stream;
  // with a device row count pp8 maps the host grid interleaved over the XCDs
  // (tile_256_host_interleaved): m-tiles padded to a multiple of 8; the Hadamard-operand
  // kernel maps the live tiles and lets the surplus blocks exit
  const int64_t tiles = (A->rows_dev ? ((M + 8 * TM - 1) / (8 * TM)) * 8 : (M + TM - 1) / TM) * ((N + TN - 1) / TN);
  const dim3 grid((unsigned)tiles), block(NT2);
  if (A->ptr2) {   // A = A1[ia] * A2[ia2] formed on load (rows whose width is not a multiple of 8)
    llp::note_kernel("gemm_nt_bf16_256<hadamard A>");
    hipLaunchKernelGGL(gemm_nt_bf16_256<true>, grid, block, 0, s, p);
    return (int)hipGetLastError();
  }
  const int mode = epi_mode_of(p);
#ifndef LLP_GEMM_NO_PERSISTENT
  // ReLU + dropout forward with an optional ReLU mask out (the teacher's hidden layers)
  const bool drop_lean = mode == EPI_ANY && p.drop_p > 0.f && !head_w && C && act == LLP_ACT_RELU &&
                         alpha == 1.f && !aux && !mask_in;
  // persistent form for the lean modes (plain operands, an even number of K-tiles): one
  // workgroup per CU walks its tiles with the next tile's first K-tile prefetched
  const bool lean_shapes = N % TN == 0 && !(ldc & 7) && !((uintptr_t)C & 15) &&
                           ((mode != EPI_FWD_RELU && !drop_lean) || !mask_out ||
                            (!(ld_mask & 3) && !((uintptr_t)mask_out & 3))) &&
                           (mode != EPI_BWD_MASK || (!(ld_mask & 15) && !((uintptr_t)mask_in & 15))) &&
                           (!bias || !((uintptr_t)bias & 15));
  if (drop_lean && lean_shapes && !A->idx && !B->idx && (K / TK) % 2 == 0 && tiles > 256) {
    llp::note_kernel("gemm_nt_bf16_pp8p<EPI_FWD_DROP> (persistent)");
    hipLaunchKernelGGL((gemm_nt_bf16_pp8p<EPI_FWD_DROP>), persistent_grid(tiles), block, 0, s, p);
    return (int)hipGetLastError();
  }
  if ((mode == EPI_FWD_RELU || mode == EPI_FWD_NONE || mode == EPI_BWD_MASK) && lean_shapes && !A->idx && !B->idx &&
      (K / TK) % 2 == 0 && tiles > 256) {
    const dim3 pgrid = persistent_grid(tiles);
    llp::note_kernel(mode == EPI_FWD_RELU   ? "gemm_nt_bf16_pp8p<EPI_FWD_RELU> (persistent)"
                     : mode == EPI_FWD_NONE ? "gemm_nt_bf16_pp8p<EPI_FWD_NONE> (persistent)"
                                            : "gemm_nt_bf16_pp8p<EPI_BWD_MASK> (persistent)");
    if (mode == EPI_FWD_RELU) hipLaunchKernelGGL((gemm_nt_bf16_pp8p<EPI_FWD_RELU>), pgrid, block, 0, s, p);
    else if (mode == EPI_FWD_NONE) hipLaunchKernelGGL((gemm_nt_bf16_pp8p<EPI_FWD_NONE>), pgrid, block, 0, s, p);
    else hipLaunchKernelGGL((gemm_nt_bf16_pp8p<EPI_BWD_MASK>), pgrid, block, 0, s, p);
    return (int)hipGetLastError();
  }
#endif
  llp::note_kernel(mode == EPI_FWD_RELU   ? "gemm_nt_bf16_pp8<EPI_FWD_RELU>"
                   : mode == EPI_FWD_NONE ? "gemm_nt_bf16_pp8<EPI_FWD_NONE>"
                   : mode == EPI_BWD_MASK ? "gemm_nt_bf16_pp8<EPI_BWD_MASK>"
                   : mode == EPI_HEAD_RELU ? "gemm_nt_bf16_pp8<EPI_HEAD_*>"
                                           : "gemm_nt_bf16_pp8<EPI_ANY>");
  switch (mode) {
    case EPI_FWD_RELU: hipLaunchKernelGGL((gemm_nt_bf16_pp8<EPI_FWD_RELU>), grid, block, 0, s, p); break;
    case EPI_FWD_NONE: hipLaunchKernelGGL((gemm_nt_bf16_pp8<EPI_FWD_NONE>), grid, block, 0, s, p); break;
    case EPI_BWD_MASK: hipLaunchKernelGGL((gemm_nt_bf16_pp8<EPI_BWD_MASK>), grid, block, 0, s, p); break;
    case EPI_HEAD_RELU:
#ifndef LLP_GEMM_NO_PERSISTENT
      if (N % TN == 0 && !((uintptr_t)head_w & 15) && (!C || (!(ldc & 7) && !((uintptr_t)C & 15))) &&
          (!bias || !((uintptr_t)bias & 15)) && !A->idx && !B->idx && (K / TK) % 2 == 0 && tiles > 256) {
        hipLaunchKernelGGL((gemm_nt_bf16_pp8p<EPI_HEAD_LEAN>), persistent_grid(tiles), block, 0, s, p);
        break;
      }
#endif
      // the head dot over the staged bf16 outputs (epilogue_lean_head) on every tile when
      // the shapes allow: 650 -> 643 us per predictor-layer launch, collab step -0.3 %
      // (3 interleaved rounds, profiles/r03_head_lean_ab.txt)
      if (N % TN == 0 && !((uintptr_t)head_w & 15) && (!C || (!(ldc & 7) && !((uintptr_t)C & 15))))
        hipLaunchKernelGGL((gemm_nt_bf16_pp8<EPI_HEAD_LEAN>), grid, block, 0, s, p);
      else
        hipLaunchKernelGGL((gemm_nt_bf16_pp8<EPI_HEAD_RELU>), grid, block, 0, s, p);
      break;
    default:
#ifndef LLP_GEMM_NO_PERSISTENT
      // ReLU + dropout + fused head (the teacher predictor's hidden layer in training)
      if (p.drop_p > 0.f && head_w && act == LLP_ACT_RELU && alpha == 1.f && !aux && !mask_in && !mask_out &&
          N % TN == 0 && !((uintptr_t)head_w & 15) && (!C || (!(ldc & 7) && !((uintptr_t)C & 15))) &&
          (!bias || !((uintptr_t)bias & 15)) && !A->idx && !B->idx && (K / TK) % 2 == 0 && tiles > 256) {
        llp::note_kernel("gemm_nt_bf16_pp8p<EPI_HEAD_DROP> (persistent)");
        hipLaunchKernelGGL((gemm_nt_bf16_pp8p<EPI_HEAD_DROP>), persistent_grid(tiles), block, 0, s, p);
        break;
      }
#endif
      hipLaunchKernelGGL((gemm_nt_bf16_pp8<EPI_ANY>), grid, block, 0, s, p);
  }
  return (int)hipGetLastError();
}

#ifdef LLP_GEMM_STAMPS
extern "C" int llp_debug_gemm_stamps(unsigned long long* host, int64_t n_blocks) {
  const int64_t n = n_blocks < STAMP_MAX ? n_blocks : STAMP_MAX;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_llp_stamps), (size_t)n * 8 * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}
#endif
