// Persistent 256 x 256 bf16 NT GEMM at ONE wave per SIMD (round 6) -- the student MLP /
// LinkPredictor Linear layers and their data gradients (src/models.py:48,143):
//
//   C[m, n] = epi(alpha * sum_k A[m, k] * B[n, k])      bf16 in, f32 accumulate, bf16 out
//
// Why this structure.  The eight-wave ping-pong kernel (gemm256.hip pp8p)
// keeps its MFMA pipes 54 % busy: one wave of each SIMD pair is parked at a barrier while the
// other computes, by design.  One wave per SIMD with a 128 x 128 tile per wave holds 256 f32
// accumulators per lane (AGPRs, through inline-asm v_mfma_f32_32x32x16_bf16 so hipcc never
// copies them) and issues every MFMA itself.  What that wave cannot afford is LDS-DMA:
// llp_stage_probe (csrc/probe.hip, profiles/r06_stage_probe.jsonl) measured a
// global_load_lds_dwordx4 piece beside back-to-back 32x32x16 MFMAs at 61.6 -> 106 shader cycles
// per MFMA (floor 32.1) for 4 -> 16 pieces per 32 MFMAs, while global_load_dwordx4 into VGPRs
// plus ds_write_b128 cost nothing measurable at the same rates (32.15-32.18).  So the operands
// are register-staged: a K-tile (64 deep: A and B images of [256 rows][128 B], 64 KiB) is
// global-loaded into one of two VGPR staging sets three K-tiles ahead, written to one of two
// LDS slots one K-tile ahead, and read as MFMA fragments from the current slot.
//
// Per K-tile and wave: 64 MFMAs (4 k-steps x 4 x 4 tiles of 32 x 32), 32 ds_read_b128 fragment
// reads (the next k-step's, one every other MFMA), 16 ds_write_b128 (the next K-tile, k-step 2)
// and 16 global_load_dwordx4 (K-tile + 3, k-step 3), and ONE barrier (inside k-step 3, after
// every wave's writes of the next K-tile and reads of this one): RAW for the next K-tile's slot,
// WAR for this one.  LDS images: 128-B rows, 16-B chunk c of row r at chunk c ^ ((r >> 1) & 7):
// conflict-free for both the ds_write pattern (8 rows x 128 B per instruction) and the 32 x 32
// fragment reads (16 consecutive rows, one chunk).  The K-tile stream runs across the
// persistent walk's tiles: the next tile's first K-tiles are loaded and written while this one
// computes, so only the epilogue stops the MFMA pipes.
//
// Fragments (v_mfma_f32_32x32x16_bf16): src0 = weight rows (B), src1 = activation rows (A);
// lane l supplies row l % 32 of its 32-row block, k = 8 (l / 32) .. + 7 of the k-step.  D: lane
// l holds output row l % 32 of the block and, for value k = 0..15, column
// 8 (k / 4) + 4 (l / 32) + (k % 4): four runs of 4 consecutive columns.
#include "llp_common.h"

#include <utility>

int llp_cu_count();

namespace {

typedef float w4_f32x16 __attribute__((ext_vector_type(16)));
typedef float w4_float2 __attribute__((ext_vector_type(2)));
typedef short w4_short2 __attribute__((ext_vector_type(2)));
typedef __bf16 w4_bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int w4_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int w4_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char w4_lds_c;
typedef __attribute__((address_space(3))) short8 w4_lds_s8;
typedef __attribute__((address_space(3))) w4_u32x4 w4_lds_u4;
typedef __attribute__((address_space(3))) float4_t w4_lds_f4;

constexpr int WT = 256;                    // tile rows / columns
constexpr int WK = 64;                     // K-tile
constexpr int WTHR = 256;                  // four waves, one per SIMD
// LDS: A images of slots 0 / 1 at 0 / 32 KiB, B images at 64 / 96 KiB (every fragment and
// staging offset past a per-lane base fits the 16-bit ds offset field), then the f32 bias of
// every column
constexpr int WB_OFF = 65536;
constexpr int WSLOT = 32768;
constexpr int WBIAS = 131072;
constexpr int WBIAS_MAX = 4096;            // columns whose bias the LDS tail holds
constexpr int W_RELU = 1, W_NONE = 2, W_BWD = 3;

struct PW4 {
  const bf16_t* A; int64_t lda;
  const bf16_t* B; int64_t ldb;
  int64_t M, N, K;
  bf16_t* C; int64_t ldc;
  const float* bias;
  float alpha;
  uint8_t* mask_out;        // W_RELU: ReLU bit mask out (bit i of byte c = column 8c + i nonzero)
  const uint8_t* mask_in;   // W_BWD: the ReLU bit mask of the layer's forward
  int64_t ld_mask;
  const int32_t* m_dev;     // device row count or NULL
};

__device__ __forceinline__ void w4_mfma(w4_f32x16& c, const short8& w, const short8& x) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(w), "v"(x) : "memory");
}
__device__ __forceinline__ void w4_mfma0(w4_f32x16& c, const short8& w, const short8& x) {   // C = 0
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(w), "v"(x) : "memory");
}
__device__ __forceinline__ uint32_t w4_pk_bf16(float a, float b) {   // v_cvt_pk_bf16_f32 (RNE, as f2bf)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((w4_float2){a, b}, w4_bf16x2));
}
__device__ __forceinline__ uint32_t w4_relu_pk(uint32_t x) {   // sign-bit ReLU on a bf16 pair (pp8p's rule)
  const w4_short2 r = __builtin_elementwise_max(__builtin_bit_cast(w4_short2, x), (w4_short2){0, 0});
  return __builtin_bit_cast(uint32_t, r);
}

// compile-time loop: f(std::integral_constant<int, i>) for i = 0 .. N-1 (every register-array index
// below must be a constant, or hipcc moves the staging / fragment arrays to scratch)
__device__ __forceinline__ uint32_t w4_nz_pk(uint32_t x) {   // v_pk_min_u16(x, 0x00010001): 1 per nonzero half
  uint32_t r;   // (an inline constant 1 would reach the low half only: op_sel_hi takes its upper 16 bits)
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(x), "s"(0x00010001u));
  return r;
}

template <typename F, int... I>
__device__ __forceinline__ void w4_sfor_impl(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void w4_sfor(F&& f) {
  w4_sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// DIAG (diagnostic A/B builds through llp_gemm_nt_w4_probe only; wrong outputs): bit 1 no
// staging loads in the loop, 2 no staging writes, 4 no barrier, 8 no fragment reads, 16 no epilogue
template <int MODE, int DIAG = 0>
__global__ __launch_bounds__(WTHR, 1) void gemm_nt_bf16_w4(PW4 p) {
  constexpr bool RELU = MODE == W_RELU;
  constexpr bool BWD = MODE == W_BWD;
  __shared__ __attribute__((aligned(16))) uint4 smem[(WBIAS + 4 * WBIAS_MAX) / 16];
  w4_lds_c* sb = (w4_lds_c*)((__attribute__((address_space(3))) uint4*)smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int hi = lane >> 5, l32 = lane & 31;

  const int64_t tilesN = p.N / WT;
  const int64_t tilesM_host = (p.M + WT - 1) / WT;
  const int64_t n_tiles = (tilesM_host + 7) / 8 * 8 * tilesN;
  int64_t M_live = p.M;
  if (p.m_dev) {
    const int64_t c = *p.m_dev;
    M_live = c < p.M ? (c > 0 ? c : 0) : p.M;
  }
  const int64_t tilesM = (M_live + WT - 1) / WT;
  // tile t -> (m0, n0): XCD t % 8 takes m-tiles t % 8, + 8, ..., each with its n-tiles (pp8p's walk)
  auto tile_of = [&](int64_t t, int64_t& m0, int64_t& n0) __attribute__((always_inline)) -> bool {
    const int64_t xcd = t % 8, loc = t / 8;
    const int64_t mt = (loc / tilesN) * 8 + xcd;
    m0 = mt * WT;
    n0 = (loc % tilesN) * WT;
    return t < n_tiles && mt < tilesM;
  };
  auto next_tile = [&](int64_t& t, int64_t& m0, int64_t& n0) __attribute__((always_inline)) -> bool {
    while (t < n_tiles && !tile_of(t, m0, n0)) t += gridDim.x;
    return t < n_tiles;
  };
  int64_t t_cur = blockIdx.x, m0 = 0, n0 = 0;
  if (!next_tile(t_cur, m0, n0)) return;
  const int nk = (int)(p.K / WK);

  // bias of every column into the LDS tail (once; zeros without a bias: the epilogue adds it
  // unconditionally)
  if (!BWD) {
    for (int c = tid * 4; c < (int)p.N; c += WTHR * 4)
      *reinterpret_cast<w4_lds_f4*>(sb + WBIAS + 4 * c) =
          p.bias ? *reinterpret_cast<const float4_t*>(p.bias + c) : float4_t{0.f, 0.f, 0.f, 0.f};
  }

  // ---- the K-tile load stream (three K-tiles ahead of the compute), across the walk's tiles.
  // Past the walk's end it keeps re-reading the last live tile's addresses (in bounds, never used).
  int64_t ls_t = t_cur, ls_m0 = m0, ls_n0 = n0;
  int ls_k = 0;
  auto ls_advance = [&]() __attribute__((always_inline)) {
    if (++ls_k == nk) {
      int64_t t2 = ls_t + gridDim.x, a = 0, b = 0;
      if (next_tile(t2, a, b)) {
        ls_t = t2; ls_m0 = a; ls_n0 = b; ls_k = 0;
      } else {
        ls_k = nk - 1;
      }
    }
  };
  // staging piece i of the K-tile at (ls_m0, ls_n0, ls_k): i < 8 A rows 64 w + 8 i + lane / 8, else B
  // rows; 16 B = logical chunk lane % 8 of the row's 128-B segment.  Buffer loads: a 32-bit lane
  // offset plus a uniform part, and the descriptors' range (A: the live rows) returns 0 past the
  // last live row of a partial tile (never stored) instead of reading past the operand
  const int lr = lane >> 3, lc = lane & 7;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.A), 0,
                                                                       (int)(M_live * p.lda * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.B), 0,
                                                                       (int)(p.N * p.ldb * 2), 0x00020000);
  const uint32_t vA = (uint32_t)(((64 * w + lr) * p.lda + lc * 8) * 2);
  const uint32_t vB = (uint32_t)(((64 * w + lr) * p.ldb + lc * 8) * 2);
  w4_u32x4 stg[2][16];   // (a native vector type: hipcc keeps HIP_vector_type arrays in scratch)
  auto load_piece = [&](auto SET, auto I) __attribute__((always_inline)) {
    constexpr int set = decltype(SET)::value, i = decltype(I)::value;
    if constexpr (DIAG & 1) return;
    if constexpr (i < 8) {
      const uint32_t u = (uint32_t)(((ls_m0 + 8 * i) * p.lda + ls_k * WK) * 2);
      stg[set][i] = __builtin_bit_cast(w4_u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, (int)(vA + u), 0, 0));
    } else {
      const uint32_t u = (uint32_t)(((ls_n0 + 8 * (i - 8)) * p.ldb + ls_k * WK) * 2);
      stg[set][i] = __builtin_bit_cast(w4_u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsB, (int)(vB + u), 0, 0));
    }
  };
  // LDS write offsets (slot 0): row 64 w + 8 i + lane / 8, physical chunk lc ^ ((row >> 1) & 7);
  // (row >> 1) & 7 = (4 (i & 1) + lane / 16) & 7
  uint32_t woff[2];
#pragma unroll
  for (int par = 0; par < 2; ++par)
    woff[par] = (uint32_t)((64 * w + lr) * 128 + ((lc ^ ((4 * par + (lane >> 4)) & 7)) << 4));
  auto write_piece = [&](auto SET, auto SLOT, auto I) __attribute__((always_inline)) {
    constexpr int set = decltype(SET)::value, slot = decltype(SLOT)::value, i = decltype(I)::value;
    constexpr int ii = i & 7;
    constexpr uint32_t c = (uint32_t)(ii * 1024 + slot * WSLOT + (i >= 8 ? WB_OFF : 0));
    if constexpr (DIAG & 2) return;
    *reinterpret_cast<w4_lds_u4*>(sb + woff[ii & 1] + c) = stg[set][i];
  };
  // fragment read offsets (slot 0) per k-step: row (lane % 32) of a 32-row block, logical chunk
  // 2 ks + lane / 32 at physical (2 ks + hi) ^ (((lane % 32) >> 1) & 7)
  uint32_t roffA[4], roffB[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const uint32_t lp = (uint32_t)(l32 * 128 + (((2 * ks + hi) ^ ((l32 >> 1) & 7)) << 4));
    roffA[ks] = lp + (uint32_t)(wm * 128 * 128);
    roffB[ks] = lp + (uint32_t)(wn * 128 * 128 + WB_OFF);
  }
  short8 fa[2][4], fb[2][4];
  auto read_frag = [&](auto F, auto IDX, auto SLOT, auto KS) __attribute__((always_inline)) {
    constexpr int f = decltype(F)::value, idx = decltype(IDX)::value, slot = decltype(SLOT)::value;
    constexpr int ks = decltype(KS)::value;
    if constexpr (DIAG & 8) return;
    if constexpr (idx < 4)
      fa[f][idx] = *reinterpret_cast<w4_lds_s8*>(sb + roffA[ks] + (uint32_t)(slot * WSLOT + idx * 4096));
    else
      fb[f][idx - 4] = *reinterpret_cast<w4_lds_s8*>(sb + roffB[ks] + (uint32_t)(slot * WSLOT + (idx - 4) * 4096));
  };
  w4_f32x16 acc[4][4];
  auto mfma_j = [&](auto F, auto J, auto FIRST) __attribute__((always_inline)) {
    constexpr int f = decltype(F)::value, j = decltype(J)::value;
    constexpr int im = j >> 2, jn = j & 3;
    if constexpr (decltype(FIRST)::value) w4_mfma0(acc[im][jn], fb[f][jn], fa[f][im]);
    else w4_mfma(acc[im][jn], fb[f][jn], fa[f][im]);
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  using NO = std::false_type;

  // ---- prologue: K-tiles 0, 1 into the staging sets, K-tile 0 into slot 0, K-tile 2 into set 0,
  // then the first k-step's fragments
  w4_sfor<16>([&](auto I) __attribute__((always_inline)) { load_piece(C0{}, I); });
  ls_advance();
  w4_sfor<16>([&](auto I) __attribute__((always_inline)) { load_piece(C1{}, I); });
  ls_advance();
  w4_sfor<16>([&](auto I) __attribute__((always_inline)) { write_piece(C0{}, C0{}, I); });
  w4_sfor<16>([&](auto I) __attribute__((always_inline)) { load_piece(C0{}, I); });
  ls_advance();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  w4_sfor<8>([&](auto I) __attribute__((always_inline)) { read_frag(C0{}, I, C0{}, C0{}); });

  // one K-tile in slot S (compile-time), its k-step-0 fragments in set 0 on entry; leaves the
  // next K-tile's k-step-0 fragments in set 0, its data in slot 1 - S, K-tile + 3 in flight.
  // Flat schedule over the K-tile's 64 MFMAs (J = 16 ks + j; set ks & 1 holds k-step ks):
  //  * J = 3i (i < 16): ds_write staging piece i of the next K-tile (set 1 - S) into slot 1 - S
  //    (free since the last barrier); J = 3i + 1: reload that register with piece i of K-tile + 3
  //    (spread over k-steps 0-2: writes and reads together at one LDS op per gap saturated the
  //    LDS queue, SQ_WAIT_INST_LDS 18 % of wave cycles);
  //  * even j of k-steps 0-2: one fragment read of k-step ks + 1 (set (ks + 1) & 1), in the order
  //    the next k-step's MFMAs take them (a0, b0, b1, b2, b3, a1, a2, a3);
  //  * after MFMA 51 (k-step 3, j = 3): lgkmcnt(0) + barrier (every wave's writes of the next
  //    K-tile and reads of this one are done), then J = 52..59: the next K-tile's k-step-0 reads.
  auto kiter = [&](auto S_, auto FIRST_) __attribute__((always_inline)) {
    constexpr int S = decltype(S_)::value;
    using NS = std::integral_constant<int, 1 - S>;
    w4_sfor<64>([&](auto J_) __attribute__((always_inline)) {
      constexpr int J = decltype(J_)::value;
      constexpr int ks = J / 16, j = J % 16;
      constexpr int ridx_tab[8] = {0, 4, 5, 6, 7, 1, 2, 3};   // a0 b0 b1 b2 b3 a1 a2 a3
      if constexpr (ks == 0)
        mfma_j(C0{}, std::integral_constant<int, j>{}, FIRST_);
      else
        mfma_j(std::integral_constant<int, ks & 1>{}, std::integral_constant<int, j>{}, NO{});
      if constexpr (J < 48) {   // one staging piece per 3 MFMAs: LDS at <= 0.75 ops per MFMA gap
        if constexpr (J % 3 == 0) write_piece(NS{}, NS{}, std::integral_constant<int, J / 3>{});
        else if constexpr (J % 3 == 1) load_piece(NS{}, std::integral_constant<int, J / 3>{});
      }
      if constexpr (J == 46) ls_advance();
      if constexpr (DIAG & 32) {   // A/B: the next k-step's reads on MFMAs 0-7 (one per gap)
        if constexpr (ks < 3 && j < 8)
          read_frag(std::integral_constant<int, (ks + 1) & 1>{}, std::integral_constant<int, ridx_tab[j]>{}, S_,
                    std::integral_constant<int, ks + 1>{});
      } else if constexpr (ks < 3 && (j & 1) == 0) {
        read_frag(std::integral_constant<int, (ks + 1) & 1>{}, std::integral_constant<int, ridx_tab[j / 2]>{}, S_,
                  std::integral_constant<int, ks + 1>{});
      }
      if constexpr (J == 51) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (!(DIAG & 4)) __builtin_amdgcn_s_barrier();
      }
      if constexpr (J >= 52 && J < 60)
        read_frag(C0{}, std::integral_constant<int, ridx_tab[J - 52]>{}, NS{}, C0{});
    });
  };

  for (;;) {
    kiter(C0{}, std::true_type{});
    for (int t = 1; t + 1 < nk; t += 2) {
      kiter(C1{}, NO{});
      kiter(C0{}, NO{});
    }
    kiter(C1{}, NO{});

    // ---- epilogue straight from the accumulators (the last MFMA's D -> v_accvgpr_read: 18 wait
    // states).  Lane (l32, hi) of block (im, jn): row m0 + 128 wm + 32 im + l32, columns
    // n0 + 128 wn + 32 jn + 8 q + 4 hi + (0..3) for q = 0..3 (values 4 q .. 4 q + 3).
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
    if constexpr ((DIAG & 16) != 0) {
      // (the MFMAs are volatile asm: skipping the epilogue deletes none of them)
    } else {
    // Per lane: row m0 + 128 wm + 32 im + l32; columns cb + 8 q + 4 hi + (0..3), cb = n0 + 128 wn + 32 jn.
    // Stores through LDS, one 32-row block (im) at a time: the lane's 8-B pieces into a row-major
    // [32][272 B] image in its wave's 16 KiB of slot 1 (free from the last K-tile's barrier to the
    // next tile's first staging write, which a barrier below orders), then 16 B per lane, 16 lanes
    // per 256-B row: 8 dwordx4 stores of 4 full rows each instead of 16 dwordx2 stores that each
    // touch 32 rows (the row-per-lane pattern was store-issue-bound: 0.21 ms of a 0.58 ms launch).
    const int64_t row0 = m0 + 128 * wm + l32;
    const int64_t col0 = n0 + 128 * wn + 4 * hi;
    const w4_lds_c* bl = sb + WBIAS + 4 * (uint32_t)col0;   // + (32 jn + 8 q) * 4: constant offsets
    constexpr int ES = 272;                                    // staged row stride (bytes)
    w4_lds_c* stg_w = sb + (uint32_t)((w < 2 ? WSLOT : WB_OFF + WSLOT) + (w & 1) * 16384);
    w4_lds_c* wr = stg_w + (uint32_t)(l32 * ES + 8 * hi);      // + (32 jn + 8 q) * 2
    const int rl = lane >> 4, rc = (lane & 15) * 16;            // read-back: row rl + 4 i, byte rc
    const w4_lds_c* rd = stg_w + (uint32_t)(rl * ES + rc);
    w4_sfor<4>([&](auto IM) __attribute__((always_inline)) {
      constexpr int im = decltype(IM)::value;
      const int64_t row = row0 + 32 * im;
      const bool live = row < M_live;
      const int64_t rr = live ? row : M_live - 1;
      uint32_t mw[4] = {0u, 0u, 0u, 0u};
      if (BWD) {   // the 128 columns' bits of this row: 16 B
        const w4_u32x4 m4 = *reinterpret_cast<const w4_u32x4*>(p.mask_in + rr * p.ld_mask + (n0 + 128 * wn) / 8);
        mw[0] = m4[0]; mw[1] = m4[1]; mw[2] = m4[2]; mw[3] = m4[3];
      }
      uint32_t mbits[4] = {0u, 0u, 0u, 0u};
      w4_sfor<4>([&](auto JN) __attribute__((always_inline)) {
        constexpr int jn = decltype(JN)::value;
        const w4_f32x16 a = acc[im][jn];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = a[4 * q + r];
          if (BWD) {
            const uint32_t bits = mw[jn] >> (8 * q + 4 * hi);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = ((bits >> r) & 1u) ? v[r] * p.alpha : 0.f;
          } else {
            const float4_t bv = *reinterpret_cast<const w4_lds_f4*>(bl + 4 * (32 * jn + 8 * q));
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += bv[r];
          }
          uint32_t lo = w4_pk_bf16(v[0], v[1]), h2 = w4_pk_bf16(v[2], v[3]);
          if (RELU) {
            lo = w4_relu_pk(lo);
            h2 = w4_relu_pk(h2);
            // nonzero flags of the 4 (non-negative) bf16 as bits 0-3: v_pk_min_u16(x, 1) per pair puts
            // them at bits 0 / 16 and 2 / 18, one fold brings 16 / 18 down to 1 / 3 (pp8p's trick)
            const uint32_t u = w4_nz_pk(lo) | (w4_nz_pk(h2) << 2);
            mbits[jn] |= ((u | (u >> 15)) & 0xFu) << (8 * q + 4 * hi);
          }
          if constexpr ((DIAG & 128) != 0) asm volatile("" ::"v"(lo), "v"(h2));   // diagnostic: no staging
          else
            *reinterpret_cast<__attribute__((address_space(3))) w4_u32x2*>(wr + 2 * (32 * jn + 8 * q)) =
                (w4_u32x2){lo, h2};
        }
      });
      if (RELU && p.mask_out) {   // the row's 16 mask bytes from lanes l32 and l32 + 32
#pragma unroll
        for (int jn = 0; jn < 4; ++jn) mbits[jn] |= (uint32_t)__shfl_xor((int)mbits[jn], 32, 64);
        if (hi == 0 && live)
          *reinterpret_cast<w4_u32x4*>(p.mask_out + row * p.ld_mask + (n0 + 128 * wn) / 8) =
              (w4_u32x4){mbits[0], mbits[1], mbits[2], mbits[3]};
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      const int64_t srow0 = m0 + 128 * wm + 32 * im + rl;
      bf16_t* cst = p.C + srow0 * p.ldc + n0 + 128 * wn + rc / 2;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const w4_u32x4 v = *reinterpret_cast<const __attribute__((address_space(3))) w4_u32x4*>(rd + i * 4 * ES);
        if constexpr ((DIAG & 64) != 0) asm volatile("" ::"v"(v));   // diagnostic: staged, not stored
        else if (srow0 + 4 * i < M_live) __builtin_nontemporal_store(v, reinterpret_cast<w4_u32x4*>(cst + 4 * i * p.ldc));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the next block's writes
      __builtin_amdgcn_wave_barrier();
    });
    // every wave's staging reads of slot 1 are done before the next tile's first writes into it
    __builtin_amdgcn_s_barrier();
    }
    int64_t t_next = t_cur + gridDim.x;
    if (!next_tile(t_next, m0, n0)) return;
    t_cur = t_next;
  }
}

}  // namespace

// Host launcher (the caller checked the shapes: plain 16-B aligned bf16 operands, N % 256 == 0,
// K % 128 == 0, N <= 4096, C 16-B aligned with ldc % 8 == 0, the mask 4-B aligned with
// ld_mask % 4 == 0).  act: LLP_ACT_RELU (optional mask out), LLP_ACT_NONE, LLP_ACT_RELU_BWD (mask in).
int llp_gemm_nt_bf16_w4(const llp_operand* A, const llp_operand* B, int64_t M, int64_t N, int64_t K, void* C,
                        int64_t ldc, const float* bias, int act, float alpha, uint8_t* mask_out,
                        const uint8_t* mask_in, int64_t ld_mask, hipStream_t s, int diag = 0) {
  PW4 p;
  p.A = (const bf16_t*)A->ptr; p.lda = A->ld;
  p.B = (const bf16_t*)B->ptr; p.ldb = B->ld;
  p.M = M; p.N = N; p.K = K;
  p.C = (bf16_t*)C; p.ldc = ldc;
  p.bias = bias; p.alpha = alpha;
  p.mask_out = mask_out; p.mask_in = mask_in; p.ld_mask = ld_mask;
  p.m_dev = A->rows_dev;
  const int64_t tiles = ((M + WT - 1) / WT + 7) / 8 * 8 * (N / WT);
  const int cus = llp_cu_count();
  const dim3 grid((unsigned)(tiles < cus ? tiles : cus)), block(WTHR);
  if (diag) {   // diagnostic builds of the plain mode (llp_gemm_nt_w4_probe)
    switch (diag) {
      case 1: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 1>), grid, block, 0, s, p); break;
      case 2: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 2>), grid, block, 0, s, p); break;
      case 3: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 3>), grid, block, 0, s, p); break;
      case 4: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 4>), grid, block, 0, s, p); break;
      case 8: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 8>), grid, block, 0, s, p); break;
      case 15: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 15>), grid, block, 0, s, p); break;
      case 16: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 16>), grid, block, 0, s, p); break;
      case 17: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 17>), grid, block, 0, s, p); break;
      case 18: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 18>), grid, block, 0, s, p); break;
      case 19: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 19>), grid, block, 0, s, p); break;
      case 20: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 20>), grid, block, 0, s, p); break;
      case 23: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 23>), grid, block, 0, s, p); break;
      case 24: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 24>), grid, block, 0, s, p); break;
      case 48: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 48>), grid, block, 0, s, p); break;
      case 64: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 64>), grid, block, 0, s, p); break;
      case 192: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 192>), grid, block, 0, s, p); break;
      case 55: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 55>), grid, block, 0, s, p); break;
      case 32: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 32>), grid, block, 0, s, p); break;
      default: hipLaunchKernelGGL((gemm_nt_bf16_w4<W_NONE, 31>), grid, block, 0, s, p); break;
    }
    return (int)hipGetLastError();
  }
  if (act == LLP_ACT_RELU) hipLaunchKernelGGL(gemm_nt_bf16_w4<W_RELU>, grid, block, 0, s, p);
  else if (act == LLP_ACT_RELU_BWD) hipLaunchKernelGGL(gemm_nt_bf16_w4<W_BWD>, grid, block, 0, s, p);
  else hipLaunchKernelGGL(gemm_nt_bf16_w4<W_NONE>, grid, block, 0, s, p);
  return (int)hipGetLastError();
}

// Diagnostic entry for A/B runs (tools/w4_bench.py): the kernel above on plain device pointers.
extern "C" int llp_gemm_nt_w4_probe(const void* A, int64_t lda, const void* B, int64_t ldb, int64_t M, int64_t N,
                                    int64_t K, void* C, int64_t ldc, const float* bias, int act, float alpha,
                                    void* mask_out, const void* mask_in, int64_t ld_mask, int diag, void* stream) {
  LLP_CHECK_ARG(A && B && C && N % 256 == 0 && N <= 4096 && K % 128 == 0 && K > 0 && M > 0 && lda % 8 == 0 &&
                    ldb % 8 == 0 && ldc % 8 == 0 && (!mask_out || ld_mask % 16 == 0) &&
                    (act != LLP_ACT_RELU_BWD || (mask_in && ld_mask % 16 == 0)),
                "llp_gemm_nt_w4_probe: shapes");
  llp_operand a = {}, b = {};
  a.ptr = A; a.ld = lda;
  b.ptr = B; b.ld = ldb;
  const int rc = llp_gemm_nt_bf16_w4(&a, &b, M, N, K, C, ldc, bias, act, alpha, (uint8_t*)mask_out,
                                     (const uint8_t*)mask_in, ld_mask, (hipStream_t)stream, diag);
  if (rc != 0) return llp::set_error(rc, "llp_gemm_nt_w4_probe: %s", hipGetErrorString((hipError_t)rc));
  return LLP_OK;
}
