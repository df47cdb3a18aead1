// Persistent 256 x 256 f32 MFMA GEMM (NT form) for the fp32 path -- the reference's own
// arithmetic (src/models.py:48,143 in fp32; main.py's default dtype):
//
//   C[m, n] = act(alpha * sum_k A[m, k] * B[n, k] + bias[n])     f32 in, f32 accumulate, f32 out
//
// The bf16 persistent kernel's pipeline (gemm256.hip gemm_nt_bf16_pp8p) with f32 operands:
// a K-tile is 32 floats, the same 128-byte row segments as the bf16 K-tile of 64, so the
// LDS-DMA images, their 16-B chunk swizzle, the four quadrant phases, the chunk-per-phase
// issue order and every counted wait are the bf16 kernel's.  Each 16-B fragment read holds
// four consecutive k; one v_mfma_f32_16x16x4_f32 per float of it (k-slot g of lane (li, g)
// takes element 16 kh + 4 g + j), in the order of gemm.hip's register-staged f32 kernel
// (kh, then j), so per accumulator the sum runs over k in the same order.
// Round 5: that kernel (128 x 128, register-staged, two workgroups per CU) reached 0.77-0.78
// of the f32 peak with its MFMA pipes 78 % busy; the stretch without MFMAs was its K-tile
// boundary (global-load wait, LDS stores, barrier), which LDS-DMA staging one K-tile ahead
// removes.  Epilogue: straight from the accumulators (each lane holds 4 consecutive columns of
// one row: one 16-B store), alpha, bias, ReLU (torch.relu's NaN rule) or the ReLU backward
// through the stored f32 activations; f32 tiles are 8x longer than bf16 ones per byte of
// output, so the epilogue is a small share.
#include "llp_common.h"

namespace {

constexpr int FT = 256;          // tile rows / columns
constexpr int FTK = 32;          // K-tile (floats): 128-byte row segments
constexpr int FNT = 512;         // 8 waves: 2 (m) x 4 (n), 128 x 64 per wave
constexpr int IMG_U4 = 256 * 8;  // one operand image of a K-tile: 256 rows x 128 B
constexpr int TILE_U4 = 2 * IMG_U4;

constexpr int F32_RELU = 1, F32_NONE = 2, F32_BWD = 3;
// F32_HEAD (round 6): F32_RELU plus LinkPredictor's Linear(N, 1) head (src/models.py:146) in the
// epilogue: head_part[n0 / 256][m] = sum over the tile's 256 columns of relu(y[m, n]) * head_w[n],
// in a fixed order (per lane its 4 column blocks x 4 columns, then the 4 lanes of a row by
// xor-shuffles, then the 4 waves of the row's 64-column quarters through LDS), so deterministic;
// the logit is bias + the partials in column-tile order (llp_head_finish / the loss launch).
// Replaces the fp32 step's separate llp_head_fwd pass over the [R2, H] activations.
constexpr int F32_HEAD = 4;

struct PF32 {
  const float* A; int64_t lda;
  const float* B; int64_t ldb;
  int64_t M, N, K;
  float* C; int64_t ldc;
  const float* bias;
  const float* aux; int64_t ld_aux;   // F32_BWD: the layer's stored f32 activations
  float alpha;
  const int32_t* m_dev;               // device row count or NULL
  const float* head_w; float* head_part; int64_t head_ld;   // F32_HEAD
};

__device__ __forceinline__ void glds16_s(uint32_t voff, const void* sbase, uint32_t lds_addr_uniform) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase),
               "s"(lds_addr_uniform)
               : "memory", "m0");
}
__device__ __forceinline__ void glds16(const void* gptr, uint32_t lds_addr_uniform) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gptr),
               "s"(lds_addr_uniform)
               : "memory", "m0");
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) void*)p);
}
// chunk-row cr in [0,128) -> tile row (gemm256.hip q64_row): chunk 0 / 3 = A rows with
// row % 128 < 64 / >= 64, chunk 1 / 2 = B rows with row % 64 < 32 / >= 32
__device__ __forceinline__ int q64_row(int chunk, int cr) {
  switch (chunk) {
    case 0: return (cr & 63) + 128 * (cr >> 6);
    case 3: return (cr & 63) + 128 * (cr >> 6) + 64;
    case 1: return (cr & 31) + 64 * (cr >> 5);
    default: return (cr & 31) + 64 * (cr >> 5) + 32;
  }
}

template <int MODE>
__global__ __launch_bounds__(FNT) void gemm_nt_f32_pp8p(PF32 p) {
  constexpr bool BWD = MODE == F32_BWD;
  constexpr bool HEAD = MODE == F32_HEAD;
  constexpr bool RELU = MODE == F32_RELU || HEAD;
  constexpr int BLDS = 2 * TILE_U4;          // the tile's 256 bias floats (1 KB)
  constexpr int HWLDS = BLDS + 64;           // the tile's 256 head weights (1 KB, F32_HEAD)
  __shared__ __attribute__((aligned(16))) uint4 smem[2 * TILE_U4 + 128];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int wm = w >> 2, wn = w & 3;
  const bool grp1 = wu >= 4;
  const int64_t tilesN = (p.N + FT - 1) / FT;
  const int64_t tilesM_host = (p.M + FT - 1) / FT;
  const int64_t n_tiles = (tilesM_host + 7) / 8 * 8 * tilesN;
  int64_t M_live = p.M;
  if (p.m_dev) {
    const int64_t c = *p.m_dev;
    M_live = c < p.M ? (c > 0 ? c : 0) : p.M;
  }
  p.M = M_live;
  const int64_t tilesM = (M_live + FT - 1) / FT;
  // tile t -> (m0, n0): XCD t % 8 takes m-tiles t % 8, + 8, ..., each with its n-tiles
  auto tile_of = [&](int64_t t, int64_t& m0, int64_t& n0) -> bool {
    const int64_t xcd = t % 8, loc = t / 8;
    const int64_t mt = (loc / tilesN) * 8 + xcd;
    m0 = mt * FT;
    n0 = (loc % tilesN) * FT;
    return t < n_tiles && mt < tilesM;
  };
  auto next_tile = [&](int64_t& t, int64_t& m0, int64_t& n0) -> bool {
    while (t < n_tiles && !tile_of(t, m0, n0)) t += gridDim.x;
    return t < n_tiles;
  };
  int64_t t = blockIdx.x, m0 = 0, n0 = 0;
  if (!next_tile(t, m0, n0)) return;

  // DMA piece: rows q64_row(..) + lane / 8 of the tile (clamped to the last live row), logical
  // 16-B chunk (lane % 8) ^ (lane / 8) of the row's 128-byte K-tile segment
  const int lr = lane >> 3;
  const uint32_t lc16 = (uint32_t)(((lane & 7) ^ (lane >> 3)) * 16);
  const uint32_t lds0 = lds_u32(smem);
  auto issue_chunk = [&](int j, int buf, int64_t tm0, int64_t tn0, int64_t koff) {
    const bool isA = j == 0 || j == 3;
    const uint32_t base = lds0 + (uint32_t)(buf * TILE_U4 * 16) + (isA ? 0u : IMG_U4 * 16u);
    const float* sb = isA ? p.A + tm0 * p.lda + koff : p.B + tn0 * p.ldb + koff;
    const int lim = (int)(isA ? min((int64_t)255, p.M - 1 - tm0) : min((int64_t)255, p.N - 1 - tn0));
    const int64_t ld = isA ? p.lda : p.ldb;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row0 = q64_row(j, 16 * wu + 8 * i);
      const uint32_t voff = (uint32_t)(min(row0 + lr, lim) * (int)ld * 4) + lc16;
      glds16_s(voff, sb, __builtin_amdgcn_readfirstlane(base + (uint32_t)(row0 * 128)));
    }
  };
  float4_t fa[2][4];
  float4_t fb[2][2][2];
  float4_t acc[4][8];
  auto read_a = [&](const uint4* sA, int mh) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int im = 0; im < 4; ++im) {
        const int r = wm * 128 + mh * 64 + im * 16 + li;
        uint4 v = sA[r * 8 + ((kh * 4 + g) ^ (r & 7))];
        fa[kh][im] = *reinterpret_cast<float4_t*>(&v);
      }
  };
  auto read_b = [&](const uint4* sB, int nh) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int jn = 0; jn < 2; ++jn) {
        const int r = wn * 64 + nh * 32 + jn * 16 + li;
        uint4 v = sB[r * 8 + ((kh * 4 + g) ^ (r & 7))];
        fb[nh][kh][jn] = *reinterpret_cast<float4_t*>(&v);
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
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[nh * 2 + jn][mh * 4 + im] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                fb[nh][kh][jn][j], fa[kh][im][j], acc[nh * 2 + jn][mh * 4 + im], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  const int64_t nk = p.K / FTK;
  const float* blds = reinterpret_cast<const float*>(smem + BLDS);

  // first tile: its K-tile 0 (all four chunks) into buffer 0
#pragma unroll
  for (int j = 0; j < 4; ++j) issue_chunk(j, 0, m0, n0, 0);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // chunks 0, 1 landed
  for (;;) {
    int64_t t_next = t + gridDim.x, m1 = 0, n1 = 0;
    const bool pf = next_tile(t_next, m1, n1);
    // this tile's bias into LDS by DMA (an ordinary load would drain the DMA ring at its use)
    if (p.bias && wu == 0) glds16(p.bias + n0 + 4 * lane, __builtin_amdgcn_readfirstlane(lds_u32(smem + BLDS)));
    if (HEAD && wu == 1) glds16(p.head_w + n0 + 4 * lane, __builtin_amdgcn_readfirstlane(lds_u32(smem + HWLDS)));
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
    for (int64_t kt = 0; kt + 1 < nk; ++kt) ktile(kt, true, (int)((kt + 1) & 1), m0, n0, (kt + 1) * FTK);
    // the last K-tile: the next tile's K-tile 0 into buffer 0 (nk is even) when prefetching
    ktile(nk - 1, pf, 0, m1, n1, 0);
    if (!grp1) barrier();         // waves 0-3 match the other half's barrier count
    // ---- epilogue from the accumulators: lane (li, g) holds columns 4 g .. 4 g + 3 of row li of
    // each 16 x 16 block; buffer 0 receives the next tile's K-tile 0 meanwhile, so no LDS is touched
    // but the bias image (read before this tile's next barrier overwrites it: see below)
    int etid = tid;
    asm volatile("" : "+v"(etid));   // keeps the epilogue's addresses out of the main loop's registers
    const int elane = etid & 63, ew = etid >> 6;
    const int eg = elane >> 4, eli = elane & 15, ewm = ew >> 2, ewn = ew & 3;
    const float* __restrict__ aux = p.aux;
    float* __restrict__ C = p.C;
    const float alpha = p.alpha;
    const float* hwl = reinterpret_cast<const float*>(smem + HWLDS);
    float hd[8];   // F32_HEAD: this lane's head dot of row block im over its 4 x 4 columns
#pragma unroll
    for (int im = 0; im < 8; ++im) hd[im] = 0.f;
    // column blocks jn = 2 jp, 2 jp + 1 are the two 64-B halves of one 128-B line of each row: the
    // two stores of a line go out back to back, so L2 merges them into one full-line write
    // (jn-outer order left them 8 stores apart and counted 1.55x the C bytes in WRITE_SIZE)
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      float4_t bv[2];
#pragma unroll
      for (int q = 0; q < 2; ++q)
        bv[q] = (!BWD && p.bias) ? *reinterpret_cast<const float4_t*>(blds + ewn * 64 + (2 * jp + q) * 16 + eg * 4)
                                 : float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ih = 0; ih < 2; ++ih) {
        // the ReLU-backward activations of these 4 rows x 2 column quads, loaded together (one
        // wait, not one round trip per row); rows past M read the last live row and are not stored
        float4_t av[4][2];
        float4_t hw[2];
        if (HEAD) {
#pragma unroll
          for (int q = 0; q < 2; ++q) hw[q] = *reinterpret_cast<const float4_t*>(hwl + ewn * 64 + (2 * jp + q) * 16 + eg * 4);
        }
        if (BWD) {
#pragma unroll
          for (int iq = 0; iq < 4; ++iq)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const int64_t row = min(m0 + ewm * 128 + (4 * ih + iq) * 16 + eli, p.M - 1);
              const int64_t col = n0 + ewn * 64 + (2 * jp + q) * 16 + eg * 4;
              av[iq][q] = *reinterpret_cast<const float4_t*>(aux + row * p.ld_aux + col);
            }
        }
#pragma unroll
        for (int iq = 0; iq < 4; ++iq) {
          const int im = 4 * ih + iq;
          const int64_t row = m0 + ewm * 128 + im * 16 + eli;
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int jn = 2 * jp + q;
            const int64_t col = n0 + ewn * 64 + jn * 16 + eg * 4;
            float4_t v;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float x = alpha * acc[jn][im][r] + bv[q][r];
              if (RELU) x = x < 0.f ? 0.f : x;   // torch.relu: a NaN stays NaN
              if (BWD) x = av[iq][q][r] > 0.f ? x : 0.f;
              v[r] = x;
              if (HEAD) hd[im] = fmaf(x, hw[q][r], hd[im]);
            }
            if (row < p.M) *reinterpret_cast<float4_t*>(C + row * p.ldc + col) = v;
          }
        }
      }
    }
    if (HEAD) {
      // the 4 lanes of a row (g = 0..3) by xor-shuffles, then the row's 4 wave quarters (ewn) through
      // LDS in buffer 1 (free: the last K-tile's reads are done, the next tile's K-tile 0 goes to buffer
      // 0); one thread per row sums them in quarter order
      float* part = reinterpret_cast<float*>(smem + TILE_U4);
#pragma unroll
      for (int im = 0; im < 8; ++im) {
        float d = hd[im];
        d += __shfl_xor(d, 16, 64);
        d += __shfl_xor(d, 32, 64);
        if (eg == 0) part[(ewm * 128 + im * 16 + eli) * 4 + ewn] = d;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      barrier();
      if (etid < 256 && m0 + etid < p.M) {
        const float4_t q4 = *reinterpret_cast<const float4_t*>(part + etid * 4);
        p.head_part[(n0 / FT) * p.head_ld + m0 + etid] = (q4[0] + q4[1]) + (q4[2] + q4[3]);
      }
    }
    if (!pf) return;
    t = t_next; m0 = m1; n0 = n1;
    // the bias / head-weight images (and the head partials in buffer 1) are rewritten by the next
    // tile's DMA: every wave has read them above
    barrier();
  }
}

}  // namespace

int llp_cu_count();

// Called from llp_gemm_nt for f32 operands when the shapes allow it (gemm.hip): plain 16-B
// aligned operands, N % 256 == 0, K % 64 == 0 (an even number of K-tiles), more than one
// wave of tiles.  mode: LLP_ACT_RELU / LLP_ACT_NONE / LLP_ACT_RELU_BWD (f32 aux activations).
int llp_gemm_nt_f32_256(const llp_operand* A, const llp_operand* B, int64_t M, int64_t N, int64_t K, float* C,
                        int64_t ldc, const float* bias, int act, const float* aux, int64_t ld_aux, float alpha,
                        hipStream_t s, const float* head_w, float* head_part) {
  PF32 p;
  p.head_w = head_w; p.head_part = head_part; p.head_ld = M;
  p.A = (const float*)A->ptr; p.lda = A->ld;
  p.B = (const float*)B->ptr; p.ldb = B->ld;
  p.M = M; p.N = N; p.K = K;
  p.C = C; p.ldc = ldc;
  p.bias = bias; p.aux = aux; p.ld_aux = ld_aux; p.alpha = alpha;
  p.m_dev = A->rows_dev;
  const int64_t tiles = ((M + FT - 1) / FT + 7) / 8 * 8 * (N / FT);
  const int cus = llp_cu_count();
  const dim3 grid((unsigned)(tiles < cus ? tiles : cus)), block(FNT);
  if (head_w) hipLaunchKernelGGL(gemm_nt_f32_pp8p<F32_HEAD>, grid, block, 0, s, p);   // (ReLU + head)
  else if (act == LLP_ACT_RELU) hipLaunchKernelGGL(gemm_nt_f32_pp8p<F32_RELU>, grid, block, 0, s, p);
  else if (act == LLP_ACT_RELU_BWD) hipLaunchKernelGGL(gemm_nt_f32_pp8p<F32_BWD>, grid, block, 0, s, p);
  else hipLaunchKernelGGL(gemm_nt_f32_pp8p<F32_NONE>, grid, block, 0, s, p);
  return (int)hipGetLastError();
}
