// Large-tile bf16 MFMA weight-gradient GEMM (TN form):
//
//   ws[z][p][q] = sum_{m in split z} A[m, p] * B[m, q]      (A = dY, B = X; f32 slabs)
//   ws_colsum[z][p] = sum_{m in split z} A[m, p]            (bias gradient, optional)
//
// Replaces autograd's weight/bias-gradient of every nn.Linear on the
// distillation path (src/main.py:132).  256 (p) x 256 (q) tile per 512-thread
// workgroup.  The contraction index m is the ROW of both operands, so a stage
// of 32 rows keeps full 512-B row segments: both operands are staged by
// global_load_lds_dwordx4 (issued from inline asm, see gemm256.hip glds16) into
// [32][256] images (16-B chunks XOR-swizzled by row) held in a 4-stage LDS
// ring with 3 stages in flight (counted vmcnt + raw barriers), and read as
// MFMA fragments with ds_read_b64_tr_b16.  Rows past the split's end read a
// zero row.  B rows may be gathered (x[this_target], the first student layer).
// MFMA roles put 4 consecutive q of one p in a lane (16-byte slab stores).
// The bias gradient rides along: waves of the q0 == 0 tiles multiply their A
// fragments by a ones fragment (4 extra MFMAs per 32 on those waves).
#include "llp_common.h"

namespace {

constexpr int TP = 256, TQ = 256, TKM = 32;
constexpr int NTT = 512;
constexpr int NS = 4;                          // LDS ring depth (stages of TKM rows)
constexpr int IMG_U4 = TKM * 32;               // one [32][256] bf16 image = 1024 uint4 = 16 KiB
constexpr int STAGE_T = 2 * IMG_U4;            // A image + B image = 32 KiB
constexpr int IDX_LDS = 8192;                  // gather indices staged in LDS (int32 slots)

__device__ __attribute__((aligned(16))) uint4 g_zero_row[64];   // 1 KiB of zeros (static init)

struct PTN {
  const bf16_t* A; const int32_t* ia; int64_t lda;
  const bf16_t* B; const int32_t* ib; int64_t ldb;
  int64_t M, P, Q, mchunk, splits;
  float* ws;
  float* ws_colsum;   // [splits][P] column sums of A (bias gradient), or NULL
  const int32_t* m_dev;   // device row count (llp_operand.rows_dev) or NULL
  int zmajor;             // block -> (split, tile) order: split-major (default) or tile-major
};

__device__ __forceinline__ int64_t xcd_remap3(int64_t bid, int64_t nwg) {
  if (nwg < 8) return bid;
  const int64_t q = nwg / 8, r = nwg % 8;
  const int64_t xcd = bid % 8, loc = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// Block -> (tile, split).  Split-major: the blocks of one split -- every tile of the same
// rows of A and B -- are consecutive, so xcd_remap3 places them on one XCD, whose L2 then
// serves each staged row to all tiles (A rows to the Q/256 column tiles, B rows to the P/256
// row tiles).  Tile-major (the old order) put the splits of one tile together: each row
// came from beyond L2 once per tile.
__device__ __forceinline__ void tn_block(int zmajor, int tiles, int splits, int64_t& tile, int64_t& z) {
  const int lt = (int)xcd_remap3(blockIdx.x, (int64_t)tiles * splits);
  const int d = zmajor ? tiles : splits;
  const int hi = lt / d, lo = lt - hi * d;
  tile = zmajor ? lo : hi;
  z = zmajor ? hi : lo;
}

typedef __attribute__((address_space(3))) short4_t lds_s4;
typedef __attribute__((address_space(3))) char lds_char;


// swizzle of the 16-B chunk index within a 512-B image row (low 4 bits only):
// T10 image (b); conflict-free for the transposed reads below.
__device__ __forceinline__ int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

__device__ __forceinline__ void glds16(const void* gptr, uint32_t lds_addr_uniform) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gptr),
               "s"(lds_addr_uniform)
               : "memory", "m0");
}

__device__ __forceinline__ void vm_wait(int64_t ahead) {   // 4 glds per wave per stage
  if (ahead <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (ahead == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
}

// STAG (2 for gathered operands; plain ones take its lean form, gemm_tn_bf16_256c): 1 = waves 4-7 run each stage's MFMAs one stage
// late (after the next barrier, before that stage's reads); 2 = as 1 with their
// DMA issued after those MFMAs.  Bit-identical (same per-accumulator order).
template <int STAG>
__global__ __launch_bounds__(NTT) void gemm_tn_bf16_256(PTN p) {
  // the ring (128 KiB), then the split's gather indices (32 KiB; one __shared__ array, so
  // hipcc's waitcnt pass sees no second object beside the LDS-DMA ring)
  __shared__ __attribute__((aligned(16))) uint4 smem[NS * STAGE_T + IDX_LDS / 4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int64_t tilesQ = (p.Q + TQ - 1) / TQ;
  const int64_t tilesP = (p.P + TP - 1) / TP;
  int64_t tile, z;
  tn_block(p.zmajor, (int)(tilesP * tilesQ), (int)p.splits, tile, z);
  const int64_t p0 = (tile / tilesQ) * TP, q0 = (tile % tilesQ) * TQ;
  if (p.m_dev) {   // live rows from the device count; the grid (splits) is the host M's
    const int64_t c = *p.m_dev;
    p.M = c < p.M ? (c > 0 ? c : 0) : p.M;
    const int64_t mc = (p.M + p.splits - 1) / p.splits;
    p.mchunk = mc > 0 ? (mc + TKM - 1) / TKM * TKM : TKM;
  }
  const int64_t mbeg = z * p.mchunk;
  const int64_t mend = min(p.M, mbeg + p.mchunk);

  // glds: wave w stages image rows [4w, 4w+4) of each operand: instruction i
  // covers rows 4w + 2i + (lane >> 5), physical chunk lane & 31.
  const int pc = lane & 31;
  const int rbase = 4 * w + (lane >> 5);
  const int wu = __builtin_amdgcn_readfirstlane(w);
  // columns past P / Q are clamped to a valid address (their products are never stored)
  const int capA = (int)max((int64_t)0, (p.P - p0) - 8), capB = (int)max((int64_t)0, (p.Q - q0) - 8);
  const bf16_t* zrow = reinterpret_cast<const bf16_t*>(g_zero_row);
  const uint32_t lds0 = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) void*)smem);

  // full stages (every row < mend, plain operands): per-lane pointers advanced
  // by a uniform stride, no per-stage address arithmetic beside the MFMAs
  const int64_t nfull = (p.ia || p.ib) ? 0 : (mend - mbeg) / TKM;
  const bf16_t* pa[2];
  const bf16_t* pb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = rbase + 2 * i;
    const int lc8 = (pc ^ swz(r)) * 8;
    pa[i] = p.A + (mbeg + r) * p.lda + p0 + min(lc8, capA);
    pb[i] = p.B + (mbeg + r) * p.ldb + q0 + min(lc8, capB);
  }
  const int64_t strideA = (int64_t)TKM * p.lda, strideB = (int64_t)TKM * p.ldb;
  // gathered rows (x[this_target], the first student layer): the split's indices are
  // staged in LDS before any DMA, so reading them never waits on the vector-memory
  // counter (a global index load would drain the in-flight DMA ring every stage)
  const int n_idx = (p.ia ? 1 : 0) + (p.ib ? 1 : 0);
  const int64_t nrows = mend > mbeg ? mend - mbeg : 0;
  const int64_t idx_cap = n_idx ? IDX_LDS / n_idx : 0;
  const bool idx_lds = n_idx > 0 && nrows <= idx_cap;
  int32_t* sidx = reinterpret_cast<int32_t*>(smem + NS * STAGE_T);
  const int32_t* sia = sidx;
  const int32_t* sib = sidx + (p.ia ? idx_cap : 0);
  if (idx_lds) {
    for (int64_t t = tid; t < nrows; t += NTT) {
      if (p.ia) sidx[t] = p.ia[mbeg + t];
      if (p.ib) sidx[(p.ia ? idx_cap : 0) + t] = p.ib[mbeg + t];
    }
    __syncthreads();   // no DMA in flight yet: this barrier's vmcnt(0) waits for the index loads only
  }
  auto issue = [&](int64_t st) {
    const int64_t mt = mbeg + st * TKM;
    const uint32_t sA = lds0 + (uint32_t)((st % NS) * STAGE_T * 16);
    const uint32_t sB = sA + IMG_U4 * 16;
    if (st < nfull) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint32_t off = (uint32_t)((4 * wu + 2 * i) * 32 * 16);
        glds16(pa[i] + st * strideA, __builtin_amdgcn_readfirstlane(sA + off));
        glds16(pb[i] + st * strideB, __builtin_amdgcn_readfirstlane(sB + off));
      }
      return;
    }
    // ragged last stage or gathered rows: rows past the split's end read zeros
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = rbase + 2 * i;
      const int lc8 = (pc ^ swz(r)) * 8;
      const int ca = min(lc8, capA), cb = min(lc8, capB);
      const int64_t m = mt + r;
      const bool v = m < mend;
      const int64_t mm = v ? m : mbeg;
      int64_t ra, rb;
      if (idx_lds) {
        ra = p.ia ? (int64_t)sia[mm - mbeg] : mm;
        rb = p.ib ? (int64_t)sib[mm - mbeg] : mm;
      } else {
        ra = p.ia ? (int64_t)p.ia[mm] : mm;
        rb = p.ib ? (int64_t)p.ib[mm] : mm;
      }
      const bf16_t* srcA = v ? p.A + ra * p.lda + p0 + ca : zrow + ca;
      const bf16_t* srcB = v ? p.B + rb * p.ldb + q0 + cb : zrow + cb;
      const uint32_t off = (uint32_t)((4 * wu + 2 * i) * 32 * 16);
      glds16(srcA, __builtin_amdgcn_readfirstlane(sA + off));
      glds16(srcB, __builtin_amdgcn_readfirstlane(sB + off));
    }
  };

  const int wq = w >> 2, wp = w & 3;
  float4_t acc[8][4];   // [q-tile jq][p-tile ip]: rows q = 16 jq + 4 g + r, col p = 16 ip + li
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = float4_t{0.f, 0.f, 0.f, 0.f};

  const int q4 = li >> 2, pp = li & 3;
  const bool do_cs = p.ws_colsum != nullptr && q0 == 0 && wq == 0;
  float4_t accb[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) accb[b] = float4_t{0.f, 0.f, 0.f, 0.f};
  short8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (short)0x3F80;   // bf16 1.0

  auto tr_read = [&](const char* img, int row, int col) -> short4_t {
    const int off = row * 512 + 16 * ((col >> 3) ^ swz(row)) + 8 * ((col >> 2) & 1);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s4*)((lds_char*)((__attribute__((address_space(3))) uint4*)img) + off));
  };

  const bool stag = STAG > 0 && wu >= 4;
  short8 fp[4];
  short8 fq[2][4];
  auto mfma_cs = [&]() {
#pragma unroll
    for (int ip = 0; ip < 4; ++ip)
      accb[ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, fp[ip], accb[ip], 0, 0, 0);
  };
  auto mfma_half = [&](int jh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int ip = 0; ip < 4; ++ip)
        acc[4 * jh + jj][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fq[jh][jj], fp[ip], acc[4 * jh + jj][ip], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto mfma_stage = [&]() {
    if (do_cs) mfma_cs();
    mfma_half(0);
    mfma_half(1);
  };

  if (mbeg < mend) {
    const int64_t nsteps = (mend - mbeg + TKM - 1) / TKM;
    for (int64_t s = 0; s < NS - 1 && s < nsteps; ++s) issue(s);
    for (int64_t st = 0; st < nsteps; ++st) {
      vm_wait(min(nsteps - 1, st + NS - 2) - st);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const bool late = STAG == 2 && wu >= 4;
      if (!late && st + NS - 1 < nsteps) issue(st + NS - 1);   // into the buffer of stage st-1
      const char* sA = reinterpret_cast<const char*>(smem + (int)(st % NS) * STAGE_T);
      const char* sB = sA + IMG_U4 * 16;
      const int row0 = 8 * g + q4;    // k rows 8g..8g+3 and 8g+4..8g+7
      if (stag && st > 0) mfma_stage();   // the previous stage's products
      if (late && st + NS - 1 < nsteps) issue(st + NS - 1);
#pragma unroll
      for (int ip = 0; ip < 4; ++ip) {
        const int col = wp * 64 + ip * 16 + 4 * pp;
        const short4_t t0 = tr_read(sA, row0, col), t1 = tr_read(sA, row0 + 4, col);
#pragma unroll
        for (int e = 0; e < 4; ++e) { fp[ip][e] = t0[e]; fp[ip][4 + e] = t1[e]; }
      }
      if (!stag && do_cs) mfma_cs();
#pragma unroll
      for (int jh = 0; jh < 2; ++jh) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int col = wq * 128 + (4 * jh + jj) * 16 + 4 * pp;
          const short4_t t0 = tr_read(sB, row0, col), t1 = tr_read(sB, row0 + 4, col);
#pragma unroll
          for (int e = 0; e < 4; ++e) { fq[jh][jj][e] = t0[e]; fq[jh][jj][4 + e] = t1[e]; }
        }
        if (!stag) mfma_half(jh);
      }
    }
    if (stag) mfma_stage();   // the last stage
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (do_cs && g == 0) {   // every row of the ones-product holds the column sums: take row 0
#pragma unroll
    for (int ip = 0; ip < 4; ++ip) {
      const int64_t pr = p0 + wp * 64 + ip * 16 + li;
      if (pr < p.P) p.ws_colsum[z * p.P + pr] = accb[ip][0];
    }
  }
  // slab store: C[p][q..q+3] as one float4
  float* out = p.ws + z * p.P * p.Q;
#pragma unroll
  for (int ip = 0; ip < 4; ++ip) {
    const int64_t pr = p0 + wp * 64 + ip * 16 + li;
    if (pr >= p.P) continue;
#pragma unroll
    for (int jq = 0; jq < 8; ++jq) {
      const int64_t qc = q0 + wq * 128 + jq * 16 + 4 * g;
      if (qc >= p.Q) continue;
      *reinterpret_cast<float4_t*>(out + pr * p.Q + qc) = acc[jq][ip];
    }
  }
}


// Lean form of the staggered loop (STAG 2; plain operands),
// plain (non-gathered) operands only.  Same stages, DMA pieces, fragments, MFMA
// operands and per-accumulator order as gemm_tn_bf16_256 (bit-identical slabs),
// without its per-stage VALU work, which at two waves per SIMD competed with the
// MFMAs for vector issue (about 2.3 VALU + 1.8 SALU per MFMA in the old loop):
//  * LDS: A images of the 4 stages in [0, 64 KiB), B images in [64, 128 KiB), so a
//    fragment read is (per-lane offset, computed once) + slot * 16 KiB, a constant
//    that folds into the ds_read offset field (the loop is unrolled by the 4 slots);
//  * DMA in SADDR form: per-lane 32-bit offsets fixed for the kernel, the stage's
//    row base in SGPRs advanced by a scalar add;
//  * per-wave roles hoisted out of the loop: waves 0-3 (the only ones that can
//    carry the ones-fragment bias MFMAs) run the plain body, waves 4-7 the
//    staggered one; the steady loop has no data-dependent branch and a constant
//    vmcnt; the last stages (and a ragged one) run the generic body.
constexpr int LIMG = 16384;                 // bytes of one [32][256] bf16 image
constexpr int LB0 = NS * LIMG;              // B images start here

__device__ __forceinline__ void glds16_s(uint32_t voff, const bf16_t* sbase, uint32_t lds_addr_uniform) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase),
               "s"(lds_addr_uniform)
               : "memory", "m0");
}

template <int STAG, bool QH = false>
__global__ __launch_bounds__(NTT) void gemm_tn_bf16_256c(PTN p) {
  __shared__ __attribute__((aligned(16))) uint4 smem[NS * STAGE_T];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int64_t tilesQ = (p.Q + TQ - 1) / TQ;
  const int64_t tilesP = (p.P + TP - 1) / TP;
  int64_t tile, z;
  tn_block(p.zmajor, (int)(tilesP * tilesQ), (int)p.splits, tile, z);
  const int64_t p0 = (tile / tilesQ) * TP, q0 = (tile % tilesQ) * TQ;
  if (p.m_dev) {
    const int64_t c = *p.m_dev;
    p.M = c < p.M ? (c > 0 ? c : 0) : p.M;
    const int64_t mc = (p.M + p.splits - 1) / p.splits;
    p.mchunk = mc > 0 ? (mc + TKM - 1) / TKM * TKM : TKM;
  }
  const int64_t mbeg = z * p.mchunk;
  const int64_t mend = min(p.M, mbeg + p.mchunk);

  const int pc = lane & 31;
  const int rbase = 4 * w + (lane >> 5);
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int capA = (int)max((int64_t)0, (p.P - p0) - 8), capB = (int)max((int64_t)0, (p.Q - q0) - 8);
  const bf16_t* zrow = reinterpret_cast<const bf16_t*>(g_zero_row);
  const uint32_t lds0 = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) void*)smem);
  const int64_t nfull = mend > mbeg ? (mend - mbeg) / TKM : 0;
  const int64_t nsteps = mend > mbeg ? (mend - mbeg + TKM - 1) / TKM : 0;

  // DMA: wave w's piece i covers image rows 4w + 2i, 4w + 2i + 1 (lane >> 5), physical chunk lane & 31
  uint32_t voA[2], voB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = rbase + 2 * i;
    const int lc8 = (pc ^ swz(r)) * 8;
    voA[i] = (uint32_t)((r * p.lda + min(lc8, capA)) * 2);
    voB[i] = (uint32_t)((r * p.ldb + min(lc8, capB)) * 2);
  }
  const bf16_t* gA = p.A + mbeg * p.lda + p0;
  const bf16_t* gB = p.B + mbeg * p.ldb + q0;
  const int64_t stepA = (int64_t)TKM * p.lda, stepB = (int64_t)TKM * p.ldb;
  const uint32_t ldw = lds0 + (uint32_t)(4 * wu * 512);
  auto issue_fast = [&](int64_t st, int slot) {
    const bf16_t* ba = gA + st * stepA;
    const bf16_t* bb = gB + st * stepB;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      glds16_s(voA[i], ba, __builtin_amdgcn_readfirstlane(ldw + (uint32_t)(slot * LIMG + i * 1024)));
      glds16_s(voB[i], bb, __builtin_amdgcn_readfirstlane(ldw + (uint32_t)(LB0 + slot * LIMG + i * 1024)));
    }
  };
  auto issue = [&](int64_t st) {   // any stage (rows past the split's end read zeros)
    const int slot = (int)(st % NS);
    if (st < nfull) { issue_fast(st, slot); return; }
    const int64_t mt = mbeg + st * TKM;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = rbase + 2 * i;
      const int lc8 = (pc ^ swz(r)) * 8;
      const int64_t m = mt + r;
      const bool v = m < mend;
      const bf16_t* srcA = v ? p.A + m * p.lda + p0 + min(lc8, capA) : zrow + min(lc8, capA);
      const bf16_t* srcB = v ? p.B + m * p.ldb + q0 + min(lc8, capB) : zrow + min(lc8, capB);
      glds16(srcA, __builtin_amdgcn_readfirstlane(ldw + (uint32_t)(slot * LIMG + i * 1024)));
      glds16(srcB, __builtin_amdgcn_readfirstlane(ldw + (uint32_t)(LB0 + slot * LIMG + i * 1024)));
    }
  };

  const int wq = w >> 2, wp = w & 3;
  float4_t acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = float4_t{0.f, 0.f, 0.f, 0.f};
  const int q4 = li >> 2, pp = li & 3;
  const bool do_cs = p.ws_colsum != nullptr && q0 == 0 && wq == 0;
  // QH (Q <= 128: the first student layer's weight gradient at F = 128, the teacher's first
  // layer): waves 4-7 own the tile's columns 128 .. 255, only padding, and skip their fragment
  // reads and MFMAs, so each SIMD runs one wave's MFMAs (they still stage their DMA pieces and
  // keep the barrier count).  A compile-time flag: a run-time test in the staggered body cost
  // every TN launch ~2 % (the lean loop's steady body has no data-dependent branch)
  constexpr bool q_live = !QH;
  float4_t accb[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) accb[b] = float4_t{0.f, 0.f, 0.f, 0.f};
  short8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (short)0x3F80;

  // per-lane fragment offsets (bytes from smem) of slot 0: rows row0 and row0 + 4
  const int row0 = 8 * g + q4;
  auto img_off = [&](int row, int col) {
    return row * 512 + 16 * ((col >> 3) ^ swz(row)) + 8 * ((col >> 2) & 1);
  };
  int oA[4][2], oB[8][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int ip = 0; ip < 4; ++ip) oA[ip][h] = img_off(row0 + 4 * h, wp * 64 + ip * 16 + 4 * pp);
#pragma unroll
    for (int jq = 0; jq < 8; ++jq) oB[jq][h] = LB0 + img_off(row0 + 4 * h, wq * 128 + jq * 16 + 4 * pp);
  }
  lds_char* sbase = (lds_char*)((__attribute__((address_space(3))) uint4*)smem);
  auto trd = [&](int off) -> short4_t { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(sbase + off)); };

  short8 fp[4];
  short8 fq[8];
  auto read_p = [&](int sl) {
#pragma unroll
    for (int ip = 0; ip < 4; ++ip)
      fp[ip] = __builtin_shufflevector(trd(oA[ip][0] + sl * LIMG), trd(oA[ip][1] + sl * LIMG), 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto read_q = [&](int sl, int j0) {
#pragma unroll
    for (int jq = j0; jq < j0 + 4; ++jq)
      fq[jq] = __builtin_shufflevector(trd(oB[jq][0] + sl * LIMG), trd(oB[jq][1] + sl * LIMG), 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto mfma_cs = [&]() {
#pragma unroll
    for (int ip = 0; ip < 4; ++ip)
      accb[ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, fp[ip], accb[ip], 0, 0, 0);
  };
  auto mfma_half = [&](int jh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int ip = 0; ip < 4; ++ip)
        acc[4 * jh + jj][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fq[4 * jh + jj], fp[ip], acc[4 * jh + jj][ip], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto head = [&](int64_t st, bool steady) {   // wait for stage st, barrier
    if (steady) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else vm_wait(min(nsteps - 1, st + NS - 2) - st);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  // plain body (waves 0-3; CS: this tile carries the bias-gradient MFMAs)
  auto body_plain = [&](auto CS, int sl, int64_t st, bool steady) {
    head(st, steady);
    if (steady) issue_fast(st + NS - 1, (sl + NS - 1) % NS);
    else if (st + NS - 1 < nsteps) issue(st + NS - 1);
    read_p(sl);
    read_q(sl, 0);
    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
    if constexpr (decltype(CS)::value) mfma_cs();
    mfma_half(0);
    read_q(sl, 4);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    mfma_half(1);
  };
  // staggered body (waves 4-7): the previous stage's MFMAs after the barrier, then (STAG 2)
  // the DMA, then this stage's fragments
  auto body_stag = [&](int sl, int64_t st, bool steady) {
    head(st, steady);
    if (STAG == 1) {
      if (steady) issue_fast(st + NS - 1, (sl + NS - 1) % NS);
      else if (st + NS - 1 < nsteps) issue(st + NS - 1);
    }
    if (st > 0 && q_live) {
      mfma_half(0);
      mfma_half(1);
    }
    if (STAG == 2) {
      if (steady) issue_fast(st + NS - 1, (sl + NS - 1) % NS);
      else if (st + NS - 1 < nsteps) issue(st + NS - 1);
    }
    if (q_live) {
      read_p(sl);
      read_q(sl, 0);
      read_q(sl, 4);
    }
  };

  if (nsteps > 0) {
    for (int64_t s = 0; s < NS - 1 && s < nsteps; ++s) issue(s);
    int64_t st = 0;
    // steady groups of NS stages: every DMA they issue (up to stage st + 2 NS - 2) is full
    const int64_t nsteady = nfull >= 2 * NS - 1 ? ((nfull - (2 * NS - 2)) / NS) * NS : 0;
    if (wu >= 4) {
      for (; st < nsteady; st += NS) {
        body_stag(0, st, true);
        body_stag(1, st + 1, true);
        body_stag(2, st + 2, true);
        body_stag(3, st + 3, true);
      }
      for (; st < nsteps; ++st) body_stag((int)(st % NS), st, false);
      if (q_live) {
        mfma_half(0);
        mfma_half(1);
      }
    } else if (do_cs) {
      for (; st < nsteady; st += NS) {
        body_plain(std::true_type{}, 0, st, true);
        body_plain(std::true_type{}, 1, st + 1, true);
        body_plain(std::true_type{}, 2, st + 2, true);
        body_plain(std::true_type{}, 3, st + 3, true);
      }
      for (; st < nsteps; ++st) body_plain(std::true_type{}, (int)(st % NS), st, false);
    } else {
      for (; st < nsteady; st += NS) {
        body_plain(std::false_type{}, 0, st, true);
        body_plain(std::false_type{}, 1, st + 1, true);
        body_plain(std::false_type{}, 2, st + 2, true);
        body_plain(std::false_type{}, 3, st + 3, true);
      }
      for (; st < nsteps; ++st) body_plain(std::false_type{}, (int)(st % NS), st, false);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (do_cs && g == 0) {
#pragma unroll
    for (int ip = 0; ip < 4; ++ip) {
      const int64_t pr = p0 + wp * 64 + ip * 16 + li;
      if (pr < p.P) p.ws_colsum[z * p.P + pr] = accb[ip][0];
    }
  }
  float* out = p.ws + z * p.P * p.Q;
#pragma unroll
  for (int ip = 0; ip < 4; ++ip) {
    const int64_t pr = p0 + wp * 64 + ip * 16 + li;
    if (pr >= p.P) continue;
#pragma unroll
    for (int jq = 0; jq < 8; ++jq) {
      const int64_t qc = q0 + wq * 128 + jq * 16 + 4 * g;
      if (qc >= p.Q) continue;
      *reinterpret_cast<float4_t*>(out + pr * p.Q + qc) = acc[jq][ip];
    }
  }
}

}  // namespace

int llp_cu_count();

int64_t llp_gemm_tn_256_splits(int64_t M, int64_t P, int64_t Q) {
  const int64_t tiles = ((P + TP - 1) / TP) * ((Q + TQ - 1) / TQ);
  const int64_t target = llp_cu_count();   // one wave of workgroups, one per CU
  // whole waves only: tiles * splits <= CUs (33 tiles x 8 splits = 264 blocks ran as two
  // rounds on 256 CUs, the second one 8 blocks long -- the physics first layer's weight gradient)
  const int64_t wave = tiles >= target ? 1 : target / tiles;
  // >= 16 m-steps per split; a short M (the physics student's 256 x 256 layer over a rank's
  // 7,761 rows: 16 splits, 21.5 us) may go down to 4 m-steps while its f32 slabs stay <= 32 MB
  const int64_t s16 = std::min<int64_t>(wave, (M + TKM * 16 - 1) / (TKM * 16));
  int64_t splits = std::min<int64_t>(wave, (M + TKM * 4 - 1) / (TKM * 4));
  const int64_t slab = P * Q * (int64_t)sizeof(float);
  if (splits * slab > (32ll << 20)) splits = std::max<int64_t>(s16, (32ll << 20) / slab);
  return splits < 1 ? 1 : splits;
}

int llp_gemm_tn_bf16_256(const llp_operand* A, const llp_operand* B, int64_t M, int64_t P, int64_t Q, float* ws,
                         float* ws_colsum, int64_t splits, hipStream_t s) {
  PTN p;
  p.ws_colsum = ws_colsum;
  p.A = (const bf16_t*)A->ptr; p.ia = A->idx; p.lda = A->ld;
  p.B = (const bf16_t*)B->ptr; p.ib = B->idx; p.ldb = B->ld;
  p.M = M; p.P = P; p.Q = Q;
  p.m_dev = A->rows_dev ? A->rows_dev : B->rows_dev;
  int64_t mchunk = (M + splits - 1) / splits;
  mchunk = (mchunk + TKM - 1) / TKM * TKM;
  p.mchunk = mchunk > 0 ? mchunk : TKM;
  p.splits = splits;
  p.ws = ws;
  const int64_t tiles = ((P + TP - 1) / TP) * ((Q + TQ - 1) / TQ);
  p.zmajor = 1;
  // the lean loop stages plain operands only; a gathered operand takes the staggered loop
  if (!A->idx && !B->idx && Q <= 128) {
#ifndef LLP_TN_NO_PAD_SKIP
    hipLaunchKernelGGL((gemm_tn_bf16_256c<2, true>), dim3((unsigned)(tiles * splits)), dim3(NTT), 0, s, p);
#else   // A/B build: waves 4-7 compute their padding columns too
    hipLaunchKernelGGL((gemm_tn_bf16_256c<2, false>), dim3((unsigned)(tiles * splits)), dim3(NTT), 0, s, p);
#endif
  } else if (!A->idx && !B->idx)
    hipLaunchKernelGGL((gemm_tn_bf16_256c<2, false>), dim3((unsigned)(tiles * splits)), dim3(NTT), 0, s, p);
  else
    hipLaunchKernelGGL(gemm_tn_bf16_256<2>, dim3((unsigned)(tiles * splits)), dim3(NTT), 0, s, p);
  return (int)hipGetLastError();
}
