// Large-tile f32 weight-gradient GEMM (TN form) for the fp32 path (the reference's own
// arithmetic, src/main.py:132):
//
//   ws[z][p][q] = sum_{m in split z} A[m, p] * B[m, q]      (A = dY, B = X; f32 slabs)
//   ws_colsum[z][p] = sum_{m in split z} A[m, p]            (bias gradient, optional)
//
// gemm256_tn.hip's bf16 structure on f32 operands: 256 (p) x 256 (q) tile per 512-thread
// workgroup, one workgroup per CU, the rows of a split staged by global_load_lds_dwordx4 into
// a 4-stage LDS ring (3 stages in flight, counted vmcnt + raw barriers).  A stage is 16 rows:
// [16][256] f32 images of 1 KiB rows (16 KiB each, the bf16 ring's bytes); no wave stagger (an
// f32 stage is 8x the MFMA time of a bf16 one on the same bytes, and the stagger's held
// fragments would spill).  Fragments are single floats read by ds_read_b32: for
// v_mfma_f32_16x16x4_f32, lane (li, g) takes row 4 t + g of the stage (k-slot g) at column
// 16 i + li, so per accumulator the sum runs over m in order, as in gemm.hip's register-staged
// f32 TN kernel.  16-B chunk swizzle: chunk ^ 4 on odd rows, so the two 16-lane halves of a
// ds_read_b32 lane group (rows r and r + 1, the same 16 columns) fall on disjoint banks.
// The bias gradient rides along as in the bf16 kernel: the q0 == 0 tiles' waves 0-3 also
// multiply their A fragments by 1.0.
// Round 5: the register-staged 128 x 128 f32 TN kernel ran at 116-117 TF/s against
// hipBLASLt's 125-127 at the dominant shape; the persistent f32 NT kernel with this staging
// went from 124 to 141 TF/s.
#include "llp_common.h"

namespace {

constexpr int TP = 256, TQ = 256, TKM = 16;
constexpr int NTT = 512;
constexpr int NS = 4;                          // LDS ring depth (stages of TKM rows)
constexpr int IMG_BYTES = TKM * 1024;          // one [16][256] f32 image = 16 KiB
constexpr int LB0 = NS * IMG_BYTES;            // A images of the 4 slots in [0, 64 KiB), B images after:
                                               // every fragment offset fits the ds_read offset field

__device__ __attribute__((aligned(16))) uint4 g_zero_row_f32[64];   // 1 KiB of zeros (static init)

struct PTNF {
  const float* A; int64_t lda;
  const float* B; int64_t ldb;
  int64_t M, P, Q, mchunk, splits;
  float* ws;
  float* ws_colsum;       // [splits][P] column sums of A (bias gradient), or NULL
  const int32_t* m_dev;   // device row count (llp_operand.rows_dev) or NULL
};

__device__ __forceinline__ int64_t xcd_remap3(int64_t bid, int64_t nwg) {
  if (nwg < 8) return bid;
  const int64_t q = nwg / 8, r = nwg % 8;
  const int64_t xcd = bid % 8, loc = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

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

// byte offset of float (row, col) in a [16][256] image: 16-B chunk col / 4, XOR 4 on odd rows
__device__ __forceinline__ int img_off(int row, int col) {
  return row * 1024 + (((col >> 2) ^ ((row & 1) << 2)) << 4) + ((col & 3) << 2);
}

__global__ __launch_bounds__(NTT) void gemm_tn_f32_256(PTNF p) {
  __shared__ __attribute__((aligned(16))) uint4 smem[2 * NS * IMG_BYTES / 16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int64_t tilesQ = (p.Q + TQ - 1) / TQ;
  const int64_t tilesP = (p.P + TP - 1) / TP;
  const int64_t tiles = tilesP * tilesQ;
  // split-major block order: the tiles of one split (the same rows of A and B) are consecutive,
  // so one XCD's L2 serves each staged row to all of them (gemm256_tn.hip tn_block)
  const int64_t lt = xcd_remap3(blockIdx.x, tiles * p.splits);
  const int64_t tile = lt % tiles, z = lt / tiles;
  const int64_t p0 = (tile / tilesQ) * TP, q0 = (tile % tilesQ) * TQ;
  if (p.m_dev) {   // live rows from the device count; the grid (splits) is the host M's
    const int64_t c = *p.m_dev;
    p.M = c < p.M ? (c > 0 ? c : 0) : p.M;
    const int64_t mc = (p.M + p.splits - 1) / p.splits;
    p.mchunk = mc > 0 ? (mc + TKM - 1) / TKM * TKM : TKM;
  }
  const int64_t mbeg = z * p.mchunk;
  const int64_t mend = min(p.M, mbeg + p.mchunk);
  const int wu = __builtin_amdgcn_readfirstlane(w);

  // DMA: wave w stages image rows 2w, 2w + 1 of each operand, one 1-KiB row per instruction:
  // lane = physical 16-B chunk, logical chunk lane ^ (4 if the row is odd); columns past P / Q
  // are clamped to a valid address (their products are never stored)
  const int capA = (int)max((int64_t)0, (p.P - p0) - 4), capB = (int)max((int64_t)0, (p.Q - q0) - 4);
  const float* zrow = reinterpret_cast<const float*>(g_zero_row_f32);
  const uint32_t lds0 = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) void*)smem);
  auto issue = [&](int64_t st) {
    const int64_t mt = mbeg + st * TKM;
    const uint32_t sA = lds0 + (uint32_t)((st % NS) * IMG_BYTES);
    const uint32_t sB = sA + LB0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = 2 * wu + i;
      const int lc = (lane ^ ((r & 1) << 2)) * 4;
      const int64_t m = mt + r;
      const bool v = m < mend;
      const float* srcA = v ? p.A + m * p.lda + p0 + min(lc, capA) : zrow + min(lc, capA);
      const float* srcB = v ? p.B + m * p.ldb + q0 + min(lc, capB) : zrow + min(lc, capB);
      glds16(srcA, __builtin_amdgcn_readfirstlane(sA + (uint32_t)(r * 1024)));
      glds16(srcB, __builtin_amdgcn_readfirstlane(sB + (uint32_t)(r * 1024)));
    }
  };

  const int wq = w >> 2, wp = w & 3;
  float4_t acc[8][4];   // [q-tile jq][p-tile ip]: rows q = 16 jq + 4 g + r, col p = 16 ip + li
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = float4_t{0.f, 0.f, 0.f, 0.f};
  const bool do_cs = p.ws_colsum != nullptr && q0 == 0 && wq == 0;
  // column sums in two levels: the ones-MFMAs accumulate 8 stages (128 rows) in accb_in, which is
  // then added to accb.  One running sum over a split's ~37k rows (the predictor's bias
  // gradients, sums that cancel to ~1e-5 of their terms) drifted 100x past the f32 reference's
  // error in the full-size oracle test; the register-staged path summed 512-row blocks.
  float4_t accb[4], accb_in[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) accb[b] = accb_in[b] = float4_t{0.f, 0.f, 0.f, 0.f};

  // per-lane fragment offsets (bytes, slot 0, t = 0): A at (g, 64 wp + 16 ip + li), B at
  // (g, 128 wq + 16 jq + li).  Row 4 t + g has the parity of g, so step t adds 4 KiB and slot s
  // 16 KiB: constants that fold into the ds_read offset field
  int oA[4], oB[8];
#pragma unroll
  for (int ip = 0; ip < 4; ++ip) oA[ip] = img_off(g, wp * 64 + ip * 16 + li);
#pragma unroll
  for (int jq = 0; jq < 8; ++jq) oB[jq] = img_off(g, wq * 128 + jq * 16 + li);
  typedef __attribute__((address_space(3))) float lds_f;
  typedef __attribute__((address_space(3))) char lds_c;
  lds_c* sbase = (lds_c*)((__attribute__((address_space(3))) uint4*)smem);
  // the fragments of one k-step t (4 A + 8 B floats), double-buffered: step t + 1's reads are
  // issued before step t's MFMAs (hipcc counts the lgkm waits; the DMA is vmcnt only)
  float fa[2][4], fb[2][8];
  auto read_t = [&](int slot, int t, int buf) {
    lds_c* bA = sbase + slot * IMG_BYTES + t * 4096;
    lds_c* bB = sbase + LB0 + slot * IMG_BYTES + t * 4096;
#pragma unroll
    for (int ip = 0; ip < 4; ++ip) fa[buf][ip] = *(lds_f*)(bA + oA[ip]);
#pragma unroll
    for (int jq = 0; jq < 8; ++jq) fb[buf][jq] = *(lds_f*)(bB + oB[jq]);
  };
  auto mfma_t = [&](int buf) {
    if (do_cs) {
#pragma unroll
      for (int ip = 0; ip < 4; ++ip) accb_in[ip] = __builtin_amdgcn_mfma_f32_16x16x4f32(1.f, fa[buf][ip], accb_in[ip], 0, 0, 0);
    }
#pragma unroll
    for (int jq = 0; jq < 8; ++jq)
#pragma unroll
      for (int ip = 0; ip < 4; ++ip)
        acc[jq][ip] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[buf][jq], fa[buf][ip], acc[jq][ip], 0, 0, 0);
  };

  if (mbeg < mend) {
    const int64_t nsteps = (mend - mbeg + TKM - 1) / TKM;
    for (int64_t s = 0; s < NS - 1 && s < nsteps; ++s) issue(s);
    for (int64_t st = 0; st < nsteps; ++st) {
      vm_wait(min(nsteps - 1, st + NS - 2) - st);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // every wave's reads of stage st-1 done
      __builtin_amdgcn_s_barrier();                         // ... and stage st landed for every wave
      if (st + NS - 1 < nsteps) issue(st + NS - 1);         // into the buffer of stage st-1
      const int slot = (int)(st % NS);
      read_t(slot, 0, 0);
      read_t(slot, 1, 1);
      __builtin_amdgcn_s_setprio(1);
      mfma_t(0);
      read_t(slot, 2, 0);
      mfma_t(1);
      read_t(slot, 3, 1);
      mfma_t(0);
      mfma_t(1);
      __builtin_amdgcn_s_setprio(0);
      if (do_cs && ((st & 7) == 7 || st + 1 == nsteps)) {
#pragma unroll
        for (int ip = 0; ip < 4; ++ip) {
          accb[ip] += accb_in[ip];
          accb_in[ip] = float4_t{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
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

}  // namespace

int llp_cu_count();

// splits of the f32 256-tile TN launch.  Each split's rows are one running f32 sum per output
// element in the MFMA accumulators, so the split length sets the rounding error: at the collab
// predictor's 603k rows, 16 splits of ~37.7k rows left its first-layer weight gradient at 2.8x
// the error of the reference's own fp32 arithmetic (CPU sgemm sums K in blocks of a few hundred)
// in the full-size oracle test.  Splits of at most TN_F32_ROWS rows, a whole number of waves of
// one workgroup per CU; the f32 slabs (splits x P x Q) are summed in split order by slab_reduce.
// At that shape: 160 splits of 3.8k rows, 640 MB of slabs written and read once (~0.25 ms of
// HBM time against the launch's ~9 ms of MFMA time).
constexpr int64_t TN_F32_ROWS = 4096;
int64_t llp_gemm_tn_f32_256_splits(int64_t M, int64_t P, int64_t Q) {
  const int64_t tiles = ((P + TP - 1) / TP) * ((Q + TQ - 1) / TQ);
  const int64_t target = llp_cu_count();
  const int64_t wave = tiles >= target ? 1 : target / tiles;
  const int64_t need = (M + TN_F32_ROWS - 1) / TN_F32_ROWS;           // splits for <= TN_F32_ROWS rows each
  int64_t splits = need <= wave ? std::min<int64_t>(wave, (M + TKM * 8 - 1) / (TKM * 8))
                                : (need + wave - 1) / wave * wave;   // whole waves
  return splits < 1 ? 1 : splits;
}

// The caller checked: plain operands (no gather, no Hadamard), 16-B aligned rows, P % 4 == 0,
// Q % 4 == 0.  ws: [splits][P][Q] f32 slabs; ws_colsum: [splits][P] or NULL.
int llp_gemm_tn_f32_256(const llp_operand* A, const llp_operand* B, int64_t M, int64_t P, int64_t Q, float* ws,
                        float* ws_colsum, int64_t splits, hipStream_t s) {
  PTNF p;
  p.A = (const float*)A->ptr; p.lda = A->ld;
  p.B = (const float*)B->ptr; p.ldb = B->ld;
  p.M = M; p.P = P; p.Q = Q;
  p.m_dev = A->rows_dev ? A->rows_dev : B->rows_dev;
  int64_t mchunk = (M + splits - 1) / splits;
  mchunk = (mchunk + TKM - 1) / TKM * TKM;
  p.mchunk = mchunk > 0 ? mchunk : TKM;
  p.splits = splits;
  p.ws = ws;
  p.ws_colsum = ws_colsum;
  const int64_t tiles = ((P + TP - 1) / TP) * ((Q + TQ - 1) / TQ);
  hipLaunchKernelGGL(gemm_tn_f32_256, dim3((unsigned)(tiles * splits)), dim3(NTT), 0, s, p);
  return (int)hipGetLastError();
}
