// CSR neighbour mean-aggregation for the GraphSAGE teacher.
//
// PyG MessagePassing(aggr='mean') over edge_index (src/models.py:113 via
// SAGEConv, src/sageconv_updated.py:71-72): out[i] = mean over edges e with
// dst[e] = i of x[src[e]], duplicates counted (Q2), empty rows -> 0.  The PyG
// GPU path materialises an E x F message tensor; here one wavefront owns a
// destination row, streams its neighbour rows straight from HBM/L2 with
// 16-byte loads (4 neighbour rows in flight per lane group) and writes the row
// once: HBM traffic = E*F*s (neighbours) + 4E (col) + 4(N+1) (rowptr) + N*F*s.
#include "llp_common.h"

#include <algorithm>
#include <type_traits>

int llp_cu_count();   // gemm256.hip

namespace {

template <typename T>
struct V16;
template <>
struct V16<float> {
  static constexpr int E = 4;
  __device__ static void add(float* a, uint4 v, float w) {
    a[0] += w * __uint_as_float(v.x); a[1] += w * __uint_as_float(v.y);
    a[2] += w * __uint_as_float(v.z); a[3] += w * __uint_as_float(v.w);
  }
  __device__ static uint4 pack(const float* a) {
    return make_uint4(__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]), __float_as_uint(a[3]));
  }
};
template <>
struct V16<bf16_t> {
  static constexpr int E = 8;
  __device__ static void add(float* a, uint4 v, float w) {
    const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[2 * i] += w * __uint_as_float(u[i] << 16);
      a[2 * i + 1] += w * __uint_as_float(u[i] & 0xFFFF0000u);
    }
  }
  __device__ static uint4 pack(const float* a) {
    uint32_t u[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] = (uint32_t)f2bf(a[2 * i]) | ((uint32_t)f2bf(a[2 * i + 1]) << 16);
    return make_uint4(u[0], u[1], u[2], u[3]);
  }
};

// Row of F elements = NCH 16-B chunks.  A wave processes one row; lanes are
// split into G = 64 / NCH_eff groups, each group walks every G-th neighbour and
// the groups are summed through LDS at the end.
template <typename T>
__global__ __launch_bounds__(256) void csr_agg_vec_kernel(int64_t n_rows, int64_t F, const int32_t* __restrict__ rowptr,
                                                          const int32_t* __restrict__ col, const T* __restrict__ x,
                                                          int64_t ldx, const float* __restrict__ inv_deg, int mode,
                                                          const float* __restrict__ bias, T* __restrict__ out,
                                                          int64_t ldo, int accumulate) {
  constexpr int E = V16<T>::E;
  __shared__ float red[4][64 * E];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t nch = F / E;                 // chunks per row (F % E == 0 here)
  const int64_t row = llp_xcd_block(blockIdx.x, gridDim.x) * 4 + w;
  if (row >= n_rows) return;
  const int64_t beg = rowptr[row], end = rowptr[row + 1];
  // chunk sweep: columns in blocks of 64 chunks
  for (int64_t c0 = 0; c0 < nch; c0 += 64) {
    const int64_t cw = min((int64_t)64, nch - c0);           // chunks in this sweep
    // lanes per group = the smallest power of two >= cw (every chunk has a lane)
    const int lanes_per_group = cw > 32 ? 64 : (cw > 16 ? 32 : (cw > 8 ? 16 : (cw > 4 ? 8 : (cw > 2 ? 4 : (int)cw))));
    const int G = 64 / lanes_per_group;
    const int grp = lane / lanes_per_group, gl = lane % lanes_per_group;
    const bool active = gl < cw;
    float acc[E];
#pragma unroll
    for (int i = 0; i < E; ++i) acc[i] = 0.f;
    if (active) {
      const int64_t ch = c0 + gl;
      // 4 neighbours in flight per group, the last round predicated: at the
      // collab degree (~10) a group sees 2-3 neighbours, which the unpredicated
      // tail walked one dependent load at a time.  Accumulation order per group
      // is unchanged (e, e+G, e+2G, ...).
      for (int64_t e = beg + grp; e < end; e += 4 * G) {
        int32_t j[4];
        bool v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[k] = e + k * G < end;
          j[k] = v[k] ? col[e + k * G] : 0;
        }
        uint4 r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          r[k] = v[k] ? *reinterpret_cast<const uint4*>(x + (int64_t)j[k] * ldx + ch * E) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (v[k]) V16<T>::add(acc, r[k], mode ? inv_deg[j[k]] : 1.f);
      }
    }
    if (G > 1) {
      // reduce the G groups through LDS (fixed order -> deterministic)
      float* r = red[w];
      __builtin_amdgcn_wave_barrier();
      if (grp > 0 && active)
#pragma unroll
        for (int i = 0; i < E; ++i) r[(grp * lanes_per_group + gl) * E + i] = acc[i];
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      if (grp == 0 && active)
        for (int g2 = 1; g2 < G; ++g2)
#pragma unroll
          for (int i = 0; i < E; ++i) acc[i] += r[(g2 * lanes_per_group + gl) * E + i];
      __builtin_amdgcn_wave_barrier();
    }
    if (grp == 0 && active) {
      const float sc = mode == 0 ? 1.f / (float)max(end - beg, (int64_t)1) : (mode == 2 ? inv_deg[row] : 1.f);
#pragma unroll
      for (int i = 0; i < E; ++i) acc[i] *= sc;
      if (bias)
#pragma unroll
        for (int i = 0; i < E; ++i) acc[i] += bias[(c0 + gl) * E + i];
      uint4* dst = reinterpret_cast<uint4*>(out + row * ldo + (c0 + gl) * E);
      if (accumulate) {
        float prev[E];
#pragma unroll
        for (int i = 0; i < E; ++i) prev[i] = 0.f;
        V16<T>::add(prev, *dst, 1.f);
#pragma unroll
        for (int i = 0; i < E; ++i) acc[i] += prev[i];
      }
      *dst = V16<T>::pack(acc);
    }
  }
}

// Rows of NCH <= 64 16-B chunks: RPW = 64 / NCH destination rows per wave, one lane per
// chunk of its row, each lane walking the row's neighbours in order with UNR row loads in
// flight (the last round predicated).  Against csr_agg_vec_kernel (one row per wave, its
// neighbours dealt to lane groups and the groups summed through LDS) a wave keeps RPW rows'
// neighbour loads in flight and needs no reduction: bf16 F=128 (256-B rows) takes 4 rows
// per wave.  Per-row accumulation in neighbour order (deterministic).
template <typename T, int NCH, int UNR>
__global__ __launch_bounds__(256) void csr_agg_rows_kernel(int64_t n_rows, const int32_t* __restrict__ rowptr,
                                                           const int32_t* __restrict__ col, const T* __restrict__ x,
                                                           int64_t ldx, const float* __restrict__ inv_deg, int mode,
                                                           const float* __restrict__ bias, T* __restrict__ out,
                                                           int64_t ldo, int accumulate) {
  constexpr int E = V16<T>::E;
  constexpr int RPW = 64 / NCH;
  const int lane = threadIdx.x & 63;
  const int rl = lane / NCH, ch = lane % NCH;
  // each XCD a contiguous range of rows: with a locality-ordered graph (llp_sage.locality_order)
  // the neighbour rows of those rows are L2 hits
  const int64_t row = (llp_xcd_block(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6)) * RPW + rl;
  if (row >= n_rows) return;
  const int64_t beg = rowptr[row], end = rowptr[row + 1];
  float acc[E];
#pragma unroll
  for (int i = 0; i < E; ++i) acc[i] = 0.f;
  const T* xc = x + ch * E;
  for (int64_t e = beg; e < end; e += UNR) {
    int32_t j[UNR];
    bool v[UNR];
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      v[k] = e + k < end;
      j[k] = v[k] ? col[e + k] : 0;
    }
    uint4 r[UNR];
#pragma unroll
    for (int k = 0; k < UNR; ++k)
      r[k] = v[k] ? *reinterpret_cast<const uint4*>(xc + (int64_t)j[k] * ldx) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < UNR; ++k)
      if (v[k]) V16<T>::add(acc, r[k], mode ? inv_deg[j[k]] : 1.f);
  }
  const float sc = mode == 0 ? 1.f / (float)max(end - beg, (int64_t)1) : (mode == 2 ? inv_deg[row] : 1.f);
#pragma unroll
  for (int i = 0; i < E; ++i) acc[i] *= sc;
  if (bias)
#pragma unroll
    for (int i = 0; i < E; ++i) acc[i] += bias[ch * E + i];
  uint4* dst = reinterpret_cast<uint4*>(out + row * ldo + ch * E);
  if (accumulate) {
    float prev[E];
#pragma unroll
    for (int i = 0; i < E; ++i) prev[i] = 0.f;
    V16<T>::add(prev, *dst, 1.f);
#pragma unroll
    for (int i = 0; i < E; ++i) acc[i] += prev[i];
  }
  *dst = V16<T>::pack(acc);
}

// Rows of NCH <= 64 16-B chunks with the block's CSR slice staged in LDS (round 5).  The rows-per-wave
// kernel above walked each row behind a dependent chain: rowptr, then per UNR neighbours a col[]
// load and only then the neighbour rows, so at the collab degree (~10) a wave waited out ~7 global
// latencies and the aggregate ran at 3.1-3.9 TB/s counted.  Here a workgroup owns
// TR = 4 * RPW consecutive rows: it loads their rowptr slice, then the whole col[] slice (and for the
// degree-weighted modes the per-neighbour weights) with one coalesced pass into LDS, and every lane
// then issues its row's neighbour loads UNR at a time with nothing in front of them but an LDS read.
// Three global latencies per row tile instead of 2 + 2 * deg / UNR.  Rows whose slice overflows the
// LDS capacity (hubs) read the excess indices from global memory.  Per-row accumulation in
// neighbour order, the same arithmetic as csr_agg_rows_kernel: bit-identical outputs.
constexpr int AGG_CAP = 1024;   // staged col[] entries per workgroup (4 KiB, + 4 KiB of weights)
#ifndef AGG_UNR
#define AGG_UNR 4               // neighbour rows in flight per lane (4 / 6 / 8 / 16: profiles/r05_agg_unr_ab.txt)
#endif
#ifndef AGG_PIPE_UNR
#define AGG_PIPE_UNR 12         // the pipelined kernel's neighbour rows in flight per lane (collab degree ~10)
#endif
#ifndef AGG_WG_PER_CU
#define AGG_WG_PER_CU 4
#endif
#ifndef AGG_WAVES
#define AGG_WAVES 4             // waves per workgroup of csr_agg_lds_kernel (rows per workgroup: AGG_WAVES * RPW)
#endif

template <typename T, int NCH, int UNR>
__global__ __launch_bounds__(64 * AGG_WAVES) void csr_agg_lds_kernel(int64_t n_rows, const int32_t* __restrict__ rowptr,
                                                          const int32_t* __restrict__ col, const T* __restrict__ x,
                                                          int64_t ldx, const float* __restrict__ inv_deg, int mode,
                                                          const float* __restrict__ bias, T* __restrict__ out,
                                                          int64_t ldo, int accumulate) {
  constexpr int E = V16<T>::E;
  constexpr int RPW = 64 / NCH;
  constexpr int TR = AGG_WAVES * RPW;   // rows per workgroup
  __shared__ int32_t s_ptr[TR + 1];
  __shared__ int32_t s_col[AGG_CAP];
  __shared__ float s_w[AGG_CAP];
  const int t = threadIdx.x;
  // each XCD a contiguous range of row tiles (locality-ordered graphs: neighbour rows hit its L2)
  const int64_t r0 = llp_xcd_block(blockIdx.x, gridDim.x) * TR;
  if (t <= TR) s_ptr[t] = rowptr[min(r0 + t, n_rows)];
  __syncthreads();
  const int32_t base = s_ptr[0];
  const int32_t n_e = s_ptr[TR] - base;
  const int32_t n_st = min(n_e, AGG_CAP);
  for (int32_t i = t; i < n_st; i += 64 * AGG_WAVES) {
    const int32_t c = col[base + i];
    s_col[i] = c;
    if (mode) s_w[i] = inv_deg[c];
  }
  __syncthreads();
  const int lane = t & 63;
  const int rl = lane / NCH, ch = lane % NCH;
  const int lr = (t >> 6) * RPW + rl;
  const int64_t row = r0 + lr;
  if (row >= n_rows) return;
  const int32_t beg = s_ptr[lr] - base, end = s_ptr[lr + 1] - base;
  float acc[E];
#pragma unroll
  for (int i = 0; i < E; ++i) acc[i] = 0.f;
  const T* xc = x + ch * E;
#ifndef LLP_AGG_NO_LDS_FAST
  if (n_e <= AGG_CAP) {
    // every index (and weight) of the workgroup is in LDS (all but hub-holding workgroups): the
    // mixed form below selects per lane between the LDS slice and col[] / inv_deg in global
    // memory, which hipcc compiles to divergent branches with a full vmcnt + lgkmcnt wait per
    // neighbour and FLAT loads for the weights.  Same values, same order: bit-identical.
    for (int32_t e = beg; e < end; e += UNR) {
      int32_t j[UNR];
      float wt[UNR];
      bool v[UNR];
#pragma unroll
      for (int k = 0; k < UNR; ++k) {
        const int32_t q = e + k;
        v[k] = q < end;
        const int32_t qq = v[k] ? q : beg;   // an in-range slot (its value unused)
        j[k] = v[k] ? s_col[qq] : 0;
        wt[k] = (mode && v[k]) ? s_w[qq] : 1.f;
      }
      uint4 r[UNR];
#pragma unroll
      for (int k = 0; k < UNR; ++k)
        r[k] = v[k] ? *reinterpret_cast<const uint4*>(xc + (int64_t)j[k] * ldx) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int k = 0; k < UNR; ++k)
        if (v[k]) V16<T>::add(acc, r[k], wt[k]);
    }
  } else
#endif
  for (int32_t e = beg; e < end; e += UNR) {
    int32_t j[UNR];
    float wt[UNR];
    bool v[UNR];
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const int32_t q = e + k;
      v[k] = q < end;
      const bool st = q < AGG_CAP;
      j[k] = v[k] ? (st ? s_col[q] : col[base + q]) : 0;
      wt[k] = 1.f;
      if (mode && v[k]) wt[k] = st ? s_w[q] : inv_deg[j[k]];
    }
    uint4 r[UNR];
#pragma unroll
    for (int k = 0; k < UNR; ++k)
      r[k] = v[k] ? *reinterpret_cast<const uint4*>(xc + (int64_t)j[k] * ldx) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < UNR; ++k)
      if (v[k]) V16<T>::add(acc, r[k], wt[k]);
  }
  const float sc = mode == 0 ? 1.f / (float)max(end - beg, 1) : (mode == 2 ? inv_deg[row] : 1.f);
#pragma unroll
  for (int i = 0; i < E; ++i) acc[i] *= sc;
  if (bias)
#pragma unroll
    for (int i = 0; i < E; ++i) acc[i] += bias[ch * E + i];
  uint4* dst = reinterpret_cast<uint4*>(out + row * ldo + ch * E);
  if (accumulate) {
    float prev[E];
#pragma unroll
    for (int i = 0; i < E; ++i) prev[i] = 0.f;
    V16<T>::add(prev, *dst, 1.f);
#pragma unroll
    for (int i = 0; i < E; ++i) acc[i] += prev[i];
  }
  *dst = V16<T>::pack(acc);
}

// Rows of NCH <= 64 16-B chunks, persistent and software-pipelined per wave (round 5, second
// form; measured SLOWER than csr_agg_lds_kernel and kept only as the LLP_AGG_PIPE A/B build:
// bf16 F = 128 forward 67-78 against 58 us, profiles/r05_agg_ab.txt).  The LDS-staged kernel above still pays three serialized memory latencies per workgroup
// of 4 * RPW rows (rowptr, then col[], then the neighbour rows) and its workgroups live one tile
// each, so at the collab degree the aggregate stayed latency-bound (bf16 F = 128: 58 us, 0.28 of
// HBM on compulsory bytes, profiles/r05_agg_ab.txt).  Here every wave walks many tiles of RPW
// rows and keeps the index stages one and two tiles ahead: while it issues tile k's neighbour
// loads it has tile k + 1's col[] slice and tile k + 2's rowptr values in flight, so a tile costs
// about one memory latency.  The col[] slice lives in two registers per lane (128 entries; a
// longer slice, i.e. a hub, reads the excess from global memory) and goes through the wave's own
// 512 B of LDS, from which each lane picks its neighbour ids (the row walks diverge, and a
// cross-lane read of an inactive lane's register is undefined).  Tiles are dealt per XCD in contiguous ranges (XCD x takes
// tiles [x T / 8, (x + 1) T / 8), its waves round-robin inside), so the tiles in flight on an XCD
// are neighbours in the (locality-ordered) graph.  Per-row accumulation in neighbour order, the
// same arithmetic as the kernels above: bit-identical outputs.
template <typename T, int NCH, int UNR>
__global__ __launch_bounds__(256) void csr_agg_pipe_kernel(int64_t n_rows, const int32_t* __restrict__ rowptr,
                                                           const int32_t* __restrict__ col, const T* __restrict__ x,
                                                           int64_t ldx, const float* __restrict__ inv_deg, int mode,
                                                           const float* __restrict__ bias, T* __restrict__ out,
                                                           int64_t ldo, int accumulate, int64_t n_tiles) {
  constexpr int E = V16<T>::E;
  constexpr int RPW = 64 / NCH;
  const int lane = threadIdx.x & 63;
  const int rl = lane / NCH, ch = lane % NCH;
  const int64_t xcd = blockIdx.x % 8, wg_x = blockIdx.x / 8;
  const int64_t nwg_x = ((int64_t)gridDim.x - xcd + 7) / 8;
  const int64_t W = nwg_x * 4;                                   // waves on this XCD
  const int64_t t_lo = xcd * n_tiles / 8, t_hi = (xcd + 1) * n_tiles / 8;
  int64_t t = t_lo + wg_x * 4 + (threadIdx.x >> 6);
  auto load_rp = [&](int64_t tt) -> int32_t {
    return (tt < t_hi && lane <= RPW) ? rowptr[min(tt * RPW + lane, n_rows)] : 0;
  };
  auto load_col = [&](int32_t rp, int32_t& ca, int32_t& cb, int32_t& base) {
    base = __shfl(rp, 0, 64);
    const int32_t len = __shfl(rp, RPW, 64) - base;
    ca = lane < len ? col[base + lane] : 0;
    cb = lane + 64 < len ? col[base + 64 + lane] : 0;
  };
  int32_t rp0 = load_rp(t), rp1 = load_rp(t + W);
  int32_t ca0, cb0, base0;
  load_col(rp0, ca0, cb0, base0);
  const T* xc = x + ch * E;
  __shared__ int32_t s_col[4][128];
  int32_t* sc = s_col[threadIdx.x >> 6];
  for (; t < t_hi; t += W) {
    // this tile's col[] slice into the wave's LDS (every lane finished the previous tile's walk)
    sc[lane] = ca0;
    sc[64 + lane] = cb0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the index stages of the next tiles, issued before this tile's neighbour loads
    const int32_t rp2 = load_rp(t + 2 * W);
    int32_t ca1 = 0, cb1 = 0, base1 = 0;
    if (t + W < t_hi) load_col(rp1, ca1, cb1, base1);
    const int64_t row = t * RPW + rl;
    const int32_t beg = __shfl(rp0, rl, 64) - base0, end = __shfl(rp0, rl + 1, 64) - base0;
    float acc[E];
#pragma unroll
    for (int i = 0; i < E; ++i) acc[i] = 0.f;
    for (int32_t e = beg; e < end; e += UNR) {
      int32_t j[UNR];
      bool v[UNR];
#pragma unroll
      for (int k = 0; k < UNR; ++k) {
        const int32_t q = e + k;
        v[k] = q < end;
        j[k] = v[k] ? (q < 128 ? sc[q] : col[base0 + q]) : 0;
      }
      uint4 r[UNR];
      float wt[UNR];
#pragma unroll
      for (int k = 0; k < UNR; ++k) {
        r[k] = v[k] ? *reinterpret_cast<const uint4*>(xc + (int64_t)j[k] * ldx) : make_uint4(0, 0, 0, 0);
        wt[k] = (mode && v[k]) ? inv_deg[j[k]] : 1.f;
      }
#pragma unroll
      for (int k = 0; k < UNR; ++k)
        if (v[k]) V16<T>::add(acc, r[k], wt[k]);
    }
    if (row < n_rows) {
      const float sc = mode == 0 ? 1.f / (float)max(end - beg, 1) : (mode == 2 ? inv_deg[row] : 1.f);
#pragma unroll
      for (int i = 0; i < E; ++i) acc[i] *= sc;
      if (bias)
#pragma unroll
        for (int i = 0; i < E; ++i) acc[i] += bias[ch * E + i];
      uint4* dst = reinterpret_cast<uint4*>(out + row * ldo + ch * E);
      if (accumulate) {
        float prev[E];
#pragma unroll
        for (int i = 0; i < E; ++i) prev[i] = 0.f;
        V16<T>::add(prev, *dst, 1.f);
#pragma unroll
        for (int i = 0; i < E; ++i) acc[i] += prev[i];
      }
      *dst = V16<T>::pack(acc);
    }
    rp0 = rp1;
    rp1 = rp2;
    ca0 = ca1;
    cb0 = cb1;
    base0 = base1;
  }
}

// Scalar fallback for feature widths that are not a multiple of the vector.
template <typename T>
__global__ __launch_bounds__(256) void csr_agg_scalar_kernel(int64_t n_rows, int64_t F,
                                                             const int32_t* __restrict__ rowptr,
                                                             const int32_t* __restrict__ col, const T* __restrict__ x,
                                                             int64_t ldx, const float* __restrict__ inv_deg, int mode,
                                                             const float* __restrict__ bias, T* __restrict__ out,
                                                             int64_t ldo, int accumulate) {
  const int lane = threadIdx.x & 63;
  const int64_t row = llp_xcd_block(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
  if (row >= n_rows) return;
  const int64_t beg = rowptr[row], end = rowptr[row + 1];
  const float sc = mode == 0 ? 1.f / (float)max(end - beg, (int64_t)1) : (mode == 2 ? inv_deg[row] : 1.f);
  for (int64_t f = lane; f < F; f += 64) {
    float acc = 0.f;
    for (int64_t e = beg; e < end; ++e) {
      const int32_t j = col[e];
      float v;
      if constexpr (sizeof(T) == 2) v = bf2f(x[(int64_t)j * ldx + f]); else v = x[(int64_t)j * ldx + f];
      acc += (mode ? inv_deg[j] : 1.f) * v;
    }
    acc *= sc;
    if (bias) acc += bias[f];
    T* d = out + row * ldo + f;
    if constexpr (sizeof(T) == 2) {
      if (accumulate) acc += bf2f(*d);
      *d = f2bf(acc);
    } else {
      if (accumulate) acc += *d;
      *d = acc;
    }
  }
}

}  // namespace

static int csr_aggregate_launch(int dtype, int64_t n_rows, int64_t F, const int32_t* rowptr, const int32_t* col,
                                const void* x, int64_t ldx, const float* inv_deg, int mode, const float* bias,
                                void* out, int64_t ldo, int accumulate, hipStream_t s) {
  if (n_rows == 0 || F == 0) return LLP_OK;
  const int es = dtype == LLP_BF16 ? 2 : 4;
  const int E = 16 / es;
  const bool vec = (F % E == 0) && (ldx % E == 0) && (ldo % E == 0) && ((uintptr_t)x % 16 == 0) &&
                   ((uintptr_t)out % 16 == 0);
  dim3 grid(ceil_div_u(n_rows, 4));
#ifdef LLP_AGG_GROUPS   // A/B build: csr_agg_vec_kernel for every width
  const int64_t nch = 0;
#else
  const int64_t nch = vec ? F / E : 0;
#endif
  if (nch == 8 || nch == 16 || nch == 32 || nch == 64) {   // rows of 8..64 chunks: rows per wave
    const dim3 g2(ceil_div_u(n_rows, 4 * (64 / nch)));
    auto go = [&](auto kern, auto* xx, auto* oo) {
      hipLaunchKernelGGL(kern, g2, dim3(256), 0, s, n_rows, rowptr, col, xx, ldx, inv_deg, mode, bias, oo, ldo,
                         accumulate);
    };
    auto pick = [&](auto* xx, auto* oo) {
      using TT = std::remove_const_t<std::remove_pointer_t<decltype(xx)>>;
#if defined(LLP_AGG_ROWS_DIRECT)   // A/B build: the round-4 kernel (col[] read behind each row walk)
      if (nch == 8) go(csr_agg_rows_kernel<TT, 8, 4>, xx, oo);
      else if (nch == 16) go(csr_agg_rows_kernel<TT, 16, 4>, xx, oo);
      else if (nch == 32) go(csr_agg_rows_kernel<TT, 32, 4>, xx, oo);
      else go(csr_agg_rows_kernel<TT, 64, 4>, xx, oo);
#elif defined(LLP_AGG_PIPE)        // A/B build: persistent software-pipelined waves (slower)
      const int64_t n_tiles = (n_rows + (64 / nch) - 1) / (64 / nch);
      const int64_t cap = (int64_t)llp_cu_count() * AGG_WG_PER_CU;
      const dim3 gp((unsigned)std::max<int64_t>(8, std::min<int64_t>((n_tiles + 3) / 4, cap)));
      auto gop = [&](auto kern, auto* xx2, auto* oo2) {
        hipLaunchKernelGGL(kern, gp, dim3(256), 0, s, n_rows, rowptr, col, xx2, ldx, inv_deg, mode, bias, oo2, ldo,
                           accumulate, n_tiles);
      };
      if (nch == 8) gop(csr_agg_pipe_kernel<TT, 8, AGG_PIPE_UNR>, xx, oo);
      else if (nch == 16) gop(csr_agg_pipe_kernel<TT, 16, AGG_PIPE_UNR>, xx, oo);
      else if (nch == 32) gop(csr_agg_pipe_kernel<TT, 32, AGG_PIPE_UNR>, xx, oo);
      else gop(csr_agg_pipe_kernel<TT, 64, AGG_PIPE_UNR>, xx, oo);
#else                              // one LDS-staged tile per workgroup (the default)
      const dim3 gl(ceil_div_u(n_rows, AGG_WAVES * (64 / nch)));
      auto gol = [&](auto kern, auto* xx2, auto* oo2) {
        hipLaunchKernelGGL(kern, gl, dim3(64 * AGG_WAVES), 0, s, n_rows, rowptr, col, xx2, ldx, inv_deg, mode, bias,
                           oo2, ldo, accumulate);
      };
      if (nch == 8) gol(csr_agg_lds_kernel<TT, 8, AGG_UNR>, xx, oo);
      else if (nch == 16) gol(csr_agg_lds_kernel<TT, 16, AGG_UNR>, xx, oo);
      else if (nch == 32) gol(csr_agg_lds_kernel<TT, 32, AGG_UNR>, xx, oo);
      else gol(csr_agg_lds_kernel<TT, 64, AGG_UNR>, xx, oo);
#endif
    };
    if (dtype == LLP_BF16) pick((const bf16_t*)x, (bf16_t*)out);
    else pick((const float*)x, (float*)out);
    LLP_LAUNCH_CHECK();
    return LLP_OK;
  }
  if (dtype == LLP_BF16) {
    if (vec)
      hipLaunchKernelGGL(csr_agg_vec_kernel<bf16_t>, grid, dim3(256), 0, s, n_rows, F, rowptr, col, (const bf16_t*)x,
                         ldx, inv_deg, mode, bias, (bf16_t*)out, ldo, accumulate);
    else
      hipLaunchKernelGGL(csr_agg_scalar_kernel<bf16_t>, grid, dim3(256), 0, s, n_rows, F, rowptr, col,
                         (const bf16_t*)x, ldx, inv_deg, mode, bias, (bf16_t*)out, ldo, accumulate);
  } else {
    if (vec)
      hipLaunchKernelGGL(csr_agg_vec_kernel<float>, grid, dim3(256), 0, s, n_rows, F, rowptr, col, (const float*)x, ldx,
                         inv_deg, mode, bias, (float*)out, ldo, accumulate);
    else
      hipLaunchKernelGGL(csr_agg_scalar_kernel<float>, grid, dim3(256), 0, s, n_rows, F, rowptr, col, (const float*)x,
                         ldx, inv_deg, mode, bias, (float*)out, ldo, accumulate);
  }
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_csr_aggregate(int dtype, int64_t n_rows, int64_t F, const int32_t* rowptr, const int32_t* col,
                                 const void* x, int64_t ldx, const float* inv_deg, int mode, void* out, int64_t ldo,
                                 int accumulate, void* stream) {
  LLP_CHECK_ARG(n_rows == 0 || F == 0 || (rowptr && x && out), "llp_csr_aggregate: null pointer");
  LLP_CHECK_ARG(mode == 0 || (mode == 1 && inv_deg), "llp_csr_aggregate: mode 1 needs inv_deg");
  return csr_aggregate_launch(dtype, n_rows, F, rowptr, col, x, ldx, inv_deg, mode, nullptr, out, ldo, accumulate,
                              (hipStream_t)stream);
}

// GCN propagation (PyG GCNConv after gcn_norm): out[i] = dinv[i] * sum_{j in row i} dinv[j] * x[j] (+ bias).
// With the self-loop CSR by destination this is the forward; with the transposed CSR and no bias, the
// backward dX of the same propagation.
extern "C" int llp_gcn_aggregate(int dtype, int64_t n_rows, int64_t F, const int32_t* rowptr, const int32_t* col,
                                 const void* x, int64_t ldx, const float* dinv, const float* bias, void* out,
                                 int64_t ldo, int accumulate, void* stream) {
  LLP_CHECK_ARG(rowptr && col && x && out && dinv, "llp_gcn_aggregate: null pointer");
  return csr_aggregate_launch(dtype, n_rows, F, rowptr, col, x, ldx, dinv, 2, bias, out, ldo, accumulate,
                              (hipStream_t)stream);
}
