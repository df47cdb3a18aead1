// Bandwidth-bound pieces of the step: Hadamard backward, clip_grad_norm_ + Adam
// (multi-tensor, fused with the bf16 weight-shadow refresh), small utilities.
#include "llp_common.h"

#include <type_traits>

namespace {

template <typename T>
__device__ __forceinline__ float ldf(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ldf<float>(const float* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ldf<bf16_t>(const bf16_t* p, int64_t i) { return bf2f(p[i]); }
__device__ __forceinline__ void stf(float* p, int64_t i, float v) { p[i] = v; }
__device__ __forceinline__ void stf(bf16_t* p, int64_t i, float v) { p[i] = f2bf(v); }

// ---------------------------------------------------------------- Hadamard backward
// blockIdx.x < B: anchor b (its anchor row + C context rows);
// else: a chunk of 64 label pairs.  Threads own columns.
// drow != NULL: dZ[r, :] = drow[r] (the 'inner' predictor, whose logit is sum(x_i*x_j)).
template <typename T>
__device__ __forceinline__ float dz_at(const T* dZ, const float* drow, int64_t r, int64_t H, int64_t n) {
  return drow ? drow[r] : ldf<T>(dZ + r * H, n);
}

template <typename T>
__global__ __launch_bounds__(256) void hadamard_bwd_blocks_kernel(int64_t B, int64_t C, int64_t L2, int64_t H,
                                                                   const T* __restrict__ dZ,
                                                                   const float* __restrict__ drow,
                                                                   const T* __restrict__ h, T* __restrict__ dh) {
  const int64_t C1 = C + 1;
  if ((int64_t)blockIdx.x < B) {
    const int64_t b = blockIdx.x;
    const T* ha = h + (b * C1) * H;
    for (int64_t n = threadIdx.x; n < H; n += blockDim.x) {
      const float a = ldf<T>(ha, n);
      float acc = 0.f;
      for (int64_t c = 0; c < C; ++c) {
        const float d = dz_at<T>(dZ, drow, b * C + c, H, n);
        acc += d * ldf<T>(h + (b * C1 + 1 + c) * H, n);
        stf(dh + (b * C1 + 1 + c) * H, n, d * a);
      }
      stf(dh + (b * C1) * H, n, acc);
    }
  } else {
    const int64_t i0 = ((int64_t)blockIdx.x - B) * 64;
    const int64_t i1 = min(L2, i0 + 64);
    const int64_t base = B * C1;
    for (int64_t i = i0; i < i1; ++i) {
      const T* hs = h + (base + i) * H;
      const T* hd = h + (base + L2 + i) * H;
      for (int64_t n = threadIdx.x; n < H; n += blockDim.x) {
        const float dv = dz_at<T>(dZ, drow, B * C + i, H, n);
        stf(dh + (base + i) * H, n, dv * ldf<T>(hd, n));
        stf(dh + (base + L2 + i) * H, n, dv * ldf<T>(hs, n));
      }
    }
  }
}

// 16-byte-chunk form of hadamard_bwd_blocks_kernel.  Anchor part: a block holds
// 256 / cpr anchors, thread = (anchor slot, chunk); label part: one thread per
// (pair, chunk).  f32 accumulation, one rounding per output element.
template <typename T>
struct Chunk {
  static constexpr int E = 16 / sizeof(T);
  float v[16 / sizeof(T)];
  __device__ __forceinline__ void load(const T* p) {
    const uint4 r = *reinterpret_cast<const uint4*>(p);
    if constexpr (sizeof(T) == 2) {
      const uint32_t u[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(u[i] << 16);
        v[2 * i + 1] = __uint_as_float(u[i] & 0xFFFF0000u);
      }
    } else {
      v[0] = __uint_as_float(r.x); v[1] = __uint_as_float(r.y); v[2] = __uint_as_float(r.z); v[3] = __uint_as_float(r.w);
    }
  }
  __device__ __forceinline__ void fill(float s) {
#pragma unroll
    for (int i = 0; i < E; ++i) v[i] = s;
  }
};
template <typename T>
__device__ __forceinline__ void store_chunk(T* p, const float* v) {
  uint4 o;
  if constexpr (sizeof(T) == 2) {
    o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
    o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
  } else {
    o = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
  }
  *reinterpret_cast<uint4*>(p) = o;
}

template <typename T>
__global__ __launch_bounds__(256) void hadamard_bwd_blocks_vec_kernel(int64_t B, int64_t C, int64_t L2, int64_t H,
                                                                       int64_t anchor_blocks,
                                                                       const T* __restrict__ dZ,
                                                                       const float* __restrict__ drow,
                                                                       const T* __restrict__ h,
                                                                       const int32_t* __restrict__ hidx,
                                                                       T* __restrict__ dh) {
  constexpr int E = 16 / sizeof(T);
  const int cpr = (int)(H / E);
  const int64_t C1 = C + 1;
  // h row of target-layout row r: r itself, or hidx[r] when h holds unique nodes only
  auto hrow = [&](int64_t r) -> int64_t { return hidx ? (int64_t)hidx[r] : r; };
  if ((int64_t)blockIdx.x < anchor_blocks) {
    const int apb = 256 / cpr;
    const int c = threadIdx.x % cpr, slot = threadIdx.x / cpr;
    const int64_t b = (int64_t)blockIdx.x * apb + slot;
    if (slot >= apb || b >= B) return;
    const int64_t col = (int64_t)c * E;
    Chunk<T> ha;
    ha.load(h + hrow(b * C1) * H + col);
    float acc[E];
#pragma unroll
    for (int i = 0; i < E; ++i) acc[i] = 0.f;
    for (int64_t cc = 0; cc < C; ++cc) {
      const int64_t r = b * C + cc;
      Chunk<T> d, hc;
      if (drow) d.fill(drow[r]); else d.load(dZ + r * H + col);
      hc.load(h + hrow(b * C1 + 1 + cc) * H + col);
      float o[E];
#pragma unroll
      for (int i = 0; i < E; ++i) {
        acc[i] = fmaf(d.v[i], hc.v[i], acc[i]);   // the order llp_hadamard_bwd_segments repeats
        o[i] = d.v[i] * ha.v[i];
      }
      store_chunk<T>(dh + (b * C1 + 1 + cc) * H + col, o);
    }
    store_chunk<T>(dh + (b * C1) * H + col, acc);
  } else {
    const int64_t t = ((int64_t)blockIdx.x - anchor_blocks) * 256 + threadIdx.x;
    if (t >= L2 * cpr) return;
    const int64_t i = t / cpr;
    const int64_t col = (t % cpr) * E;
    const int64_t base = B * C1;
    const int64_t r = B * C + i;
    Chunk<T> d, hs, hd;
    if (drow) d.fill(drow[r]); else d.load(dZ + r * H + col);
    hs.load(h + hrow(base + i) * H + col);
    hd.load(h + hrow(base + L2 + i) * H + col);
    float o1[E], o2[E];
#pragma unroll
    for (int k = 0; k < E; ++k) {
      o1[k] = d.v[k] * hd.v[k];
      o2[k] = d.v[k] * hs.v[k];
    }
    store_chunk<T>(dh + (base + i) * H + col, o1);
    store_chunk<T>(dh + (base + L2 + i) * H + col, o2);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void hadamard_bwd_scatter_kernel(int64_t R, int64_t H, const T* __restrict__ dZ,
                                                                    const float* __restrict__ drow,
                                                                    const int32_t* __restrict__ ia,
                                                                    const int32_t* __restrict__ ib,
                                                                    const T* __restrict__ h, float* __restrict__ dh) {
  const int64_t r = blockIdx.x;
  if (r >= R) return;
  const int64_t a = ia[r], bb = ib[r];
  for (int64_t n = threadIdx.x; n < H; n += blockDim.x) {
    const float d = dz_at<T>(dZ, drow, r, H, n);
    atomicAdd(dh + a * H + n, d * ldf<T>(h + bb * H, n));
    atomicAdd(dh + bb * H + n, d * ldf<T>(h + a * H, n));
  }
}

// out[r, :] = a[ia[r], :] * b[ib[r], :]  — 16-byte chunks, one per thread.
template <typename T>
__global__ __launch_bounds__(256) void hadamard_rows_kernel(int64_t R, int64_t H, const T* __restrict__ a,
                                                             const int32_t* __restrict__ ia, const T* __restrict__ b,
                                                             const int32_t* __restrict__ ib, T* __restrict__ out) {
  constexpr int E = 16 / sizeof(T);
  const int64_t cpr = H / E;
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= R * cpr) return;
  const int64_t r = t / cpr, c = t % cpr;
  const int64_t ra = ia ? (int64_t)ia[r] : r, rb = ib ? (int64_t)ib[r] : r;
  const uint4 x = *reinterpret_cast<const uint4*>(a + ra * H + c * E);
  const uint4 y = *reinterpret_cast<const uint4*>(b + rb * H + c * E);
  uint4 o;
  if constexpr (sizeof(T) == 2) {
    auto m2 = [](uint32_t p, uint32_t q) {
      return (uint32_t)f2bf(__uint_as_float(p << 16) * __uint_as_float(q << 16)) |
             ((uint32_t)f2bf(__uint_as_float(p & 0xFFFF0000u) * __uint_as_float(q & 0xFFFF0000u)) << 16);
    };
    o = make_uint4(m2(x.x, y.x), m2(x.y, y.y), m2(x.z, y.z), m2(x.w, y.w));
  } else {
    o = make_uint4(__float_as_uint(__uint_as_float(x.x) * __uint_as_float(y.x)),
                   __float_as_uint(__uint_as_float(x.y) * __uint_as_float(y.y)),
                   __float_as_uint(__uint_as_float(x.z) * __uint_as_float(y.z)),
                   __float_as_uint(__uint_as_float(x.w) * __uint_as_float(y.w)));
  }
  *reinterpret_cast<uint4*>(out + r * H + c * E) = o;
}

// Same products, G row groups per wave.  LPR = 64: a row is 64 * NCH 16-B chunks, lane
// l owns chunks l, l + 64, ..., and the row indices are wave-uniform (scalar loads, once
// per row instead of once per chunk); LPR = 32: a row is 32 chunks, each half-wave takes
// one row of the group.  The 2 * G * NCH operand loads of a lane issue together, and a
// block covers 4 * G * (64 / LPR) rows (301k blocks -> 38k at the collab shape).
template <typename T, int NCH, int G, int LPR>
__global__ __launch_bounds__(256) void hadamard_rows_wave_kernel(int64_t R, int64_t H, const T* __restrict__ a,
                                                                  const int32_t* __restrict__ ia,
                                                                  const T* __restrict__ b,
                                                                  const int32_t* __restrict__ ib, T* __restrict__ out) {
  constexpr int E = 16 / sizeof(T);
  constexpr int RPG = 64 / LPR;   // rows per group (one per LPR lanes)
  const int lane = threadIdx.x & 63;
  const int c = lane % LPR, sub = lane / LPR;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * G * RPG;
  if (r0 >= R) return;
  int64_t ra[G], rb[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int64_t rr = r0 + g * RPG + sub;
    const int64_t r = rr < R ? rr : R - 1;
    ra[g] = ia ? (int64_t)ia[r] : r;
    rb[g] = ib ? (int64_t)ib[r] : r;
  }
  uint4 x[G][NCH], y[G][NCH];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int64_t col = (int64_t)(c + LPR * j) * E;
      x[g][j] = *reinterpret_cast<const uint4*>(a + ra[g] * H + col);
      y[g][j] = *reinterpret_cast<const uint4*>(b + rb[g] * H + col);
    }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int64_t r = r0 + g * RPG + sub;
    if (r0 + g * RPG >= R) break;   // (wave-uniform)
    if (r >= R) continue;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      uint4 o;
      const uint4 p = x[g][j], q = y[g][j];
      if constexpr (sizeof(T) == 2) {
        auto m2 = [](uint32_t u, uint32_t v) {
          return (uint32_t)f2bf(__uint_as_float(u << 16) * __uint_as_float(v << 16)) |
                 ((uint32_t)f2bf(__uint_as_float(u & 0xFFFF0000u) * __uint_as_float(v & 0xFFFF0000u)) << 16);
        };
        o = make_uint4(m2(p.x, q.x), m2(p.y, q.y), m2(p.z, q.z), m2(p.w, q.w));
      } else {
        o = make_uint4(__float_as_uint(__uint_as_float(p.x) * __uint_as_float(q.x)),
                       __float_as_uint(__uint_as_float(p.y) * __uint_as_float(q.y)),
                       __float_as_uint(__uint_as_float(p.z) * __uint_as_float(q.z)),
                       __float_as_uint(__uint_as_float(p.w) * __uint_as_float(q.w)));
      }
      *reinterpret_cast<uint4*>(out + r * H + (int64_t)(c + LPR * j) * E) = o;
    }
  }
}

// ---------------------------------------------------------------- optimiser
constexpr int OPT_CHUNK = 4096;  // elements per block of the gradient norm (fixes its summation order)
#ifndef LLP_ADAM_CHUNK
#define LLP_ADAM_CHUNK 1024
#endif
constexpr int ADAM_CHUNK = LLP_ADAM_CHUNK;   // elements per block of Adam / the shadow refresh (one 4-wide pass)

// element e = (r, c) of a [rows, cols] parameter -> its slot in a shadow with
// leading dimension shadow_ld (0 = packed)
__device__ __forceinline__ int64_t shadow_index(const llp_tensor_desc& d, int64_t e) {
  if (d.shadow_ld == 0 || d.shadow_ld == d.cols) return e;
  return (e / d.cols) * d.shadow_ld + e % d.cols;
}

// Pointers read from the descriptor table are generic: hipcc then emits FLAT loads and stores,
// which count on lgkmcnt as well as vmcnt, so every LDS wait (the transposed shadow's tile) also
// waited for the tensor traffic in flight.  These casts to the global address space make them
// global_load / global_store (round 6: the physics optimizer's Adam).
typedef __attribute__((address_space(1))) float g_f32;
typedef __attribute__((address_space(1))) bf16_t g_bf16;
typedef __attribute__((address_space(1))) float4_t g_f4;
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) u32x2_t g_u2;
__device__ __forceinline__ g_f32* gbl(float* p) { return (g_f32*)p; }
__device__ __forceinline__ const g_f32* gbl(const float* p) { return (const g_f32*)p; }

__device__ __forceinline__ void put_elem(void* base, int64_t i, float v, int dt) {
  if (dt == LLP_BF16)
    ((g_bf16*)base)[i] = f2bf(v);
  else
    ((g_f32*)base)[i] = v;
}

// one thread's share of a chunk's sum of squares: its OPT_CHUNK / 256 loads issued together
// (a loop that waits on each is latency-bound: 18 us for the 2.3 M-parameter physics student),
// summed in element order (the order fixes the result; both norm kernels use this)
__device__ __forceinline__ float chunk_sumsq(const float* __restrict__ grad_, int64_t e0, int64_t e1) {
  constexpr int PER = OPT_CHUNK / 256;
  const g_f32* grad = gbl(grad_);
  float x[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int64_t e = e0 + threadIdx.x + 256 * k;
    x[k] = e < e1 ? grad[e] : 0.f;
  }
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k)
    if (e0 + threadIdx.x + 256 * k < e1) acc += x[k] * x[k];
  return acc;
}

__global__ __launch_bounds__(256) void grad_sumsq_kernel(const llp_tensor_desc* __restrict__ descs, int64_t max_chunks,
                                                         float* __restrict__ partial) {
  __shared__ float red[4];
  const llp_tensor_desc d = descs[blockIdx.y];
  const int64_t e0 = (int64_t)blockIdx.x * OPT_CHUNK;
  float acc = 0.f;
  if (e0 < d.numel) acc = chunk_sumsq(d.grad, e0, min(d.numel, e0 + OPT_CHUNK));
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.y * max_chunks + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// chunks of the gradient norm in tensor t
__device__ __forceinline__ uint32_t sumsq_chunks(const llp_tensor_desc* __restrict__ descs, int t) {
  return (uint32_t)((descs[t].numel + OPT_CHUNK - 1) / OPT_CHUNK);
}

// Compact grids (llp_grad_sumsq_w / llp_adam_step_w): workgroup w of a 1-D grid of n_work takes
// work item w of the tensors' items laid end to end (tensor 0's items first).  Wave-parallel
// prefix over the descriptors (one round trip per 64 tensors); every thread gets (t, blk, nblk).
// The 2-D grids (max chunks x tensors) left most workgroups idle past the small tensors' ends,
// and each idle one still paid a descriptor load: ~20k of them in the physics optimizer.
template <typename BlocksOf>
__device__ __forceinline__ void work_item(const llp_tensor_desc* __restrict__ descs, int n_tensors, uint32_t w,
                                          BlocksOf blocks_of, int& t_out, int64_t& blk, int64_t& nblk) {
  __shared__ int s_t;
  __shared__ uint32_t s_base, s_n;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    if (lane == 0) {   // no item matched (a host n_work past the table's items): t_out = -1
      s_t = -1;
      s_base = w;
      s_n = 0;
    }
    uint32_t base = 0;
    for (int t0 = 0; t0 < n_tensors; t0 += 64) {
      const int t = t0 + lane;
      const uint32_t nb = t < n_tensors ? blocks_of(descs[t]) : 0u;
      uint32_t inc = nb;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
      }
      const uint32_t lo = base + inc - nb;
      if (t < n_tensors && w >= lo && w < lo + nb) {
        s_t = t;
        s_base = lo;
        s_n = nb;
      }
      base += __shfl(inc, 63, 64);
    }
  }
  __syncthreads();
  t_out = s_t;
  blk = (int64_t)(w - s_base);
  nblk = (int64_t)s_n;
}

__device__ __forceinline__ uint32_t sumsq_blocks(const llp_tensor_desc& d) {
  return (uint32_t)((d.numel + OPT_CHUNK - 1) / OPT_CHUNK);
}

template <bool HANDOFF>
__device__ __forceinline__ void grad_sumsq_finalize_block(const llp_tensor_desc* __restrict__ descs, int n_tensors,
                                                          int64_t max_chunks, const float* partial, int n_groups,
                                                          float* __restrict__ sumsq) {
  // one block, one pass over every tensor's chunk partials at once (n_tensors <= 256): thread t
  // holds tensor t's chunk count, a block scan gives each tensor's first flat index, and thread i
  // sums (in double) the flat partials i, i+256, .. into its group's register, then a fixed LDS
  // tree per group (deterministic).  A loop over tensors waited one memory round trip each.
  __shared__ double red[8][256];
  __shared__ uint32_t pre[257];
  __shared__ int grp[256];
  __shared__ uint32_t wtot[4];
  const int tid = threadIdx.x, lane = tid & 63;
  uint32_t v = 0;
  if (tid < n_tensors) {
    v = sumsq_chunks(descs, tid);
    grp[tid] = descs[tid].group;
  }
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  if (lane == 63) wtot[tid >> 6] = v;
  __syncthreads();
  for (int w = 0; w < (tid >> 6); ++w) v += wtot[w];
  pre[tid + 1] = v;
  if (tid == 0) pre[0] = 0;
  __syncthreads();
  const uint32_t total = pre[n_tensors];
  double gs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t j0 = 0; j0 < total; j0 += 4 * 256) {
    float x[4];
    int gi[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t j = j0 + tid + 256 * u;
      x[u] = 0.f;
      gi[u] = -1;
      if (j < total) {
        int lo = 0, hi = n_tensors - 1;   // the last tensor whose first flat index is <= j
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (pre[mid] <= j) lo = mid; else hi = mid - 1;
        }
        const float* src = partial + lo * max_chunks + (j - pre[lo]);
        x[u] = HANDOFF ? llp_load_handed(src) : *src;
        gi[u] = grp[lo];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k == gi[u]) gs[k] += (double)x[u];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[k][tid] = gs[k];
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st)
#pragma unroll
      for (int k = 0; k < 8; ++k) red[k][tid] += red[k][tid + st];
    __syncthreads();
  }
  if (tid < n_groups) sumsq[tid] = (float)red[tid][0];
}

__global__ __launch_bounds__(256) void grad_sumsq_finalize(const llp_tensor_desc* __restrict__ descs, int n_tensors,
                                                           int64_t max_chunks, const float* __restrict__ partial,
                                                           int n_groups, float* __restrict__ sumsq) {
  grad_sumsq_finalize_block<false>(descs, n_tensors, max_chunks, partial, n_groups, sumsq);
}

// grad_sumsq_kernel with the finalize in the launch's last workgroup (ticket block: zero, left
// zero).  Only the workgroups that own a chunk arrive (the grid is max_chunks x n_tensors, most
// of it idle past the small tensors' ends): arrival index = the chunks of the tensors before
// this one + this chunk.
// n_work > 0: the compact 1-D grid of n_work workgroups (work_item), arrival index = blockIdx.x.
__global__ __launch_bounds__(256) void grad_sumsq_fused_kernel(const llp_tensor_desc* __restrict__ descs,
                                                               int n_tensors, int64_t max_chunks, float* partial,
                                                               int n_groups, float* __restrict__ sumsq,
                                                               uint32_t* ticket, int64_t n_work) {
  __shared__ float red[4];
  int t;
  int64_t blk, nblk_unused;
  uint32_t arrival, total;
  if (n_work > 0) {
    work_item(descs, n_tensors, blockIdx.x, [](const llp_tensor_desc& d) { return sumsq_blocks(d); }, t, blk,
              nblk_unused);
    arrival = blockIdx.x;
    total = (uint32_t)n_work;
    if (t < 0) {   // past the table's items: arrive with nothing (so the last arriver still finalizes)
      if (llp_arrive_last_tree(ticket, arrival, total))
        grad_sumsq_finalize_block<true>(descs, n_tensors, max_chunks, partial, n_groups, sumsq);
      return;
    }
  } else {
    t = blockIdx.y;
    blk = blockIdx.x;
    if (blk * OPT_CHUNK >= descs[t].numel) return;
    // this arrival's index and the number of arrivals: every wave reads the descriptors in
    // parallel (one round trip per 64 tensors) and sums them across its lanes
    uint32_t before = 0;
    total = 0;
    for (int t0 = 0; t0 < n_tensors; t0 += 64) {
      const int tt_ = t0 + (threadIdx.x & 63);
      const uint32_t nch = tt_ < n_tensors ? sumsq_chunks(descs, tt_) : 0u;
      uint32_t bb = tt_ < t ? nch : 0u, tt = nch;
      for (int o = 32; o > 0; o >>= 1) {
        bb += __shfl_xor(bb, o, 64);
        tt += __shfl_xor(tt, o, 64);
      }
      before += bb;
      total += tt;
    }
    arrival = before + (uint32_t)blk;
  }
  const llp_tensor_desc d = descs[t];
  const int64_t e0 = blk * OPT_CHUNK;
  float acc = chunk_sumsq(d.grad, e0, min(d.numel, e0 + OPT_CHUNK));
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) llp_store_handed(partial + t * max_chunks + blk, red[0] + red[1] + red[2] + red[3]);
  if (llp_arrive_last_tree(ticket, arrival, total))
    grad_sumsq_finalize_block<true>(descs, n_tensors, max_chunks, partial, n_groups, sumsq);
}

// Every contraction written out (fmaf), so the arithmetic does not depend on which kernel the
// compiler inlines it into (the one-launch and two-launch Adam agree bit for bit).
__device__ __forceinline__ float adam_elem(float g, float& m, float& v, float p, float beta1, float beta2, float eps,
                                           float bc2s, float step_size) {
  m = fmaf(beta1, m, (1.f - beta1) * g);
  v = fmaf(beta2, v, ((1.f - beta2) * g) * g);
  const float denom = sqrtf(v) / bc2s + eps;
  return fmaf(-step_size, m / denom, p);
}

// torch.optim.Adam (foreach=False semantics, see reference main.py:train_minibatch
// optimizer.step) after clip_grad_norm_.  Each block owns OPT_CHUNK elements of
// one tensor; 16-byte vector path when the tensor's buffers allow it.  The
// transposed shadow is written by shadow_t_kernel (LDS-tiled) afterwards.
__global__ __launch_bounds__(256) void adam_kernel(const llp_tensor_desc* __restrict__ descs,
                                                   const float* __restrict__ sumsq, float max_norm, float lr,
                                                   float beta1, float beta2, float eps,
                                                   const int64_t* __restrict__ step) {
  const llp_tensor_desc d = descs[blockIdx.y];
  const int64_t e0 = (int64_t)blockIdx.x * ADAM_CHUNK;
  if (e0 >= d.numel) return;
  const int64_t e1 = min(d.numel, e0 + ADAM_CHUNK);
  float coef = 1.f;
  if (sumsq) {
    const float total = sqrtf(sumsq[d.group]);
    // clip_grad_norm_: clamp(max_norm / (total + 1e-6), max=1); torch.clamp propagates a
    // NaN norm into every gradient (fminf would drop it and leave them unclipped)
    const float q = max_norm / (total + 1e-6f);
    coef = (q != q) ? q : fminf(q, 1.f);
  }
  const double t = (double)(*step + 1);
  const float bc1 = (float)(1.0 - pow((double)beta1, t));
  const float bc2s = (float)sqrt(1.0 - pow((double)beta2, t));
  const float step_size = lr / bc1;
  const bool vec = ((d.numel & 3) == 0) &&
                   ((((uintptr_t)d.grad) | ((uintptr_t)d.exp_avg) | ((uintptr_t)d.exp_avg_sq) | ((uintptr_t)d.param) |
                     (d.shadow ? (uintptr_t)d.shadow : 0)) & 15) == 0 &&
                   (d.shadow_ld == 0 || d.shadow_ld == d.cols);
  if (vec) {
    for (int64_t e = e0 + 4 * threadIdx.x; e < e1; e += 4 * blockDim.x) {
      float4 g = *reinterpret_cast<const float4*>(d.grad + e);
      if (coef != 1.f) {
        g.x *= coef; g.y *= coef; g.z *= coef; g.w *= coef;
        *reinterpret_cast<float4*>(d.grad + e) = g;   // clip_grad_norm_ scales .grad in place
      }
      float4 m = *reinterpret_cast<const float4*>(d.exp_avg + e);
      float4 v = *reinterpret_cast<const float4*>(d.exp_avg_sq + e);
      float4 p = *reinterpret_cast<const float4*>(d.param + e);
      p.x = adam_elem(g.x, m.x, v.x, p.x, beta1, beta2, eps, bc2s, step_size);
      p.y = adam_elem(g.y, m.y, v.y, p.y, beta1, beta2, eps, bc2s, step_size);
      p.z = adam_elem(g.z, m.z, v.z, p.z, beta1, beta2, eps, bc2s, step_size);
      p.w = adam_elem(g.w, m.w, v.w, p.w, beta1, beta2, eps, bc2s, step_size);
      *reinterpret_cast<float4*>(d.exp_avg + e) = m;
      *reinterpret_cast<float4*>(d.exp_avg_sq + e) = v;
      *reinterpret_cast<float4*>(d.param + e) = p;
      if (d.shadow) {
        if (d.shadow_dtype == LLP_BF16) {
          uint2 o;
          o.x = (uint32_t)f2bf(p.x) | ((uint32_t)f2bf(p.y) << 16);
          o.y = (uint32_t)f2bf(p.z) | ((uint32_t)f2bf(p.w) << 16);
          *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(d.shadow) + e) = o;
        } else {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(d.shadow) + e) = p;
        }
      }
    }
    return;
  }
  for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
    const float g = d.grad[e] * coef;
    if (coef != 1.f) d.grad[e] = g;
    float m = d.exp_avg[e], v = d.exp_avg_sq[e];
    const float pnew = adam_elem(g, m, v, d.param[e], beta1, beta2, eps, bc2s, step_size);
    d.exp_avg[e] = m;
    d.exp_avg_sq[e] = v;
    d.param[e] = pnew;
    if (d.shadow) put_elem(d.shadow, shadow_index(d, e), pnew, d.shadow_dtype);
  }
}

// shadow_t[c, r] = param[r, c] in the shadow dtype, 64x64 tiles through LDS so
// both the read and the write are row-coalesced.  Grid-strided over tiles.
__global__ __launch_bounds__(256) void shadow_t_kernel(const llp_tensor_desc* __restrict__ descs,
                                                       int64_t* __restrict__ step) {
  __shared__ float tile[64][65];
  // the Adam step counter advances here (after adam_kernel read it), saving a launch
  if (step && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *step += 1;
  const llp_tensor_desc d = descs[blockIdx.y];
  if (!d.shadow_t) return;
  const int64_t rows = d.rows, cols = d.cols;
  const int64_t ldt = d.shadow_t_ld ? d.shadow_t_ld : rows;
  const int64_t tr = (rows + 63) / 64, tc = (cols + 63) / 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int64_t tI = blockIdx.x; tI < tr * tc; tI += gridDim.x) {
    const int64_t r0 = (tI / tc) * 64, c0 = (tI % tc) * 64;
#pragma unroll 4
    for (int i = ty; i < 64; i += 4) {
      const int64_t r = r0 + i, c = c0 + tx;
      tile[i][tx] = (r < rows && c < cols) ? d.param[r * cols + c] : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int i = ty; i < 64; i += 4) {   // output row = column c0+i, output col = r0+tx
      const int64_t c = c0 + i, r = r0 + tx;
      if (c < cols && r < rows) put_elem(d.shadow_t, c * ldt + r, tile[tx][i], d.shadow_dtype);
    }
    __syncthreads();
  }
}

// adam_kernel and shadow_t_kernel in one launch.  A tensor with a transposed shadow is walked
// in 64 x 64 tiles on shadow_t_kernel's mapping (lane l of wave w: column c0 + l, rows w, w + 4,
// ..): every load and store of the Adam pass is lane-contiguous whatever the row width and
// alignment (the physics input weight is 8,415 wide), the row-major shadow is written from
// registers and the transposed one through the LDS tile.  Other tensors take adam_kernel's
// 1,024-element chunks.  Grid-strided over each tensor's tiles / chunks.  The Adam step counter
// is read, not advanced (llp_step_end2 follows).
__device__ __forceinline__ uint32_t adam_blocks(const llp_tensor_desc& d) {
  return d.shadow_t ? (uint32_t)(((d.rows + 63) / 64) * ((d.cols + 63) / 64))
                    : (uint32_t)((d.numel + ADAM_CHUNK - 1) / ADAM_CHUNK);
}

// n_work > 0: the compact 1-D grid (work_item), one tile / chunk per workgroup; otherwise the
// 2-D grid max chunks x tensors, grid-strided.
__global__ __launch_bounds__(256) void adam_fused_kernel(const llp_tensor_desc* __restrict__ descs,
                                                         const float* __restrict__ sumsq, float max_norm, float lr,
                                                         float beta1, float beta2, float eps,
                                                         const int64_t* __restrict__ step, int n_tensors,
                                                         int64_t n_work) {
  __shared__ float tile[64][65];
  int t;
  int64_t blk0, bstride;
  if (n_work > 0) {
    int64_t nblk;
    work_item(descs, n_tensors, blockIdx.x, [](const llp_tensor_desc& d) { return adam_blocks(d); }, t, blk0, nblk);
    if (t < 0) return;     // past the table's items (a stale host n_work): nothing to update
    bstride = nblk;        // one item: the grid-strided loops below run once
  } else {
    t = blockIdx.y;
    blk0 = blockIdx.x;
    bstride = gridDim.x;
  }
  const llp_tensor_desc d = descs[t];
  // most of the 2-D grid (max chunks x tensors) owns nothing: leave before the double pow below
  // (every thread of ~21k idle workgroups evaluating it cost ~40 us of the physics step)
  if (d.shadow_t ? blk0 >= ((d.rows + 63) / 64) * ((d.cols + 63) / 64) : blk0 * ADAM_CHUNK >= d.numel) return;
  float coef = 1.f;
  if (sumsq) {
    const float total = sqrtf(sumsq[d.group]);
    const float q = max_norm / (total + 1e-6f);
    coef = (q != q) ? q : fminf(q, 1.f);
  }
  const double tt = (double)(*step + 1);
  const float bc1 = (float)(1.0 - pow((double)beta1, tt));
  const float bc2s = (float)sqrt(1.0 - pow((double)beta2, tt));
  const float step_size = lr / bc1;
  if (d.shadow_t) {
    const int64_t rows = d.rows, cols = d.cols;
    const int64_t ldt = d.shadow_t_ld ? d.shadow_t_ld : rows;
    const int64_t lds = d.shadow_ld ? d.shadow_ld : cols;
    const int64_t tr = (rows + 63) / 64, tc = (cols + 63) / 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int64_t ti = blk0; ti < tr * tc; ti += bstride) {
      const int64_t r0 = (ti / tc) * 64, c0 = (ti % tc) * 64;
      const int64_t c = c0 + tx;
      // every load of the tile issued before the first store (the stores may alias later
      // loads as far as the compiler knows, which kept it to one row's round trip at a time)
      float gv[16], mv[16], vv[16], pv[16];
      g_f32* const gg = gbl(d.grad);
      g_f32* const gm = gbl(d.exp_avg);
      g_f32* const gvv = gbl(d.exp_avg_sq);
      g_f32* const gp = gbl(d.param);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int64_t r = r0 + ty + 4 * k, e = r * cols + c;
        const bool ok = r < rows && c < cols;
        gv[k] = ok ? gg[e] : 0.f;
        mv[k] = ok ? gm[e] : 0.f;
        vv[k] = ok ? gvv[e] : 0.f;
        pv[k] = ok ? gp[e] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int i = ty + 4 * k;
        const int64_t r = r0 + i;
        float pnew = 0.f;
        if (r < rows && c < cols) {
          const int64_t e = r * cols + c;
          const float g = gv[k] * coef;
          if (coef != 1.f) gg[e] = g;
          pnew = adam_elem(g, mv[k], vv[k], pv[k], beta1, beta2, eps, bc2s, step_size);
          gm[e] = mv[k];
          gvv[e] = vv[k];
          gp[e] = pnew;
          if (d.shadow) put_elem(d.shadow, r * lds + c, pnew, d.shadow_dtype);
        }
        tile[i][tx] = pnew;
      }
      __syncthreads();
#pragma unroll 4
      for (int i = ty; i < 64; i += 4) {   // output row = column c0 + i, output col = r0 + tx
        const int64_t oc = c0 + i, orow = r0 + tx;
        if (oc < cols && orow < rows) put_elem(d.shadow_t, oc * ldt + orow, tile[tx][i], d.shadow_dtype);
      }
      __syncthreads();
    }
  } else {
    const bool vec = ((d.numel & 3) == 0) &&
                     ((((uintptr_t)d.grad) | ((uintptr_t)d.exp_avg) | ((uintptr_t)d.exp_avg_sq) | ((uintptr_t)d.param) |
                       (d.shadow ? (uintptr_t)d.shadow : 0)) & 15) == 0 &&
                     (d.shadow_ld == 0 || d.shadow_ld == d.cols);
    for (int64_t e0 = blk0 * ADAM_CHUNK; e0 < d.numel; e0 += bstride * ADAM_CHUNK) {
      const int64_t e1 = min(d.numel, e0 + ADAM_CHUNK);
      g_f32* const gg = gbl(d.grad);
      g_f32* const gm = gbl(d.exp_avg);
      g_f32* const gvv = gbl(d.exp_avg_sq);
      g_f32* const gp = gbl(d.param);
      if (vec) {
        for (int64_t e = e0 + 4 * threadIdx.x; e < e1; e += 4 * blockDim.x) {
          const float4_t g4 = *(const g_f4*)(gg + e);
          float4 g = make_float4(g4.x, g4.y, g4.z, g4.w);
          if (coef != 1.f) {
            g.x *= coef; g.y *= coef; g.z *= coef; g.w *= coef;
            *(g_f4*)(gg + e) = float4_t{g.x, g.y, g.z, g.w};
          }
          const float4_t m4 = *(const g_f4*)(gm + e);
          const float4_t v4 = *(const g_f4*)(gvv + e);
          const float4_t p4 = *(const g_f4*)(gp + e);
          float4 m = make_float4(m4.x, m4.y, m4.z, m4.w);
          float4 v = make_float4(v4.x, v4.y, v4.z, v4.w);
          float4 p = make_float4(p4.x, p4.y, p4.z, p4.w);
          p.x = adam_elem(g.x, m.x, v.x, p.x, beta1, beta2, eps, bc2s, step_size);
          p.y = adam_elem(g.y, m.y, v.y, p.y, beta1, beta2, eps, bc2s, step_size);
          p.z = adam_elem(g.z, m.z, v.z, p.z, beta1, beta2, eps, bc2s, step_size);
          p.w = adam_elem(g.w, m.w, v.w, p.w, beta1, beta2, eps, bc2s, step_size);
          *(g_f4*)(gm + e) = float4_t{m.x, m.y, m.z, m.w};
          *(g_f4*)(gvv + e) = float4_t{v.x, v.y, v.z, v.w};
          *(g_f4*)(gp + e) = float4_t{p.x, p.y, p.z, p.w};
          if (d.shadow) {
            if (d.shadow_dtype == LLP_BF16) {
              u32x2_t o;
              o.x = (uint32_t)f2bf(p.x) | ((uint32_t)f2bf(p.y) << 16);
              o.y = (uint32_t)f2bf(p.z) | ((uint32_t)f2bf(p.w) << 16);
              *(g_u2*)((g_bf16*)d.shadow + e) = o;
            } else {
              *(g_f4*)((g_f32*)d.shadow + e) = float4_t{p.x, p.y, p.z, p.w};
            }
          }
        }
      } else {
        for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
          const float g = gg[e] * coef;
          if (coef != 1.f) gg[e] = g;
          float m = gm[e], v = gvv[e];
          const float pnew = adam_elem(g, m, v, gp[e], beta1, beta2, eps, bc2s, step_size);
          gm[e] = m;
          gvv[e] = v;
          gp[e] = pnew;
          if (d.shadow) put_elem(d.shadow, shadow_index(d, e), pnew, d.shadow_dtype);
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void shadow_kernel(const llp_tensor_desc* __restrict__ descs) {
  const llp_tensor_desc d = descs[blockIdx.y];
  const int64_t e0 = (int64_t)blockIdx.x * ADAM_CHUNK;
  if (e0 >= d.numel) return;
  const int64_t e1 = min(d.numel, e0 + ADAM_CHUNK);
  for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x)
    if (d.shadow) put_elem(d.shadow, shadow_index(d, e), d.param[e], d.shadow_dtype);
}

__global__ void increment_kernel(int64_t* ctr) { *ctr += 1; }

__global__ void convert_kernel(int src_bf16, int dst_bf16, int64_t n, const void* __restrict__ src,
                               void* __restrict__ dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = src_bf16 ? bf2f(reinterpret_cast<const bf16_t*>(src)[i]) : reinterpret_cast<const float*>(src)[i];
    if (dst_bf16)
      reinterpret_cast<bf16_t*>(dst)[i] = f2bf(v);
    else
      reinterpret_cast<float*>(dst)[i] = v;
  }
}

__global__ void accumulate_kernel(int64_t n, const float* __restrict__ src, float weight, double* __restrict__ dst,
                                  int64_t* __restrict__ ctr, int64_t* __restrict__ ctr2) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) dst[i] += (double)src[i] * (double)weight;
  if (ctr && i == 0) *ctr += 1;
  if (ctr2 && i == 0) *ctr2 += 1;
}

int64_t max_chunks_of(int64_t max_numel) { return (max_numel + OPT_CHUNK - 1) / OPT_CHUNK; }
int64_t adam_chunks_of(int64_t max_numel) { return (max_numel + ADAM_CHUNK - 1) / ADAM_CHUNK; }

}  // namespace

extern "C" int llp_hadamard_bwd_blocks(int dtype, int64_t B, int64_t C, int64_t L2, int64_t H, const void* dZ,
                                       const float* drow, const void* h, const int32_t* hidx, void* dh,
                                       void* stream) {
  LLP_CHECK_ARG((dZ || drow) && h && dh, "llp_hadamard_bwd_blocks: null pointer");
  const int64_t nblk = B + (L2 + 63) / 64;
  if (nblk == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  {
    const int es = dtype == LLP_BF16 ? 2 : 4;
    const int64_t cpr = H * es / 16;
    const bool vec = (H * es) % 16 == 0 && cpr <= 256 && (uintptr_t)h % 16 == 0 && (uintptr_t)dh % 16 == 0 &&
                     (!dZ || (uintptr_t)dZ % 16 == 0);
    LLP_CHECK_ARG(vec || !hidx, "llp_hadamard_bwd_blocks: hidx needs 16-B aligned rows");
    if (vec) {
      const int64_t apb = 256 / cpr;
      const int64_t ab = (B + apb - 1) / apb;
      const int64_t lb = (L2 * cpr + 255) / 256;
      if (ab + lb == 0) return LLP_OK;
      if (dtype == LLP_BF16)
        hipLaunchKernelGGL(hadamard_bwd_blocks_vec_kernel<bf16_t>, dim3((unsigned)(ab + lb)), dim3(256), 0, s, B, C,
                           L2, H, ab, (const bf16_t*)dZ, drow, (const bf16_t*)h, hidx, (bf16_t*)dh);
      else
        hipLaunchKernelGGL(hadamard_bwd_blocks_vec_kernel<float>, dim3((unsigned)(ab + lb)), dim3(256), 0, s, B, C,
                           L2, H, ab, (const float*)dZ, drow, (const float*)h, hidx, (float*)dh);
      LLP_LAUNCH_CHECK();
      return LLP_OK;
    }
  }
  if (dtype == LLP_BF16)
    hipLaunchKernelGGL(hadamard_bwd_blocks_kernel<bf16_t>, dim3((unsigned)nblk), dim3(256), 0, s, B, C, L2, H,
                       (const bf16_t*)dZ, drow, (const bf16_t*)h, (bf16_t*)dh);
  else
    hipLaunchKernelGGL(hadamard_bwd_blocks_kernel<float>, dim3((unsigned)nblk), dim3(256), 0, s, B, C, L2, H,
                       (const float*)dZ, drow, (const float*)h, (float*)dh);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_hadamard_rows(int dtype, int64_t R, int64_t H, const void* a, const int32_t* ia, const void* b,
                                 const int32_t* ib, void* out, void* stream) {
  LLP_CHECK_ARG(R == 0 || H == 0 || (a && b && out), "llp_hadamard_rows: null pointer");
  const int es = dtype == LLP_BF16 ? 2 : 4;
  LLP_CHECK_ARG((H * es) % 16 == 0 && (uintptr_t)a % 16 == 0 && (uintptr_t)b % 16 == 0 && (uintptr_t)out % 16 == 0,
                "llp_hadamard_rows: rows must be 16-byte multiples and aligned");
  const int64_t n = R * (H * es / 16);
  if (n == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  // rows of 32, 64, 128 or 256 chunks: row groups per wave, else one chunk per thread
  const int64_t cpr = H * es / 16;
  if ((cpr == 32 || cpr == 64 || cpr == 128 || cpr == 256)) {
    auto go = [&](auto kern, auto* pa, auto* pb, auto* po, int rows_per_wave) {
      hipLaunchKernelGGL(kern, dim3(ceil_div_u(R, 4 * rows_per_wave)), dim3(256), 0, s, R, H, pa, ia, pb, ib, po);
    };
    auto pick = [&](auto* pa, auto* pb, auto* po) {
      using TT = std::remove_const_t<std::remove_pointer_t<decltype(pa)>>;
      if (cpr == 32) go(hadamard_rows_wave_kernel<TT, 1, 4, 32>, pa, pb, po, 8);
      else if (cpr == 64) go(hadamard_rows_wave_kernel<TT, 1, 8, 64>, pa, pb, po, 8);
      else if (cpr == 128) go(hadamard_rows_wave_kernel<TT, 2, 4, 64>, pa, pb, po, 4);
      else go(hadamard_rows_wave_kernel<TT, 4, 2, 64>, pa, pb, po, 2);
    };
    if (dtype == LLP_BF16) pick((const bf16_t*)a, (const bf16_t*)b, (bf16_t*)out);
    else pick((const float*)a, (const float*)b, (float*)out);
    LLP_LAUNCH_CHECK();
    return LLP_OK;
  }
  if (dtype == LLP_BF16)
    hipLaunchKernelGGL(hadamard_rows_kernel<bf16_t>, dim3(ceil_div_u(n, 256)), dim3(256), 0, s, R, H,
                       (const bf16_t*)a, ia, (const bf16_t*)b, ib, (bf16_t*)out);
  else
    hipLaunchKernelGGL(hadamard_rows_kernel<float>, dim3(ceil_div_u(n, 256)), dim3(256), 0, s, R, H, (const float*)a,
                       ia, (const float*)b, ib, (float*)out);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_hadamard_bwd_scatter(int dtype, int64_t R, int64_t H, const void* dZ, const float* drow,
                                        const int32_t* ia, const int32_t* ib, const void* h, float* dh, void* stream) {
  LLP_CHECK_ARG((R == 0) || ((dZ || drow) && ia && ib && h && dh), "llp_hadamard_bwd_scatter: null pointer");
  if (R == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == LLP_BF16)
    hipLaunchKernelGGL(hadamard_bwd_scatter_kernel<bf16_t>, dim3((unsigned)R), dim3(256), 0, s, R, H,
                       (const bf16_t*)dZ, drow, ia, ib, (const bf16_t*)h, dh);
  else
    hipLaunchKernelGGL(hadamard_bwd_scatter_kernel<float>, dim3((unsigned)R), dim3(256), 0, s, R, H, (const float*)dZ,
                       drow, ia, ib, (const float*)h, dh);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

// The descriptor table is in device memory; the caller passes max_numel (the
// largest numel in the table) so the grid is sized without reading it back.
extern "C" int64_t llp_grad_sumsq_workspace_bytes(int n_tensors, int64_t max_numel) {
  return (int64_t)n_tensors * max_chunks_of(max_numel) * (int64_t)sizeof(float);
}

extern "C" int llp_grad_sumsq_t(const llp_tensor_desc* descs, int n_tensors, int64_t max_numel, int n_groups,
                                float* sumsq, uint32_t* ticket, void* workspace, int64_t workspace_bytes,
                                void* stream) {
  LLP_CHECK_ARG(descs && sumsq && workspace, "llp_grad_sumsq: null pointer");
  LLP_CHECK_ARG(n_groups >= 1 && n_groups <= 8, "llp_grad_sumsq: n_groups in [1,8]");
  LLP_CHECK_ARG(n_tensors >= 1 && n_tensors <= 256, "llp_grad_sumsq: n_tensors in [1,256]");
  LLP_CHECK_ARG(workspace_bytes >= llp_grad_sumsq_workspace_bytes(n_tensors, max_numel),
                "llp_grad_sumsq: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int64_t mc = max_chunks_of(max_numel);
  // blocks past a tensor's numel exit immediately; x extent bounded by kMaxNumel
  if (ticket) {   // one launch: the last workgroup finalizes
    hipLaunchKernelGGL(grad_sumsq_fused_kernel, dim3((unsigned)mc, (unsigned)n_tensors), dim3(256), 0, s, descs,
                       n_tensors, mc, (float*)workspace, n_groups, sumsq, ticket, (int64_t)0);
    LLP_LAUNCH_CHECK();
    return LLP_OK;
  }
  hipLaunchKernelGGL(grad_sumsq_kernel, dim3((unsigned)mc, (unsigned)n_tensors), dim3(256), 0, s, descs, mc,
                     (float*)workspace);
  LLP_LAUNCH_CHECK();
  hipLaunchKernelGGL(grad_sumsq_finalize, dim3(1), dim3(256), 0, s, descs, n_tensors, mc, (const float*)workspace,
                     n_groups, sumsq);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_grad_sumsq(const llp_tensor_desc* descs, int n_tensors, int64_t max_numel, int n_groups,
                              float* sumsq, void* workspace, int64_t workspace_bytes, void* stream) {
  return llp_grad_sumsq_t(descs, n_tensors, max_numel, n_groups, sumsq, nullptr, workspace, workspace_bytes, stream);
}

extern "C" int llp_adam_step_t(const llp_tensor_desc* descs, int n_tensors, int64_t max_numel, const float* sumsq,
                               float max_norm, float lr, float beta1, float beta2, float eps, const int64_t* step,
                               void* stream) {
  LLP_CHECK_ARG(descs && step, "llp_adam_step_t: null pointer");
  hipLaunchKernelGGL(adam_fused_kernel, dim3((unsigned)adam_chunks_of(max_numel), (unsigned)n_tensors), dim3(256), 0,
                     (hipStream_t)stream, descs, sumsq, max_norm, lr, beta1, beta2, eps, step, n_tensors, (int64_t)0);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

// The compact-grid forms: n_work = the number of work items (llp_adam_work_items /
// llp_grad_sumsq_work_items over the table's shapes, which the caller knows); the same
// arithmetic in the same order as llp_grad_sumsq_t / llp_adam_step_t (bit-identical).
extern "C" int64_t llp_grad_sumsq_work_items(int64_t numel) { return (numel + OPT_CHUNK - 1) / OPT_CHUNK; }
extern "C" int64_t llp_adam_work_items(int64_t numel, int64_t rows, int64_t cols, int transposed_shadow) {
  return transposed_shadow ? ((rows + 63) / 64) * ((cols + 63) / 64) : (numel + ADAM_CHUNK - 1) / ADAM_CHUNK;
}

extern "C" int llp_grad_sumsq_w(const llp_tensor_desc* descs, int n_tensors, int64_t max_numel, int64_t n_work,
                                int n_groups, float* sumsq, uint32_t* ticket, void* workspace,
                                int64_t workspace_bytes, void* stream) {
  LLP_CHECK_ARG(descs && sumsq && workspace && ticket, "llp_grad_sumsq_w: null pointer");
  LLP_CHECK_ARG(n_groups >= 1 && n_groups <= 8, "llp_grad_sumsq_w: n_groups in [1,8]");
  LLP_CHECK_ARG(n_tensors >= 1 && n_tensors <= 256 && n_work >= 1 && n_work < (1ll << 31),
                "llp_grad_sumsq_w: n_tensors in [1,256], n_work >= 1");
  LLP_CHECK_ARG(workspace_bytes >= llp_grad_sumsq_workspace_bytes(n_tensors, max_numel),
                "llp_grad_sumsq_w: workspace too small");
  const int64_t mc = max_chunks_of(max_numel);
#ifdef LLP_OPT_2D_GRID   // A/B build: the 2-D grid of llp_grad_sumsq_t
  return llp_grad_sumsq_t(descs, n_tensors, max_numel, n_groups, sumsq, ticket, workspace, workspace_bytes, stream);
#endif
  hipLaunchKernelGGL(grad_sumsq_fused_kernel, dim3((unsigned)n_work), dim3(256), 0, (hipStream_t)stream, descs,
                     n_tensors, mc, (float*)workspace, n_groups, sumsq, ticket, n_work);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_adam_step_w(const llp_tensor_desc* descs, int n_tensors, int64_t max_numel, int64_t n_work,
                               const float* sumsq,
                               float max_norm, float lr, float beta1, float beta2, float eps, const int64_t* step,
                               void* stream) {
  LLP_CHECK_ARG(descs && step, "llp_adam_step_w: null pointer");
  LLP_CHECK_ARG(n_tensors >= 1 && n_work >= 1 && n_work < (1ll << 31), "llp_adam_step_w: sizes");
#ifdef LLP_OPT_2D_GRID   // A/B build: the 2-D grid of llp_adam_step_t
  hipLaunchKernelGGL(adam_fused_kernel, dim3((unsigned)adam_chunks_of(max_numel), (unsigned)n_tensors), dim3(256), 0,
                     (hipStream_t)stream, descs, sumsq, max_norm, lr, beta1, beta2, eps, step, n_tensors, (int64_t)0);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
#endif
  hipLaunchKernelGGL(adam_fused_kernel, dim3((unsigned)n_work), dim3(256), 0, (hipStream_t)stream, descs, sumsq,
                     max_norm, lr, beta1, beta2, eps, step, n_tensors, n_work);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_adam_step(const llp_tensor_desc* descs, int n_tensors, int64_t max_numel, const float* sumsq,
                             float max_norm, float lr, float beta1, float beta2, float eps, int64_t* step,
                             void* stream) {
  LLP_CHECK_ARG(descs && step, "llp_adam_step: null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int64_t mc = max_chunks_of(max_numel);
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)adam_chunks_of(max_numel), (unsigned)n_tensors), dim3(256), 0, s, descs,
                     sumsq, max_norm, lr, beta1, beta2, eps, (const int64_t*)step);
  LLP_LAUNCH_CHECK();
  hipLaunchKernelGGL(shadow_t_kernel, dim3((unsigned)mc, (unsigned)n_tensors), dim3(256), 0, s, descs, step);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_refresh_shadows(const llp_tensor_desc* descs, int n_tensors, int64_t max_numel, void* stream) {
  LLP_CHECK_ARG(descs, "llp_refresh_shadows: null pointer");
  const int64_t mc = max_chunks_of(max_numel);
  hipLaunchKernelGGL(shadow_kernel, dim3((unsigned)adam_chunks_of(max_numel), (unsigned)n_tensors), dim3(256), 0,
                     (hipStream_t)stream, descs);
  LLP_LAUNCH_CHECK();
  hipLaunchKernelGGL(shadow_t_kernel, dim3((unsigned)mc, (unsigned)n_tensors), dim3(256), 0, (hipStream_t)stream,
                     descs, (int64_t*)nullptr);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_convert(int src_dtype, int dst_dtype, int64_t n, const void* src, void* dst, void* stream) {
  LLP_CHECK_ARG((n == 0) || (src && dst), "llp_convert: null pointer");
  if (n == 0) return LLP_OK;
  unsigned nb = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(convert_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, src_dtype == LLP_BF16,
                     dst_dtype == LLP_BF16, n, src, dst);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_accumulate(int64_t n, const float* src, float weight, double* dst, void* stream) {
  LLP_CHECK_ARG(src && dst, "llp_accumulate: null pointer");
  hipLaunchKernelGGL(accumulate_kernel, dim3(ceil_div_u(n, 256)), dim3(256), 0, (hipStream_t)stream, n, src, weight,
                     dst, (int64_t*)nullptr, (int64_t*)nullptr);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

// zero `bytes` bytes at p: 16-B stores over the aligned body, byte stores for the ends.
// A kernel, not hipMemsetAsync: a memset node in a captured hipGraph left half of its
// buffer unzeroed at replay on this ROCm (tools/memset_capture_probe.py).
__global__ void zero_bytes_kernel(uint8_t* __restrict__ p, int64_t head, int64_t n16, int64_t bytes) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n16) reinterpret_cast<uint4*>(p + head)[i] = make_uint4(0u, 0u, 0u, 0u);
  if (i < head) p[i] = 0;
  const int64_t t = head + n16 * 16 + i;
  if (i < 16 && t < bytes) p[t] = 0;
}

extern "C" int llp_zero(void* p, int64_t bytes, void* stream) {
  LLP_CHECK_ARG(p || bytes == 0, "llp_zero: null pointer");
  LLP_CHECK_ARG(bytes >= 0, "llp_zero: negative size");
  if (bytes == 0) return LLP_OK;
  const int64_t head = std::min<int64_t>(bytes, (16 - (int64_t)((uintptr_t)p % 16)) % 16);
  const int64_t n16 = (bytes - head) / 16;
  const int64_t threads = std::max<int64_t>(std::max<int64_t>(n16, 16), head);
  hipLaunchKernelGGL(zero_bytes_kernel, dim3(ceil_div_u(threads, 256)), dim3(256), 0, (hipStream_t)stream,
                     (uint8_t*)p, head, n16, bytes);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_step_end(const float* loss, float weight, double* loss_sum, int64_t* step_ctr, void* stream) {
  LLP_CHECK_ARG(loss && loss_sum && step_ctr, "llp_step_end: null pointer");
  hipLaunchKernelGGL(accumulate_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (int64_t)1, loss, weight, loss_sum,
                     step_ctr, (int64_t*)nullptr);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_step_end2(const float* loss, float weight, double* loss_sum, int64_t* step_ctr, int64_t* adam_step,
                             void* stream) {
  LLP_CHECK_ARG(loss && loss_sum && step_ctr && adam_step, "llp_step_end2: null pointer");
  hipLaunchKernelGGL(accumulate_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (int64_t)1, loss, weight, loss_sum,
                     step_ctr, adam_step);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_increment(int64_t* ctr, void* stream) {
  LLP_CHECK_ARG(ctr, "llp_increment: null pointer");
  hipLaunchKernelGGL(increment_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, ctr);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}
