// Unique-node compaction of the student's gathered rows (minibatch path).
//
// train_minibatch evaluates the student on data.x[this_target] (src/main.py:95-96):
// ~747k rows per collab step drawn from ~225k distinct nodes (anchors, walk
// contexts, random negatives and edge endpoints repeat).  Without dropout the
// MLP is a row-wise function, so duplicate rows produce bit-identical
// activations: the engine runs the student on the unique nodes and reduces
// each node's row gradients (a deterministic segmented sum over its rows, in
// row order) before the student backward.
#include "llp_common.h"


#include <type_traits>

namespace {

template <typename T>
struct V8;
template <>
struct V8<bf16_t> {
  static constexpr int E = 8;
  __device__ static void add(float* a, uint4 v) {
    const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[2 * i] += __uint_as_float(u[i] << 16);
      a[2 * i + 1] += __uint_as_float(u[i] & 0xFFFF0000u);
    }
  }
  __device__ static uint4 pack(const float* a) {
    uint32_t u[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] = (uint32_t)f2bf(a[2 * i]) | ((uint32_t)f2bf(a[2 * i + 1]) << 16);
    return make_uint4(u[0], u[1], u[2], u[3]);
  }
};
template <>
struct V8<float> {
  static constexpr int E = 4;
  __device__ static void add(float* a, uint4 v) {
    a[0] += __uint_as_float(v.x); a[1] += __uint_as_float(v.y);
    a[2] += __uint_as_float(v.z); a[3] += __uint_as_float(v.w);
  }
  __device__ static uint4 pack(const float* a) {
    return make_uint4(__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]), __float_as_uint(a[3]));
  }
};

// out[u] = sum over k in [seg_ptr[u], seg_ptr[u+1]) of src[rows[k]] (f32 accumulate,
// row order): one thread per 16-B column chunk, a block covers 256/cpr segments.
// TO: the output type (the input's, or f32: the sums unrounded, e.g. for a following
// cross-rank reduction).
template <typename T, typename TO>
__global__ __launch_bounds__(256) void segment_sum_kernel(int64_t U, int64_t H, const int32_t* __restrict__ seg_ptr,
                                                          const int32_t* __restrict__ rows,
                                                          const T* __restrict__ src, int64_t lds_,
                                                          TO* __restrict__ out, int64_t ldo,
                                                          const int32_t* __restrict__ out_rows,
                                                          const int32_t* __restrict__ u_dev) {
  constexpr int E = V8<T>::E;
  const int cpr = (int)(H / E);
  const int spb = 256 / cpr;
  const int c = threadIdx.x % cpr, slot = threadIdx.x / cpr;
  const int64_t u = (int64_t)blockIdx.x * spb + slot;
  if (u_dev && (int64_t)*u_dev < U) U = *u_dev;
  if (slot >= spb || u >= U) return;
  float acc[E];
#pragma unroll
  for (int i = 0; i < E; ++i) acc[i] = 0.f;
  const int beg = seg_ptr[u], end = seg_ptr[u + 1];
  int k = beg;
  for (; k + 1 < end; k += 2) {   // two rows in flight
    const uint4 v0 = *reinterpret_cast<const uint4*>(src + (int64_t)rows[k] * lds_ + c * E);
    const uint4 v1 = *reinterpret_cast<const uint4*>(src + (int64_t)rows[k + 1] * lds_ + c * E);
    V8<T>::add(acc, v0);
    V8<T>::add(acc, v1);
  }
  if (k < end) V8<T>::add(acc, *reinterpret_cast<const uint4*>(src + (int64_t)rows[k] * lds_ + c * E));
  const int64_t orow = out_rows ? (int64_t)out_rows[u] : u;
  if constexpr (std::is_same<T, TO>::value) {
    *reinterpret_cast<uint4*>(out + orow * ldo + c * E) = V8<T>::pack(acc);
  } else {
#pragma unroll
    for (int i = 0; i < E; i += 4)
      *reinterpret_cast<uint4*>(out + orow * ldo + c * E + i) = V8<float>::pack(acc + i);
  }
}

// Fused Hadamard backward + per-node reduction (the unique-node student path),
// bit-identical to llp_hadamard_bwd_blocks + llp_segment_sum_rows.  The predictor
// input of pair row z is h[a_z] * h[b_z]; its gradient dZ[z] reaches a_z as
// dZ[z] * h[b_z] and b_z as dZ[z] * h[a_z].  Target rows (the student's gathered
// layout, src/main.py:95) are [B anchors x (1 + C)] then [L2 sources | L2
// destinations]; pair rows are [B x C anchor-context] then [L2 links].
//   pass 1 (anchor rows): arow[b] = sum_cc dZ[b*C+cc] * h[pos[b*C1+1+cc]]  (f32 fma
//          chain in cc order, rounded once to the compute dtype)
//   pass 2 (per node u, its target rows in row order, f32 sum of each row's value
//          rounded to the compute dtype exactly as the row kernel stores it):
//          anchor row b*C1 -> arow[b]; context row b*C1+1+cc -> dZ[b*C+cc] * h[pos[b*C1]];
//          source row base+i -> dZ[B*C+i] * h[pos[base+L2+i]]; destination row
//          base+L2+i -> dZ[B*C+i] * h[pos[base+i]].
// Against the two-kernel path this drops the [R1, H] row-gradient buffer: its write
// and its read (2 x 1.5 GB at the collab shape) for a second read of the context
// pairs' dZ rows.  drow: the 'inner' predictor's per-pair scalar (dZ = NULL).
template <typename T>
__device__ __forceinline__ void unpack16(const uint4 r, float* v) {
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

template <typename T>
__device__ __forceinline__ void load16(const T* p, float* v) {
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

template <typename T>
__device__ __forceinline__ float round_to(float x) {
  if constexpr (sizeof(T) == 2) return __uint_as_float(((uint32_t)f2bf(x)) << 16);
  else return x;
}

// one 16-B input chunk's E sums into an output row of type TO (T: rounded once; f32: as summed)
template <typename T, typename TO>
__device__ __forceinline__ void store_sums(TO* p, const float* acc) {
  if constexpr (std::is_same<T, TO>::value) {
    *reinterpret_cast<uint4*>(p) = V8<T>::pack(acc);
  } else {
#pragma unroll
    for (int i = 0; i < V8<T>::E; i += 4) *reinterpret_cast<uint4*>(p + i) = V8<float>::pack(acc + i);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void hadamard_anchor_rows_kernel(int64_t B, int64_t C, int64_t H,
                                                                   const T* __restrict__ dZ,
                                                                   const float* __restrict__ drow,
                                                                   const T* __restrict__ h,
                                                                   const int32_t* __restrict__ pos,
                                                                   T* __restrict__ arow) {
  constexpr int E = V8<T>::E;
  const int cpr = (int)(H / E);
  const int apb = 256 / cpr;
  const int c = threadIdx.x % cpr, slot = threadIdx.x / cpr;
  const int64_t b = (int64_t)blockIdx.x * apb + slot;
  if (slot >= apb || b >= B) return;
  const int64_t col = (int64_t)c * E, C1 = C + 1;
  const int32_t* pc = pos + b * C1 + 1;
  float acc[E];
#pragma unroll
  for (int i = 0; i < E; ++i) acc[i] = 0.f;
#pragma unroll 4
  for (int64_t cc = 0; cc < C; ++cc) {
    const int64_t z = b * C + cc;
    float d[E], hc[E];
    if (drow) {
#pragma unroll
      for (int i = 0; i < E; ++i) d[i] = drow[z];
    } else {
      load16<T>(dZ + z * H + col, d);
    }
    load16<T>(h + (int64_t)pc[cc] * H + col, hc);
#pragma unroll
    for (int i = 0; i < E; ++i) acc[i] = fmaf(d[i], hc[i], acc[i]);
  }
  *reinterpret_cast<uint4*>(arow + b * H + col) = V8<T>::pack(acc);
}

// Same sums, one wave per anchor: lane l owns the 16-B chunks l, l + 64, ... (NCH of them,
// H / E = 64 * NCH).  The anchor is wave-uniform, so its C context slots are scalar loads,
// and the dZ and h[ctx] loads of G contexts issue together before their fmas, which run
// in context order per element (bit-identical to the kernel above).
template <typename T, int NCH, int G>
__global__ __launch_bounds__(256) void hadamard_anchor_rows_wave_kernel(int64_t B, int64_t C, int64_t H,
                                                                        const T* __restrict__ dZ,
                                                                        const float* __restrict__ drow,
                                                                        const T* __restrict__ h,
                                                                        const int32_t* __restrict__ pos,
                                                                        T* __restrict__ arow) {
  constexpr int E = V8<T>::E;
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (b >= B) return;
  const int32_t* pc = pos + b * (C + 1) + 1;
  float acc[NCH][E];
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int i = 0; i < E; ++i) acc[j][i] = 0.f;
  for (int64_t c0 = 0; c0 < C; c0 += G) {
    uint4 rd[G][NCH], rh[G][NCH];
    float s[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t cc = c0 + g < C ? c0 + g : C - 1;
      const int64_t z = b * C + cc;
      const T* ph = h + (int64_t)pc[cc] * H;
      s[g] = drow ? drow[z] : 0.f;
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        const int64_t col = (int64_t)(lane + 64 * j) * E;
        if (!drow) rd[g][j] = *reinterpret_cast<const uint4*>(dZ + z * H + col);
        rh[g][j] = *reinterpret_cast<const uint4*>(ph + col);
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (c0 + g >= C) break;   // (wave-uniform)
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        float d[E], hc[E];
        if (drow) {
#pragma unroll
          for (int i = 0; i < E; ++i) d[i] = s[g];
        } else {
          unpack16<T>(rd[g][j], d);
        }
        unpack16<T>(rh[g][j], hc);
#pragma unroll
        for (int i = 0; i < E; ++i) acc[j][i] = fmaf(d[i], hc[i], acc[j][i]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NCH; ++j)
    *reinterpret_cast<uint4*>(arow + b * H + (int64_t)(lane + 64 * j) * E) = V8<T>::pack(acc[j]);
}

template <typename T, typename TO>
__global__ __launch_bounds__(256) void hadamard_bwd_segments_kernel(
    int64_t U, int64_t B, int64_t C, int64_t L2, int64_t H, const int32_t* __restrict__ seg_ptr,
    const int32_t* __restrict__ rows, const int32_t* __restrict__ pos, const T* __restrict__ dZ,
    const float* __restrict__ drow, const T* __restrict__ h, const T* __restrict__ arow, TO* __restrict__ dh,
    int64_t ldo, const int32_t* __restrict__ out_rows, const int32_t* __restrict__ u_dev) {
  constexpr int E = V8<T>::E;
  const int cpr = (int)(H / E);
  const int spb = 256 / cpr;
  const int c = threadIdx.x % cpr, slot = threadIdx.x / cpr;
  const int64_t u = (int64_t)blockIdx.x * spb + slot;
  if (u_dev && (int64_t)*u_dev < U) U = *u_dev;
  if (slot >= spb || u >= U) return;
  const int64_t C1 = C + 1, base = B * C1, col = (int64_t)c * E;
  // row r -> (first operand row, h row of the partner, is-anchor); branch-free so the
  // loads of two rows issue together (the partner of an anchor row is unused: row 0)
  struct Src { const T* a; const T* hp; float s; bool anchor; };
  auto src_of = [&](int64_t r) -> Src {
    Src o;
    int64_t z, hr;
    bool anchor = false;
    if (r < base) {
      const int64_t b = r / C1, j = r - b * C1;
      anchor = j == 0;
      z = anchor ? b : b * C + j - 1;
      hr = anchor ? 0 : pos[b * C1];
    } else {
      const int64_t i = r - base;
      const bool src_side = i < L2;
      const int64_t li = src_side ? i : i - L2;
      z = B * C + li;
      hr = pos[src_side ? base + L2 + li : base + li];
    }
    o.anchor = anchor;
    o.a = anchor ? arow + z * H + col : (dZ ? dZ + z * H + col : h);
    o.s = (!anchor && drow) ? drow[z] : 0.f;
    o.hp = h + hr * H + col;
    return o;
  };
  auto value = [&](const Src& o, const float* va, const float* vh, float* out) {
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const float d = (drow && !o.anchor) ? o.s : va[i];
      out[i] = o.anchor ? va[i] : round_to<T>(d * vh[i]);
    }
  };
  float acc[E];
#pragma unroll
  for (int i = 0; i < E; ++i) acc[i] = 0.f;
  const int beg = seg_ptr[u], end = seg_ptr[u + 1];
  int k = beg;
  for (; k + 1 < end; k += 2) {   // two rows (four loads) in flight
    const Src o0 = src_of(rows[k]), o1 = src_of(rows[k + 1]);
    float a0[E], h0[E], a1[E], h1[E], v0[E], v1[E];
    load16<T>(o0.a, a0);
    load16<T>(o0.hp, h0);
    load16<T>(o1.a, a1);
    load16<T>(o1.hp, h1);
    value(o0, a0, h0, v0);
    value(o1, a1, h1, v1);
#pragma unroll
    for (int i = 0; i < E; ++i) acc[i] += v0[i];
#pragma unroll
    for (int i = 0; i < E; ++i) acc[i] += v1[i];
  }
  if (k < end) {
    const Src o0 = src_of(rows[k]);
    float a0[E], h0[E], v0[E];
    load16<T>(o0.a, a0);
    load16<T>(o0.hp, h0);
    value(o0, a0, h0, v0);
#pragma unroll
    for (int i = 0; i < E; ++i) acc[i] += v0[i];
  }
  store_sums<T, TO>(dh + (out_rows ? (int64_t)out_rows[u] : u) * ldo + col, acc);
}

// Same sums, NPW nodes per wave (LPN = 64 / NPW lanes per node; lane l of a node owns
// the 16-B chunks l, l + LPN, ..., NCH of them: H / E = LPN * NCH).  The kernel above
// walks a node's rows two at a time, each behind a chain of dependent loads (row id ->
// slot of the partner -> the two operand rows), so a node costs about three memory
// latencies per pair of rows and the launch is latency-bound (≈3.4 TB/s at the collab
// shape).  Here lane j of a node resolves row j of its segment (row id, pair row z,
// partner slot, anchor flag, inner scalar) in one parallel step, and the operand loads
// of G rows at a time are issued together from the broadcast descriptors; several
// nodes per wave keep more of those chains in flight.  Same values, same f32 additions
// in row order: bit-identical to the kernel above.
template <typename T, typename TO, int NCH, int G, int NPW>
__global__ __launch_bounds__(256) void hadamard_bwd_segments_wave_kernel(
    int64_t U, int64_t B, int64_t C, int64_t L2, int64_t H, const int32_t* __restrict__ seg_ptr,
    const int32_t* __restrict__ rows, const int32_t* __restrict__ pos, const T* __restrict__ dZ,
    const float* __restrict__ drow, const T* __restrict__ h, const T* __restrict__ arow, TO* __restrict__ dh,
    int64_t ldo, const int32_t* __restrict__ out_rows, const int32_t* __restrict__ u_dev) {
  constexpr int E = V8<T>::E;
  constexpr int LPN = 64 / NPW;
  const int lane = threadIdx.x & 63;
  const int nl = lane % LPN, nbase = lane - nl;   // lane within the node, first lane of the node
  const int64_t u = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * NPW + lane / LPN;
  if (u_dev && (int64_t)*u_dev < U) U = *u_dev;
  const bool live = u < U;
  const int64_t C1 = C + 1, base = B * C1;
  float acc[NCH][E];
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int i = 0; i < E; ++i) acc[j][i] = 0.f;
  const int beg = live ? seg_ptr[u] : 0, end = live ? seg_ptr[u + 1] : 0;
  // every node of the wave runs the same number of rounds (the shuffles need all lanes)
  int len = end - beg;
#pragma unroll
  for (int o = LPN; o < 64; o <<= 1) len = max(len, __shfl_xor(len, o, 64));
  for (int k0 = 0; k0 < len; k0 += LPN) {
    const int cnt = max(0, min(LPN, end - beg - k0));   // this node's rows in this round
    int64_t z = 0, hr = 0;
    int anch = 0;
    float sc = 0.f;
    if (nl < cnt) {   // lane nl: descriptor of the node's row beg + k0 + nl
      const int64_t r = rows[beg + k0 + nl];
      if (r < base) {
        const int64_t b = r / C1, jj = r - b * C1;
        anch = jj == 0;
        z = anch ? b : b * C + jj - 1;
        hr = anch ? 0 : pos[b * C1];
      } else {
        const int64_t i = r - base;
        const bool src_side = i < L2;
        const int64_t li = src_side ? i : i - L2;
        z = B * C + li;
        hr = pos[src_side ? base + L2 + li : base + li];
      }
      if (drow && !anch) sc = drow[z];
    }
    const int32_t zl = (int32_t)z, hl = (int32_t)hr;
    int cmax = cnt;
#pragma unroll
    for (int o = LPN; o < 64; o <<= 1) cmax = max(cmax, __shfl_xor(cmax, o, 64));
    for (int g0 = 0; g0 < cmax; g0 += G) {
      uint4 ra[G][NCH], rh[G][NCH];
      int an[G];
      float s[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int src = nbase + min(g0 + g, max(cnt - 1, 0));
        const int64_t zg = __shfl(zl, src, 64), hg = __shfl(hl, src, 64);
        an[g] = __shfl(anch, src, 64);
        s[g] = __shfl(sc, src, 64);
        const T* pa = an[g] ? arow + zg * H : (dZ ? dZ + zg * H : h);
        const T* ph = h + hg * H;
        if (g0 + g < cnt) {
#pragma unroll
          for (int j = 0; j < NCH; ++j) {
            const int64_t col = (int64_t)(nl + LPN * j) * E;
            ra[g][j] = *reinterpret_cast<const uint4*>(pa + col);
            rh[g][j] = *reinterpret_cast<const uint4*>(ph + col);
          }
        }
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        if (g0 + g < cnt) {
#pragma unroll
          for (int j = 0; j < NCH; ++j) {
            float va[E], vh[E];
            unpack16<T>(ra[g][j], va);
            unpack16<T>(rh[g][j], vh);
#pragma unroll
            for (int i = 0; i < E; ++i) {
              const float d = (drow && !an[g]) ? s[g] : va[i];
              acc[j][i] += an[g] ? va[i] : round_to<T>(d * vh[i]);
            }
          }
        }
      }
    }
  }
  if (!live) return;
  const int64_t orow = out_rows ? (int64_t)out_rows[u] : u;
#pragma unroll
  for (int j = 0; j < NCH; ++j) store_sums<T, TO>(dh + orow * ldo + (int64_t)(nl + LPN * j) * E, acc[j]);
}

// out row r = src row idx[r] for r < min(n, *count): 16-byte chunks, one thread each
__global__ void gather_rows16_kernel(int64_t n, int64_t chunks, const int32_t* __restrict__ idx,
                                     const uint4* __restrict__ src, int64_t ld_src16, uint4* __restrict__ out,
                                     int64_t ld_out16, const int32_t* __restrict__ count) {
  const int64_t live = count ? min(n, (int64_t)*count) : n;
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t r = t / chunks, c = t - r * chunks;
  if (r < live) out[r * ld_out16 + c] = src[(int64_t)idx[r] * ld_src16 + c];
}
__global__ void gather_rows1_kernel(int64_t n, int64_t bytes, const int32_t* __restrict__ idx,
                                    const uint8_t* __restrict__ src, int64_t ld_src, uint8_t* __restrict__ out,
                                    int64_t ld_out, const int32_t* __restrict__ count) {
  const int64_t live = count ? min(n, (int64_t)*count) : n;
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t r = t / bytes, c = t - r * bytes;
  if (r < live) out[r * ld_out + c] = src[(int64_t)idx[r] * ld_src + c];
}

__global__ void gather_i32_kernel(int64_t n, const int32_t* __restrict__ idx, const int32_t* __restrict__ src,
                                  int32_t* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) out[i] = src[idx[i]];
}

int64_t al256(int64_t b) { return (b + 255) & ~(int64_t)255; }

// ---------------------------------------------------------------- compaction
// Per-node row counts (integer atomics: exact) with each row's arrival rank, one
// exclusive scan of (present, count) packed in a u64 gives every node its slot and its
// segment start, rows are scattered to start + rank without atomics, then every segment
// is sorted by row id, which restores row order: the same outputs as a stable sort of
// the rows by node.
//
// Every pass is a kernel of this file (no hipMemsetAsync node, no rocprim): the whole
// compaction is plain kernel nodes under stream capture.  A hipMemsetAsync node in a
// thread-local segment capture made the multi-rank step's segmented hipGraph replay
// fault at the collab size in round 2; with the count zeroed by a kernel the replays are
// bit-identical to eager steps, with rocprim's scan or this file's.
// Segments are sorted one thread each up to SHORT_SEG rows, one wave each up to WAVE_SEG
// rows (spread over the whole grid, so hot nodes with neighbouring ids do not queue on
// one block: 389 -> 28 us on the skewed probe of tools/dedup_probe.py), one block each
// past that.
constexpr int SHORT_SEG = 32;   // segments up to this length sort in one thread's LDS row
constexpr int LONG_LDS = 4096;  // longer ones: one block each, ranks counted in LDS up to this length

__device__ __host__ __forceinline__ uint64_t pack_count(int32_t c) {
  return (c > 0 ? (1ull << 32) : 0ull) | (uint64_t)(uint32_t)c;
}

// count pass that also records each row's arrival rank within its node (returning
// atomic), so the scatter needs no atomics.  Collab R = 747k rows: 46 us.
__global__ void count_rank_kernel(int64_t R, const int32_t* __restrict__ target, int32_t* __restrict__ cnt,
                                  int32_t* __restrict__ rank) {
  const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (r < R) rank[r] = atomicAdd(&cnt[target[r]], 1);
}

__global__ void scatter_rank_kernel(int64_t R, const int32_t* __restrict__ target, const int32_t* __restrict__ uidx,
                                    const int32_t* __restrict__ start, const int32_t* __restrict__ rank,
                                    int32_t* __restrict__ pos, int32_t* __restrict__ seg_rows) {
  const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (r >= R) return;
  const int32_t v = target[r];
  pos[r] = uidx[v];
  seg_rows[start[v] + rank[r]] = (int32_t)r;
}

__global__ void zero_i32_kernel(int64_t n, int32_t* __restrict__ p) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0;
}

// Exclusive scan of pack_count(cnt[v]) over v < n in three launches: per-block sums,
// one block scanning the sums, per-block scans with their offsets.  u64 integer sums,
// so any association gives the same result.
constexpr int OS_T = 256, OS_I = 8, OS_B = OS_T * OS_I;   // 2,048 values per block

__global__ __launch_bounds__(OS_T) void os_block_sum_kernel(int64_t n, const int32_t* __restrict__ cnt,
                                                            uint64_t* __restrict__ bsum) {
  __shared__ uint64_t red[OS_T];
  const int64_t base = blockIdx.x * (int64_t)OS_B + threadIdx.x * OS_I;
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < OS_I; ++i) s += base + i < n ? pack_count(cnt[base + i]) : 0ull;
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = OS_T / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = red[0];
}

// one block: bsum[0..nb) -> exclusive prefix, 1,024 values per round with a carry
__global__ __launch_bounds__(1024) void os_scan_sums_kernel(int64_t nb, uint64_t* __restrict__ bsum) {
  __shared__ uint64_t buf[1024];
  const int t = threadIdx.x;
  uint64_t carry = 0;
  for (int64_t c0 = 0; c0 < nb; c0 += 1024) {
    const int64_t i = c0 + t;
    const uint64_t x = i < nb ? bsum[i] : 0ull;
    buf[t] = x;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const uint64_t y = t >= o ? buf[t - o] : 0ull;
      __syncthreads();
      buf[t] += y;
      __syncthreads();
    }
    if (i < nb) bsum[i] = carry + buf[t] - x;
    carry += buf[1023];
    __syncthreads();
  }
}

__global__ __launch_bounds__(OS_T) void os_block_scan_kernel(int64_t n, const int32_t* __restrict__ cnt,
                                                             const uint64_t* __restrict__ boff,
                                                             uint64_t* __restrict__ pre) {
  __shared__ uint64_t ts[OS_T];
  const int t = threadIdx.x;
  const int64_t base = blockIdx.x * (int64_t)OS_B + t * OS_I;
  uint64_t v[OS_I];
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < OS_I; ++i) {
    v[i] = base + i < n ? pack_count(cnt[base + i]) : 0ull;
    s += v[i];
  }
  ts[t] = s;
  __syncthreads();
  for (int o = 1; o < OS_T; o <<= 1) {
    const uint64_t y = t >= o ? ts[t - o] : 0ull;
    __syncthreads();
    ts[t] += y;
    __syncthreads();
  }
  uint64_t run = boff[blockIdx.x] + ts[t] - s;
#pragma unroll
  for (int i = 0; i < OS_I; ++i) {
    if (base + i < n) pre[base + i] = run;
    run += v[i];
  }
}

__global__ void compact_count_kernel(int64_t N, int64_t R, const int32_t* __restrict__ cnt,
                                     const uint64_t* __restrict__ pre, int32_t* __restrict__ uniq,
                                     int32_t* __restrict__ seg_ptr, int32_t* __restrict__ uidx,
                                     int32_t* __restrict__ cursor, int32_t* __restrict__ n_unique,
                                     int32_t* __restrict__ n_long) {
  const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (v >= N) return;
  const int32_t c = cnt[v];
  const uint64_t q = pre[v];
  const int32_t slot = (int32_t)(q >> 32), start = (int32_t)(q & 0xFFFFFFFFull);
  if (c > 0) {
    uniq[slot] = (int32_t)v;
    seg_ptr[slot] = start;
    uidx[v] = slot;
    cursor[v] = start;
  }
  if (v == N - 1) {
    const int32_t U = slot + (c > 0 ? 1 : 0);
    *n_unique = U;
    seg_ptr[U] = (int32_t)R;
    n_long[0] = 0;
    n_long[1] = 0;
  }
}


// rank-by-count of one long segment by a whole block: each row id's rank = the number
// of smaller ids in the segment (ids are distinct); read from LDS (`buf`, `cap` ints) or
// from a copy in `scratch` past that
__device__ __forceinline__ void rank_segment_block(int32_t* __restrict__ seg_rows, int32_t b, int32_t len,
                                                   int32_t* buf, int cap, int32_t* __restrict__ scratch) {
  const bool in_lds = len <= cap;
  const int32_t* src = in_lds ? buf : scratch + b;
  for (int32_t k = threadIdx.x; k < len; k += blockDim.x) {
    if (in_lds) buf[k] = seg_rows[b + k];
    else scratch[b + k] = seg_rows[b + k];
  }
  __syncthreads();
  for (int32_t k = threadIdx.x; k < len; k += blockDim.x) {
    const int32_t x = src[k];
    int32_t rank = 0;
    for (int32_t j = 0; j < len; ++j) rank += src[j] < x ? 1 : 0;
    seg_rows[b + rank] = x;
  }
  __syncthreads();
}

// one thread per segment: up to SHORT_SEG row ids sorted in registers by a bitonic
// network (the slots past the segment hold INT32_MAX and sort to the end), all loads in
// flight together; longer segments go on the global list for segsort_mid_wave_kernel.
// (An insertion sort in an LDS row per thread waited out the LDS latency on every step
// of the longest segment in its wave: 35 us on the physics step's 31k nodes.)
__global__ __launch_bounds__(256) void segsort_short_kernel(const int32_t* __restrict__ n_unique,
                                                            const int32_t* __restrict__ seg_ptr,
                                                            int32_t* __restrict__ seg_rows,
                                                            int32_t* __restrict__ long_list,
                                                            int32_t* __restrict__ n_long) {
  const int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (s >= *n_unique) return;
  const int32_t b = seg_ptr[s], len = seg_ptr[s + 1] - b;
  if (len <= 1) return;
  if (len > SHORT_SEG) {
    long_list[atomicAdd(n_long, 1)] = (int32_t)s;
    return;
  }
  int32_t v[SHORT_SEG];
#pragma unroll
  for (int i = 0; i < SHORT_SEG; ++i) v[i] = i < len ? seg_rows[b + i] : INT32_MAX;
#pragma unroll
  for (int k = 2; k <= SHORT_SEG; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
      for (int i = 0; i < SHORT_SEG; ++i) {
        const int l = i ^ j;
        if (l > i) {
          const int32_t lo = min(v[i], v[l]), hi = max(v[i], v[l]);
          if ((i & k) == 0) { v[i] = lo; v[l] = hi; } else { v[i] = hi; v[l] = lo; }
        }
      }
#pragma unroll
  for (int i = 0; i < SHORT_SEG; ++i)
    if (i < len) seg_rows[b + i] = v[i];
}

// the long segments ranked one WAVE per segment across the whole grid (up to WAVE_SEG
// rows, from the wave's own LDS row), so hot nodes with neighbouring ids do not queue on
// the few blocks that own those ids; longer segments go on to a second list for
// segsort_long_kernel.  Control flow is wave-uniform, so the LDS row needs only
// wave-scope ordering.
constexpr int WAVE_SEG = 1024;

__global__ __launch_bounds__(256) void segsort_mid_wave_kernel(const int32_t* __restrict__ n_long,
                                                               const int32_t* __restrict__ long_list,
                                                               const int32_t* __restrict__ seg_ptr,
                                                               int32_t* __restrict__ seg_rows,
                                                               int32_t* __restrict__ huge_list,
                                                               int32_t* __restrict__ n_huge) {
  __shared__ int32_t buf[4][WAVE_SEG];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int32_t* b = buf[w];
  const int32_t nl = *n_long;
  for (int64_t i = (int64_t)blockIdx.x * 4 + w; i < nl; i += (int64_t)gridDim.x * 4) {
    const int32_t sg = long_list[i];
    const int32_t beg = seg_ptr[sg], len = seg_ptr[sg + 1] - beg;
    if (len > WAVE_SEG) {
      if (lane == 0) huge_list[atomicAdd(n_huge, 1)] = sg;
      continue;
    }
    for (int k = lane; k < len; k += 64) b[k] = seg_rows[beg + k];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int k = lane; k < len; k += 64) {
      const int32_t x = b[k];
      int32_t rank = 0;
      for (int j = 0; j < len; ++j) rank += b[j] < x ? 1 : 0;
      seg_rows[beg + rank] = x;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // every lane's reads before the next fill
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// one block per huge segment (grid-strided over the list)
__global__ __launch_bounds__(256) void segsort_long_kernel(const int32_t* __restrict__ n_huge,
                                                           const int32_t* __restrict__ huge_list,
                                                           const int32_t* __restrict__ seg_ptr,
                                                           int32_t* __restrict__ seg_rows,
                                                           int32_t* __restrict__ scratch) {
  __shared__ int32_t buf[LONG_LDS];
  const int32_t nh = *n_huge;
  for (int32_t i = blockIdx.x; i < nh; i += gridDim.x) {
    const int32_t s = huge_list[i];
    const int32_t b = seg_ptr[s], len = seg_ptr[s + 1] - b;
    rank_segment_block(seg_rows, b, len, buf, LONG_LDS, scratch);
  }
}

// ---------------------------------------------------------------- the compaction in four launches
// (llp_dedup_rows2).  Same outputs as llp_dedup_rows; launches:
//   count_rank_kernel                      per-node counts and each row's arrival rank
//   dedup_scan_kernel                      ONE pass over the nodes: the exclusive scan of
//                                          pack_count by decoupled look-back between blocks, the
//                                          compaction (compact_count_kernel's writes), the counts
//                                          returned to zero, optionally zero rows for absent nodes
//   scatter_rank_kernel                    rows to their segment slots
//   segsort_all_kernel                     every segment sorted, short / mid / huge in one launch
// The count array, the look-back flags and the control words persist in the workspace between
// calls: zero at the first call (a zeroing launch when the caller does not vouch for it), left so
// by every call (counts reset by the scan, the ticket by its last workgroup, the flags tagged with a
// per-call epoch that the last workgroup advances).
// nodes per scan block LB_T * I: 512 up to 64k nodes (coauthor-physics' 31,044: 61 workgroups
// instead of 16), 2,048 above (collab's 235,868: 116; at 512 per block its look-back over 461
// workgroups cost 13.8 against 10.8 us, tools/dedup2_probe.py).  The workspace's look-back arrays
// are sized for the smaller blocks.
constexpr int LB_T = 256, LB_I_MIN = 2, LB_B_MIN = LB_T * LB_I_MIN;
constexpr int64_t LB_SMALL_N = 65536;
static int lb_items(int64_t num_nodes) { return num_nodes <= LB_SMALL_N ? 2 : 8; }
struct ScanArgs {
  int64_t N, R;
  int32_t* cnt;                 // [N] per-node counts (zeroed here after use)
  uint32_t* flags;              // [nb] (epoch << 2) | status
  unsigned long long* agg;      // [nb] block aggregates
  unsigned long long* incl;     // [nb] block inclusive prefixes
  uint32_t* ctl;                // [0] epoch of the last completed call, [1] ticket, [2] error
  int32_t* uniq; int32_t* seg_ptr; int32_t* uidx; int32_t* start;
  int32_t* n_unique; int32_t* n_long;
  char* zero_rows; int64_t zero_ld; int64_t zero_u4;   // optional: rows of absent nodes zeroed (16-B words)
};

template <int LB_I>
__global__ __launch_bounds__(LB_T) void dedup_scan_kernel(ScanArgs a) {
  constexpr int LB_B = LB_T * LB_I;
  __shared__ unsigned long long ts[LB_T];
  __shared__ int32_t absent[LB_B];   // this workgroup's absent nodes (local index), n_absent of them
  __shared__ int n_absent;
  const int t = threadIdx.x;
  const int64_t b = blockIdx.x;
  const uint32_t epoch = a.ctl[0] + 1u;   // read by every workgroup before its ticket add
  const int64_t base = b * (int64_t)LB_B + t * LB_I;
  int32_t c[LB_I];
  unsigned long long v[LB_I];
  unsigned long long s = 0;
#pragma unroll
  for (int i = 0; i < LB_I; ++i) {
    c[i] = base + i < a.N ? a.cnt[base + i] : 0;
    v[i] = pack_count(c[i]);
    s += v[i];
  }
  ts[t] = s;
  __syncthreads();
  for (int o = 1; o < LB_T; o <<= 1) {   // inclusive scan of the thread sums
    const unsigned long long y = t >= o ? ts[t - o] : 0ull;
    __syncthreads();
    ts[t] += y;
    __syncthreads();
  }
  const unsigned long long blk_sum = ts[LB_T - 1];
  if (t == 0) n_absent = 0;
  const unsigned long long excl = llp_lookback_u64(a.flags, a.agg, a.incl, b, blk_sum, epoch, &a.ctl[2]);
  // compaction (compact_count_kernel's writes), counts back to zero, absent nodes' rows zeroed
  unsigned long long run = excl + ts[t] - s;
#pragma unroll
  for (int i = 0; i < LB_I; ++i) {
    const int64_t node = base + i;
    if (node < a.N) {
      const int32_t slot = (int32_t)(run >> 32), st = (int32_t)(run & 0xFFFFFFFFull);
      if (c[i] > 0) {
        a.uniq[slot] = (int32_t)node;
        a.seg_ptr[slot] = st;
        a.uidx[node] = slot;
        a.start[node] = st;
        a.cnt[node] = 0;
      }
      if (node == a.N - 1) {
        const int32_t U = slot + (c[i] > 0 ? 1 : 0);
        *a.n_unique = U;
        a.seg_ptr[U] = (int32_t)a.R;
        a.n_long[0] = 0;
        a.n_long[1] = 0;
      }
    }
    run += v[i];
    if (a.zero_rows && node < a.N && c[i] == 0) absent[atomicAdd(&n_absent, 1)] = t * LB_I + i;
  }
  if (a.zero_rows) {   // absent nodes' rows (few): consecutive threads on consecutive 16-B words
    __syncthreads();
    const int32_t wpr = (int32_t)a.zero_u4, total = n_absent * wpr;
    for (int32_t q = t; q < total; q += LB_T) {
      const int32_t n = absent[q / wpr], wd = q % wpr;
      reinterpret_cast<uint4*>(a.zero_rows + (b * (int64_t)LB_B + n) * a.zero_ld)[wd] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  // the last workgroup advances the epoch (every workgroup read it above)
  if (llp_arrive_last(&a.ctl[1], gridDim.x) && t == 0)
    __hip_atomic_store(&a.ctl[0], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Every segment sorted by row id in one launch (segsort_short / mid_wave / long fused): thread t of
// block b takes slot t * gridDim + b (strided, so hot nodes with neighbouring ids land in different
// blocks); a segment of up to SHORT_SEG rows is sorted in the thread's registers, longer ones go
// on the block's LDS lists and are ranked by one wave each (up to WAVE_SEG rows) or by the whole
// block, as the three-launch form does.
constexpr int SS_T = 256;
__global__ __launch_bounds__(SS_T) void segsort_all_kernel(const int32_t* __restrict__ n_unique,
                                                           const int32_t* __restrict__ seg_ptr,
                                                           int32_t* __restrict__ seg_rows,
                                                           int32_t* __restrict__ scratch) {
  __shared__ int32_t wbuf[4][WAVE_SEG];
  __shared__ int32_t mid_list[SS_T], huge_list[SS_T];
  __shared__ int n_mid, n_huge;
  const int32_t U = *n_unique;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t per_round = (int64_t)gridDim.x * SS_T;
  for (int64_t r0 = 0; r0 < U; r0 += per_round) {
    if (threadIdx.x == 0) n_mid = n_huge = 0;
    __syncthreads();
    const int64_t s = r0 + (int64_t)threadIdx.x * gridDim.x + blockIdx.x;
    if (s < U) {
      const int32_t b = seg_ptr[s], len = seg_ptr[s + 1] - b;
      if (len > WAVE_SEG) {
        huge_list[atomicAdd(&n_huge, 1)] = (int32_t)s;
      } else if (len > SHORT_SEG) {
        mid_list[atomicAdd(&n_mid, 1)] = (int32_t)s;
      } else if (len > 1) {
        int32_t v[SHORT_SEG];
#pragma unroll
        for (int i = 0; i < SHORT_SEG; ++i) v[i] = i < len ? seg_rows[b + i] : INT32_MAX;
#pragma unroll
        for (int k = 2; k <= SHORT_SEG; k <<= 1)
#pragma unroll
          for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
            for (int i = 0; i < SHORT_SEG; ++i) {
              const int l = i ^ j;
              if (l > i) {
                const int32_t lo = min(v[i], v[l]), hi = max(v[i], v[l]);
                if ((i & k) == 0) { v[i] = lo; v[l] = hi; } else { v[i] = hi; v[l] = lo; }
              }
            }
#pragma unroll
        for (int i = 0; i < SHORT_SEG; ++i)
          if (i < len) seg_rows[b + i] = v[i];
      }
    }
    __syncthreads();
    const int nm = n_mid, nh = n_huge;
    for (int i = w; i < nm; i += 4) {   // a wave per mid segment, from its own LDS row
      const int32_t sg = mid_list[i];
      const int32_t beg = seg_ptr[sg], len = seg_ptr[sg + 1] - beg;
      int32_t* bw = wbuf[w];
      for (int k = lane; k < len; k += 64) bw[k] = seg_rows[beg + k];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int k = lane; k < len; k += 64) {
        const int32_t x = bw[k];
        int32_t rank = 0;
        for (int j = 0; j < len; ++j) rank += bw[j] < x ? 1 : 0;
        seg_rows[beg + rank] = x;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __syncthreads();
    for (int i = 0; i < nh; ++i) {   // the whole block per huge segment (LDS up to 4 x WAVE_SEG ids)
      const int32_t sg = huge_list[i];
      const int32_t beg = seg_ptr[sg], len = seg_ptr[sg + 1] - beg;
      rank_segment_block(seg_rows, beg, len, &wbuf[0][0], 4 * WAVE_SEG, scratch);
    }
    __syncthreads();
  }
}

__global__ void zero_u32_kernel(int64_t n, uint32_t* __restrict__ p) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0u;
}

}  // namespace

static int64_t counting_ws_bytes(int64_t num_nodes, int64_t R) {
  return 3 * al256((num_nodes + 1) * 4) + al256(num_nodes * 8) + 2 * al256(R * 4) + al256(256) +
         al256(((num_nodes + OS_B - 1) / OS_B) * 8) + 512;
}

extern "C" int64_t llp_dedup_rows_workspace_bytes(int64_t num_nodes, int64_t R) {
  return counting_ws_bytes(num_nodes, R);
}

extern "C" int llp_dedup_rows(int64_t num_nodes, int64_t R, const int32_t* target, int32_t* uniq, int32_t* pos,
                              int32_t* n_unique, int32_t* seg_ptr, int32_t* seg_rows, void* workspace,
                              int64_t workspace_bytes, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (R == 0) {   // an empty batch: no unique nodes, seg_ptr = {0} (zeroed by a kernel: no memset node)
    LLP_CHECK_ARG(n_unique && seg_ptr, "llp_dedup_rows: null");
    hipLaunchKernelGGL(zero_i32_kernel, dim3(1), dim3(256), 0, s, (int64_t)1, n_unique);
    hipLaunchKernelGGL(zero_i32_kernel, dim3(1), dim3(256), 0, s, (int64_t)1, seg_ptr);
    LLP_LAUNCH_CHECK();
    return LLP_OK;
  }
  LLP_CHECK_ARG(target && uniq && pos && n_unique && seg_ptr && seg_rows && workspace, "llp_dedup_rows: null");
  LLP_CHECK_ARG(num_nodes > 0 && num_nodes < (1ll << 31) && R > 0 && R < (1ll << 31), "llp_dedup_rows: sizes");
  LLP_CHECK_ARG(workspace_bytes >= llp_dedup_rows_workspace_bytes(num_nodes, R), "llp_dedup_rows: workspace");
  char* w = reinterpret_cast<char*>(workspace);
  int32_t* cnt = reinterpret_cast<int32_t*>(w);
  w += al256((num_nodes + 1) * 4);
  int32_t* uidx = reinterpret_cast<int32_t*>(w);
  w += al256((num_nodes + 1) * 4);
  int32_t* cursor = reinterpret_cast<int32_t*>(w);
  w += al256((num_nodes + 1) * 4);
  uint64_t* pre = reinterpret_cast<uint64_t*>(w);
  w += al256(num_nodes * 8);
  int32_t* long_list = reinterpret_cast<int32_t*>(w);
  w += al256(R * 4);
  int32_t* scratch = reinterpret_cast<int32_t*>(w);   // row ranks until the segment sort
  w += al256(R * 4);
  int32_t* n_long = reinterpret_cast<int32_t*>(w);    // [0] long segments, [1] huge ones (wave sort)
  w += al256(256);
  uint64_t* os_sums = reinterpret_cast<uint64_t*>(w);   // per-block sums / offsets of the scan

  hipLaunchKernelGGL(zero_i32_kernel, dim3(ceil_div_u(num_nodes, 256)), dim3(256), 0, s, num_nodes, cnt);
  hipLaunchKernelGGL(count_rank_kernel, dim3(ceil_div_u(R, 256)), dim3(256), 0, s, R, target, cnt, scratch);
  LLP_LAUNCH_CHECK();
  {
    const int64_t nb = (num_nodes + OS_B - 1) / OS_B;
    hipLaunchKernelGGL(os_block_sum_kernel, dim3((unsigned)nb), dim3(OS_T), 0, s, num_nodes, cnt, os_sums);
    hipLaunchKernelGGL(os_scan_sums_kernel, dim3(1), dim3(1024), 0, s, nb, os_sums);
    hipLaunchKernelGGL(os_block_scan_kernel, dim3((unsigned)nb), dim3(OS_T), 0, s, num_nodes, cnt, os_sums, pre);
    LLP_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(compact_count_kernel, dim3(ceil_div_u(num_nodes, 256)), dim3(256), 0, s, num_nodes, R, cnt, pre,
                     uniq, seg_ptr, uidx, cursor, n_unique, n_long);
  LLP_LAUNCH_CHECK();
  // cursor[v] = segment start of v (compact_count_kernel); scratch[r] = rank of row r
  hipLaunchKernelGGL(scatter_rank_kernel, dim3(ceil_div_u(R, 256)), dim3(256), 0, s, R, target, uidx, cursor, scratch,
                     pos, seg_rows);
  LLP_LAUNCH_CHECK();
  const int64_t ubound = R < num_nodes ? R : num_nodes;
  int32_t* huge_list = long_list + (R + 1) / 2;   // long segments are > 32 rows: fewer than R / 33 of them
  hipLaunchKernelGGL(segsort_short_kernel, dim3(ceil_div_u(ubound, 256)), dim3(256), 0, s, n_unique, seg_ptr,
                     seg_rows, long_list, n_long);
  hipLaunchKernelGGL(segsort_mid_wave_kernel, dim3(1024), dim3(256), 0, s, n_long, long_list, seg_ptr, seg_rows,
                     huge_list, n_long + 1);
  hipLaunchKernelGGL(segsort_long_kernel, dim3(256), dim3(256), 0, s, n_long + 1, huge_list, seg_ptr, seg_rows,
                     scratch);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

// workspace of llp_dedup_rows2: [state: counts | look-back flags | control words] then scratch
static int64_t dedup2_state_bytes(int64_t num_nodes) {
  const int64_t nb = (num_nodes + LB_B_MIN - 1) / LB_B_MIN;
  return al256((num_nodes + 1) * 4) + al256(nb * 4) + 256;
}

extern "C" int64_t llp_dedup_rows2_state_bytes(int64_t num_nodes) { return dedup2_state_bytes(num_nodes); }

extern "C" int64_t llp_dedup_rows2_workspace_bytes(int64_t num_nodes, int64_t R) {
  const int64_t nb = (num_nodes + LB_B_MIN - 1) / LB_B_MIN;   // look-back arrays: the most blocks
  return dedup2_state_bytes(num_nodes) + 2 * al256(nb * 8) + 2 * al256((num_nodes + 1) * 4) + 2 * al256(R * 4) + 512;
}

extern "C" int llp_dedup_rows2(int64_t num_nodes, int64_t R, const int32_t* target, int32_t* uniq, int32_t* pos,
                               int32_t* n_unique, int32_t* seg_ptr, int32_t* seg_rows, void* zero_rows,
                               int64_t zero_ld_bytes, int64_t zero_row_bytes, int state_clean, void* workspace,
                               int64_t workspace_bytes, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  LLP_CHECK_ARG(num_nodes > 0 && num_nodes < (1ll << 31) && R >= 0 && R < (1ll << 31), "llp_dedup_rows2: sizes");
  LLP_CHECK_ARG(workspace && workspace_bytes >= llp_dedup_rows2_workspace_bytes(num_nodes, R),
                "llp_dedup_rows2: workspace");
  LLP_CHECK_ARG(!zero_rows || (zero_row_bytes % 16 == 0 && zero_ld_bytes % 16 == 0 && ((uintptr_t)zero_rows & 15) == 0),
                "llp_dedup_rows2: zero_rows must be 16-B aligned rows of a multiple of 16 bytes");
  char* w = reinterpret_cast<char*>(workspace);
  const int64_t nb = (num_nodes + LB_B_MIN - 1) / LB_B_MIN;   // look-back arrays: the most blocks
  if (!state_clean) {   // first call on this workspace: the persistent state from zero
    const int64_t n32 = dedup2_state_bytes(num_nodes) / 4;
    hipLaunchKernelGGL(zero_u32_kernel, dim3(ceil_div_u(n32, 256)), dim3(256), 0, s, n32, (uint32_t*)w);
    LLP_LAUNCH_CHECK();
  }
  ScanArgs a = {};
  a.N = num_nodes; a.R = R;
  a.cnt = reinterpret_cast<int32_t*>(w);
  w += al256((num_nodes + 1) * 4);
  a.flags = reinterpret_cast<uint32_t*>(w);
  w += al256(nb * 4);
  a.ctl = reinterpret_cast<uint32_t*>(w);
  w += 256;
  a.agg = reinterpret_cast<unsigned long long*>(w);
  w += al256(nb * 8);
  a.incl = reinterpret_cast<unsigned long long*>(w);
  w += al256(nb * 8);
  a.uidx = reinterpret_cast<int32_t*>(w);
  w += al256((num_nodes + 1) * 4);
  a.start = reinterpret_cast<int32_t*>(w);
  w += al256((num_nodes + 1) * 4);
  int32_t* rank = reinterpret_cast<int32_t*>(w);   // row ranks, then the huge segments' scratch
  w += al256(R * 4);
  w += al256(R * 4);                                // (the long lists of the three-launch form: unused)
  a.n_long = reinterpret_cast<int32_t*>(w);
  a.uniq = uniq; a.seg_ptr = seg_ptr; a.n_unique = n_unique;
  a.zero_rows = reinterpret_cast<char*>(zero_rows);
  a.zero_ld = zero_ld_bytes;
  a.zero_u4 = zero_row_bytes / 16;
  if (R > 0) {
    LLP_CHECK_ARG(target && uniq && pos && n_unique && seg_ptr && seg_rows, "llp_dedup_rows2: null");
    hipLaunchKernelGGL(count_rank_kernel, dim3(ceil_div_u(R, 256)), dim3(256), 0, s, R, target, a.cnt, rank);
    LLP_LAUNCH_CHECK();
  }
  const int li = lb_items(num_nodes);
  const int64_t nbk = (num_nodes + LB_T * li - 1) / (LB_T * li);
  if (li == 2) hipLaunchKernelGGL(dedup_scan_kernel<2>, dim3((unsigned)nbk), dim3(LB_T), 0, s, a);
  else hipLaunchKernelGGL(dedup_scan_kernel<8>, dim3((unsigned)nbk), dim3(LB_T), 0, s, a);
  LLP_LAUNCH_CHECK();
  if (R == 0) return LLP_OK;
  hipLaunchKernelGGL(scatter_rank_kernel, dim3(ceil_div_u(R, 256)), dim3(256), 0, s, R, target, a.uidx, a.start,
                     rank, pos, seg_rows);
  LLP_LAUNCH_CHECK();
  const int64_t ubound = R < num_nodes ? R : num_nodes;
  const int64_t g = std::min<int64_t>((ubound + SS_T - 1) / SS_T, 4096);
  hipLaunchKernelGGL(segsort_all_kernel, dim3((unsigned)g), dim3(SS_T), 0, s, n_unique, seg_ptr, seg_rows, rank);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_segment_sum_rows(int dtype, int64_t U, int64_t H, const int32_t* seg_ptr, const int32_t* rows,
                                    const void* src, int64_t ld_src, void* out, int64_t ld_out, int out_dtype,
                                    const int32_t* out_rows, const int32_t* u_dev, void* stream) {
  LLP_CHECK_ARG((U == 0) || (seg_ptr && rows && src && out), "llp_segment_sum_rows: null");
  LLP_CHECK_ARG(out_dtype == dtype || out_dtype == LLP_F32, "llp_segment_sum_rows: out_dtype must be dtype or f32");
  const int E = dtype == LLP_BF16 ? 8 : 4;
  const int es = dtype == LLP_BF16 ? 2 : 4;
  const int eo = out_dtype == LLP_BF16 ? 2 : 4;
  LLP_CHECK_ARG(H % E == 0 && H / E <= 256 && (ld_src * es) % 16 == 0 && (ld_out * eo) % 16 == 0 &&
                    (uintptr_t)src % 16 == 0 && (uintptr_t)out % 16 == 0,
                "llp_segment_sum_rows: rows must be 16-B aligned, H <= 256 chunks");
  if (U == 0) return LLP_OK;
  const int64_t cpr = H / E, spb = 256 / cpr;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(ceil_div_u(U, spb));
  if (dtype == LLP_BF16 && out_dtype == LLP_BF16)
    hipLaunchKernelGGL((segment_sum_kernel<bf16_t, bf16_t>), grid, dim3(256), 0, s, U, H, seg_ptr, rows,
                       (const bf16_t*)src, ld_src, (bf16_t*)out, ld_out, out_rows, u_dev);
  else if (dtype == LLP_BF16)
    hipLaunchKernelGGL((segment_sum_kernel<bf16_t, float>), grid, dim3(256), 0, s, U, H, seg_ptr, rows,
                       (const bf16_t*)src, ld_src, (float*)out, ld_out, out_rows, u_dev);
  else
    hipLaunchKernelGGL((segment_sum_kernel<float, float>), grid, dim3(256), 0, s, U, H, seg_ptr, rows,
                       (const float*)src, ld_src, (float*)out, ld_out, out_rows, u_dev);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_gather_i32(int64_t n, const int32_t* idx, const int32_t* src, int32_t* out, void* stream) {
  LLP_CHECK_ARG((n == 0) || (idx && src && out), "llp_gather_i32: null");
  if (n == 0) return LLP_OK;
  hipLaunchKernelGGL(gather_i32_kernel, dim3(ceil_div_u(n, 256)), dim3(256), 0, (hipStream_t)stream, n, idx, src,
                     out);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_gather_rows(int64_t n, int64_t row_bytes, const int32_t* idx, const void* src,
                               int64_t ld_src_bytes, void* out, int64_t ld_out_bytes, const int32_t* count_dev,
                               void* stream) {
  LLP_CHECK_ARG(n >= 0 && row_bytes >= 0 && (n == 0 || (idx && src && out)), "llp_gather_rows: null / negative");
  LLP_CHECK_ARG(ld_src_bytes >= row_bytes && ld_out_bytes >= row_bytes, "llp_gather_rows: ld < row_bytes");
  if (n == 0 || row_bytes == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  const bool v16 = row_bytes % 16 == 0 && ld_src_bytes % 16 == 0 && ld_out_bytes % 16 == 0 &&
                   (uintptr_t)src % 16 == 0 && (uintptr_t)out % 16 == 0;
  if (v16) {
    const int64_t ch = row_bytes / 16;
    hipLaunchKernelGGL(gather_rows16_kernel, dim3(ceil_div_u(n * ch, 256)), dim3(256), 0, s, n, ch, idx,
                       (const uint4*)src, ld_src_bytes / 16, (uint4*)out, ld_out_bytes / 16, count_dev);
  } else {
    hipLaunchKernelGGL(gather_rows1_kernel, dim3(ceil_div_u(n * row_bytes, 256)), dim3(256), 0, s, n, row_bytes,
                       idx, (const uint8_t*)src, ld_src_bytes, (uint8_t*)out, ld_out_bytes, count_dev);
  }
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_hadamard_bwd_segments(int dtype, int64_t U, int64_t B, int64_t C, int64_t L2, int64_t H,
                                         const int32_t* seg_ptr, const int32_t* rows, const int32_t* pos,
                                         const void* dZ, const float* drow, const void* h, void* anchor_rows,
                                         void* dh, int64_t ld_dh, int out_dtype, const int32_t* out_rows,
                                         const int32_t* u_dev, void* stream) {
  LLP_CHECK_ARG(seg_ptr && rows && pos && h && dh && (dZ || drow) && (anchor_rows || B == 0),
                "llp_hadamard_bwd_segments: null");
  LLP_CHECK_ARG(out_dtype == dtype || out_dtype == LLP_F32, "llp_hadamard_bwd_segments: out_dtype must be dtype or f32");
  const int E = dtype == LLP_BF16 ? 8 : 4;
  const int es = out_dtype == LLP_BF16 ? 2 : 4;   // of the output rows
  LLP_CHECK_ARG(H % E == 0 && H / E <= 256 && (ld_dh * es) % 16 == 0 && (uintptr_t)h % 16 == 0 &&
                    (uintptr_t)dh % 16 == 0 && (!dZ || (uintptr_t)dZ % 16 == 0) &&
                    (uintptr_t)anchor_rows % 16 == 0,
                "llp_hadamard_bwd_segments: rows must be 16-B aligned, H <= 256 chunks");
  if (U == 0) return LLP_OK;
  const int64_t cpr = H / E, spb = 256 / cpr;
  hipStream_t s = (hipStream_t)stream;
  if (B > 0) {
    const int anch = (cpr % 64 == 0) ? (int)(cpr / 64) : 0;   // chunks per lane, one wave per anchor
#ifdef LLP_ANCHOR_THREADS   // A/B build: the thread-per-chunk kernel
    if (false) {
#else
    if (anch == 1 || anch == 2 || anch == 4) {
#endif
      auto go = [&](auto kern, auto* dz, auto* hh, auto* ar) {
        hipLaunchKernelGGL(kern, dim3(ceil_div_u(B, 4)), dim3(256), 0, s, B, C, H, dz, drow, hh, pos, ar);
      };
      auto pick = [&](auto* dz, auto* hh, auto* ar) {
        using TT = std::remove_const_t<std::remove_pointer_t<decltype(dz)>>;
        if (anch == 1) go(hadamard_anchor_rows_wave_kernel<TT, 1, 8>, dz, hh, ar);
        else if (anch == 2) go(hadamard_anchor_rows_wave_kernel<TT, 2, 4>, dz, hh, ar);
        else go(hadamard_anchor_rows_wave_kernel<TT, 4, 2>, dz, hh, ar);
      };
      if (dtype == LLP_BF16) pick((const bf16_t*)dZ, (const bf16_t*)h, (bf16_t*)anchor_rows);
      else pick((const float*)dZ, (const float*)h, (float*)anchor_rows);
    } else if (dtype == LLP_BF16) {
      hipLaunchKernelGGL(hadamard_anchor_rows_kernel<bf16_t>, dim3(ceil_div_u(B, spb)), dim3(256), 0, s, B, C, H,
                         (const bf16_t*)dZ, drow, (const bf16_t*)h, pos, (bf16_t*)anchor_rows);
    } else {
      hipLaunchKernelGGL(hadamard_anchor_rows_kernel<float>, dim3(ceil_div_u(B, spb)), dim3(256), 0, s, B, C, H,
                         (const float*)dZ, drow, (const float*)h, pos, (float*)anchor_rows);
    }
    LLP_LAUNCH_CHECK();
  }
  // one wave per node when a row is 64 * NCH 16-B chunks (1, 2, 4 or 8 per lane): 487 us at the
  // collab shape against 598 for the thread-group kernel below; two or four nodes per wave
  // measured 530 / 633 us (profiles/r02_seg_npw.txt)
  // rows of 32 or 16 chunks (H = 256 / 128 bf16, the physics student): two / four nodes per wave,
  // a 32- / 16-lane group each (the thread-group kernel below ran 117 us on the physics step)
  const int nch = (cpr % 64 == 0) ? (int)(cpr / 64) : 0;   // chunks per lane
  const int npw = cpr == 32 ? 2 : (cpr == 16 ? 4 : 1);     // nodes per wave for rows under 64 chunks
  if (nch == 1 || nch == 2 || nch == 4 || nch == 8 || npw > 1) {
    auto launch = [&](auto kern, auto* dz, auto* hh, auto* ar, auto* out) {
      hipLaunchKernelGGL(kern, dim3(ceil_div_u(U, 4 * npw)), dim3(256), 0, s, U, B, C, L2, H, seg_ptr, rows, pos, dz,
                         drow, hh, ar, out, ld_dh, out_rows, u_dev);
    };
    auto pick = [&](auto* dz, auto* hh, auto* ar, auto* out) {
      using TT = std::remove_const_t<std::remove_pointer_t<decltype(dz)>>;
      using TO = std::remove_pointer_t<decltype(out)>;
      if (npw == 2) launch(hadamard_bwd_segments_wave_kernel<TT, TO, 1, 8, 2>, dz, hh, ar, out);
      else if (npw == 4) launch(hadamard_bwd_segments_wave_kernel<TT, TO, 1, 8, 4>, dz, hh, ar, out);
      else if (nch == 1) launch(hadamard_bwd_segments_wave_kernel<TT, TO, 1, 8, 1>, dz, hh, ar, out);
      else if (nch == 2) launch(hadamard_bwd_segments_wave_kernel<TT, TO, 2, 4, 1>, dz, hh, ar, out);
      else if (nch == 4) launch(hadamard_bwd_segments_wave_kernel<TT, TO, 4, 2, 1>, dz, hh, ar, out);
      else launch(hadamard_bwd_segments_wave_kernel<TT, TO, 8, 1, 1>, dz, hh, ar, out);
    };
    if (dtype == LLP_BF16 && out_dtype == LLP_BF16)
      pick((const bf16_t*)dZ, (const bf16_t*)h, (const bf16_t*)anchor_rows, (bf16_t*)dh);
    else if (dtype == LLP_BF16)
      pick((const bf16_t*)dZ, (const bf16_t*)h, (const bf16_t*)anchor_rows, (float*)dh);
    else
      pick((const float*)dZ, (const float*)h, (const float*)anchor_rows, (float*)dh);
    LLP_LAUNCH_CHECK();
    return LLP_OK;
  }
  auto go = [&](auto* dz, auto* hh, auto* ar, auto* out) {
    using TT = std::remove_const_t<std::remove_pointer_t<decltype(dz)>>;
    using TO = std::remove_pointer_t<decltype(out)>;
    hipLaunchKernelGGL((hadamard_bwd_segments_kernel<TT, TO>), dim3(ceil_div_u(U, spb)), dim3(256), 0, s, U, B, C, L2,
                       H, seg_ptr, rows, pos, dz, drow, hh, ar, out, ld_dh, out_rows, u_dev);
  };
  if (dtype == LLP_BF16 && out_dtype == LLP_BF16)
    go((const bf16_t*)dZ, (const bf16_t*)h, (const bf16_t*)anchor_rows, (bf16_t*)dh);
  else if (dtype == LLP_BF16)
    go((const bf16_t*)dZ, (const bf16_t*)h, (const bf16_t*)anchor_rows, (float*)dh);
  else
    go((const float*)dZ, (const float*)h, (const float*)anchor_rows, (float*)dh);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}
