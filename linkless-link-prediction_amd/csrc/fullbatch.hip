// Full-batch distillation step helpers (reference ``train``, src/main.py:147-236):
//   * dense negative sampling on the device (a3; PyG 2.2.0 negative_sampling,
//     method='dense', called at src/main.py:206 and src/train_teacher_gnn.py:50),
//   * predictor-row index build for h[samples] / h[train_edges] (src/main.py:184-186,213),
//   * the KD_RM (cosine, src/main.py:24-25) and KD_LM (MSE, src/main.py:219) terms
//     with their gradients.
#include "llp_common.h"

namespace {

constexpr uint64_t kEmpty = ~0ull;

__device__ __forceinline__ bool in_sorted(const int64_t* __restrict__ keys, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    const int64_t k = keys[mid];
    if (k < v) lo = mid + 1; else hi = mid;
  }
  return lo < n && keys[lo] == v;
}

__device__ __forceinline__ uint32_t mix32(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return (uint32_t)k;
}

// the graph's edge keys in an open-addressing set (linear probing, kEmpty = free), built
// once per graph (llp_edge_table_build): a candidate's membership costs one or two probes
// instead of a binary search of ~18 dependent loads over the sorted keys
__device__ __forceinline__ bool in_table(const uint64_t* __restrict__ t, int64_t T, uint64_t v) {
  uint32_t h = mix32(v) & (uint32_t)(T - 1);
  while (true) {
    const uint64_t k = t[h];
    if (k == v) return true;
    if (k == kEmpty) return false;
    h = (h + 1) & (uint32_t)(T - 1);
  }
}

__global__ void edge_table_fill(uint64_t* __restrict__ t, int64_t T) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < T) t[i] = kEmpty;
}

__global__ void edge_table_insert(const int64_t* __restrict__ keys, int64_t n, uint64_t* __restrict__ t, int64_t T) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t c = (uint64_t)keys[i];
  uint32_t h = mix32(c) & (uint32_t)(T - 1);
  while (true) {
    const unsigned long long prev = atomicCAS((unsigned long long*)&t[h], (unsigned long long)kEmpty,
                                              (unsigned long long)c);
    if (prev == kEmpty || prev == c) return;
    h = (h + 1) & (uint32_t)(T - 1);
  }
}

__global__ void neg_table_init(uint64_t* __restrict__ tkeys, int32_t* __restrict__ tmin, int64_t T) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < T) {
    tkeys[i] = kEmpty;
    tmin[i] = 0x7fffffff;
  }
}

// Candidate i of the round stream: the population index itself (population <=
// sample_size: PyG enumerates range(population)) or a 64-bit Philox draw
// floor(u64 * population / 2^64).  Candidates that are existing edges are
// marked -1; the others are inserted in an open-addressing table keeping the
// smallest draw index per value (first occurrence = sampling without replacement).
__global__ void neg_candidates(int64_t M, int enumerate_all, uint64_t population, uint64_t seed,
                               const int64_t* __restrict__ step_ctr, int64_t stream_offset,
                               const int64_t* __restrict__ edge_keys, int64_t n_keys,
                               const uint64_t* __restrict__ edge_table, int64_t edge_table_size,
                               int64_t* __restrict__ cand,
                               int32_t* __restrict__ slot, uint64_t* __restrict__ tkeys, int32_t* __restrict__ tmin,
                               int64_t T) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= M) return;
  uint64_t c;
  if (enumerate_all) {
    c = (uint64_t)(i % (int64_t)population);
  } else {
    const uint64_t stream = (uint64_t)(LLP_STREAMS_PER_STEP * (*step_ctr) + stream_offset);
    const uint64_t lo = philox_u32(seed, stream, 2 * (uint64_t)i);
    const uint64_t hi = philox_u32(seed, stream, 2 * (uint64_t)i + 1);
    c = __umul64hi((hi << 32) | lo, population);
  }
  cand[i] = (int64_t)c;
  if (edge_table ? in_table(edge_table, edge_table_size, c) : in_sorted(edge_keys, n_keys, (int64_t)c)) {
    slot[i] = -1;
    return;
  }
  uint32_t h = mix32(c) & (uint32_t)(T - 1);
  while (true) {
    const unsigned long long prev = atomicCAS((unsigned long long*)&tkeys[h], (unsigned long long)kEmpty,
                                              (unsigned long long)c);
    if (prev == kEmpty || prev == c) {
      atomicMin(&tmin[h], (int32_t)i);
      slot[i] = (int32_t)h;
      return;
    }
    h = (h + 1) & (uint32_t)(T - 1);
  }
}

// Ordered compaction of the valid candidates: the first num_neg of them in
// stream order, decoded as PyG does: row = idx / (N-1), col = idx % (N-1),
// col += (row <= col).  Three passes over tiles of 1024 candidates (256
// threads x 4): per-tile valid counts, one-block exclusive scan of the tile
// counts (and the final count), per-tile scan + scatter.
constexpr int NC_TILE = 1024;

__device__ __forceinline__ int neg_valid(int64_t i, int64_t M, const int32_t* __restrict__ slot,
                                         const int32_t* __restrict__ tmin) {
  if (i >= M) return 0;
  const int32_t s = slot[i];
  return (s >= 0 && tmin[s] == (int32_t)i) ? 1 : 0;
}

// block-wide exclusive scan of one int per thread (256 threads); returns the exclusive
// prefix, *total = block sum
__device__ __forceinline__ int block_excl_scan256(int v, int* wsum, int* total) {
  const int tid = threadIdx.x;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    if ((tid & 63) >= o) incl += y;
  }
  if ((tid & 63) == 63) wsum[tid >> 6] = incl;
  __syncthreads();
  int wbase = 0;
  for (int w = 0; w < (tid >> 6); ++w) wbase += wsum[w];
  *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  return wbase + incl - v;
}

__global__ __launch_bounds__(256) void neg_tile_count(int64_t M, const int32_t* __restrict__ slot,
                                                      const int32_t* __restrict__ tmin, int32_t* __restrict__ tcount) {
  __shared__ int wsum[4];
  const int64_t i0 = (int64_t)blockIdx.x * NC_TILE + 4 * threadIdx.x;
  int v = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) v += neg_valid(i0 + k, M, slot, tmin);
  int total;
  block_excl_scan256(v, wsum, &total);
  if (threadIdx.x == 0) tcount[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void neg_tile_scan(int64_t ntiles, int64_t num_neg, int32_t* __restrict__ tbase,
                                                     int32_t* __restrict__ count) {
  __shared__ int wsum[4];
  int64_t carry = 0;
  for (int64_t t0 = 0; t0 < ntiles; t0 += 256) {
    const int64_t t = t0 + threadIdx.x;
    const int v = t < ntiles ? tbase[t] : 0;       // tile counts in, tile bases out (in place)
    int total;
    const int ex = block_excl_scan256(v, wsum, &total);
    __syncthreads();
    if (t < ntiles) tbase[t] = (int32_t)min(carry + ex, (int64_t)0x7FFFFFFF);
    carry += total;
    __syncthreads();
  }
  if (threadIdx.x == 0) *count = (int32_t)min(carry, num_neg);
}

__global__ __launch_bounds__(256) void neg_tile_scatter(int64_t M, int64_t num_nodes, int64_t num_neg,
                                                        const int64_t* __restrict__ cand,
                                                        const int32_t* __restrict__ slot,
                                                        const int32_t* __restrict__ tmin,
                                                        const int32_t* __restrict__ tbase, int32_t* __restrict__ out,
                                                        int64_t ld_out) {
  __shared__ int wsum[4];
  const int64_t base = tbase[blockIdx.x];
  if (base >= num_neg) return;                      // uniform per block
  const int64_t i0 = (int64_t)blockIdx.x * NC_TILE + 4 * threadIdx.x;
  int v[4], mine = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = neg_valid(i0 + k, M, slot, tmin);
    mine += v[k];
  }
  int total;
  int64_t pos = base + block_excl_scan256(mine, wsum, &total);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (v[k]) {
      if (pos < num_neg) {
        const int64_t c = cand[i0 + k];
        const int64_t r = c / (num_nodes - 1);
        int64_t cc = c % (num_nodes - 1);
        if (r <= cc) cc += 1;
        out[pos] = (int32_t)r;
        out[ld_out + pos] = (int32_t)cc;
      }
      ++pos;
    }
  }
}

// ---------------------------------------------------------------- dense negatives in two launches
// (llp_neg_sample_dense2; the same outputs as llp_neg_sample_dense): the candidates' table and the
// tile scan's look-back flags persist in the workspace with a per-call epoch instead of being
// reset every call (neg_table_init), and the tile count / scan / scatter run as ONE pass with a
// decoupled look-back.  Table entry = (epoch & 0xFFFFFF) << 40 | the index of the FIRST candidate
// holding the slot's value (indices < 2^31); the value itself is read from cand[], which each
// candidate stores write-through before its claim can be seen.  An entry of another epoch is free.
// One atomic per candidate (the claim); a repeated value takes an atomicMin on the entry, so the
// lowest index keeps it -- the first occurrence, as torch.unique-then-first does (the two-word
// form took a second atomic, the first-index atomicMax, for every candidate).
constexpr int64_t NEG2_VALUE_BITS = 40;
constexpr uint64_t NEG2_VALUE_MASK = (1ull << NEG2_VALUE_BITS) - 1;

// Candidates [i_lo, i_hi).  gate (may be NULL): the whole launch does nothing when *gate >= num_neg
// (the first round's candidates already hold enough negatives; llp_neg_sample_dense2 below).
__global__ void neg_candidates2(int64_t i_lo, int64_t i_hi, int enumerate_all, uint64_t population, uint64_t seed,
                                const int64_t* __restrict__ step_ctr, int64_t stream_offset,
                                const int64_t* __restrict__ edge_keys, int64_t n_keys,
                                const uint64_t* __restrict__ edge_table, int64_t edge_table_size,
                                int64_t* cand, int32_t* __restrict__ slot, uint64_t* __restrict__ tkeys, int64_t T,
                                const uint32_t* __restrict__ ctl, const int32_t* __restrict__ gate, int64_t num_neg) {
  if (gate && (int64_t)*gate >= num_neg) return;
  const int64_t i = i_lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= i_hi) return;
  const uint32_t epoch = ctl[0] + 1u;
  const uint64_t tag = (uint64_t)(epoch & 0xFFFFFFu) << NEG2_VALUE_BITS;
  uint64_t c;
  if (enumerate_all) {
    c = (uint64_t)(i % (int64_t)population);
  } else {
    // draws 2i and 2i + 1 are components of one Philox block (philox_u32: word idx & 3 of block
    // idx >> 2), so one philox4 gives both
    const uint64_t stream = (uint64_t)(LLP_STREAMS_PER_STEP * (*step_ctr) + stream_offset);
    const uint4 x4 = philox4((uint64_t)i >> 1, stream, seed);
    const uint64_t lo = (i & 1) ? x4.z : x4.x;
    const uint64_t hi = (i & 1) ? x4.w : x4.y;
    c = __umul64hi((hi << 32) | lo, population);
  }
  // write-through, drained before the claim below publishes this index
  __hip_atomic_store((unsigned long long*)&cand[i], (unsigned long long)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (edge_table ? in_table(edge_table, edge_table_size, c) : in_sorted(edge_keys, n_keys, (int64_t)c)) {
    slot[i] = -1;
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long mine = tag | (unsigned long long)i;
  uint32_t h = mix32(c) & (uint32_t)(T - 1);
  while (true) {
    unsigned long long e = __hip_atomic_load((unsigned long long*)&tkeys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((e & ~NEG2_VALUE_MASK) != tag) {   // free in this epoch: claim it
      const unsigned long long prev = atomicCAS((unsigned long long*)&tkeys[h], e, mine);
      if (prev == e) break;
      continue;                            // taken meanwhile: look at the same slot again
    }
    const unsigned long long cj = __hip_atomic_load((unsigned long long*)&cand[e & NEG2_VALUE_MASK], __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
    if (cj == c) {                         // the same value: the lower index keeps the slot
      atomicMin((unsigned long long*)&tkeys[h], mine);
      break;
    }
    h = (h + 1) & (uint32_t)(T - 1);
  }
  slot[i] = (int32_t)h;
}

// Tiles [tile_lo, tile_lo + gridDim.x) of the candidates [0, M); the look-back runs over the
// global tile index, so a second launch continues the first one's prefix (same epoch: only the
// launch with ``advance`` moves the epoch on).  gate as neg_candidates2 (the launch then only
// arrives on its ticket and, with ``advance``, moves the epoch on).
__global__ __launch_bounds__(256) void neg_compact2(int64_t M, int64_t num_nodes, int64_t num_neg,
                                                    const int64_t* __restrict__ cand, const int32_t* __restrict__ slot,
                                                    const uint64_t* __restrict__ tkeys,
                                                    uint32_t* flags, unsigned long long* agg, unsigned long long* incl,
                                                    uint32_t* ctl, int32_t* __restrict__ out, int64_t ld_out,
                                                    int32_t* __restrict__ count, int64_t tile_lo, int advance,
                                                    const int32_t* __restrict__ gate) {
  __shared__ int wsum[4];
  __shared__ int gated;
  const uint32_t epoch = ctl[0] + 1u;
  if (threadIdx.x == 0) gated = gate && (int64_t)*gate >= num_neg;
  __syncthreads();
  if (gated) {
    if (llp_arrive_last(&ctl[1], gridDim.x) && threadIdx.x == 0 && advance) {
      const uint32_t next = ((epoch + 1u) & 0xFFFFFFu) == 0u ? epoch + 1u : epoch;
      __hip_atomic_store(&ctl[0], next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  const int64_t b = tile_lo + blockIdx.x;
  const int64_t i0 = b * NC_TILE + 4 * threadIdx.x;
  int v[4], mine = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t i = i0 + k;
    v[k] = 0;
    if (i < M) {
      const int32_t s = slot[i];
      v[k] = (s >= 0 && tkeys[s] == ((uint64_t)(epoch & 0xFFFFFFu) << NEG2_VALUE_BITS | (uint64_t)i)) ? 1 : 0;
    }
    mine += v[k];
  }
  int total;
  const int ex = block_excl_scan256(mine, wsum, &total);
  const int64_t base = (int64_t)llp_lookback_u64(flags, agg, incl, b, (unsigned long long)total, epoch, &ctl[2]);
  int64_t pos = base + ex;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (v[k]) {
      if (pos < num_neg) {
        const int64_t c = cand[i0 + k];
        const int64_t r = c / (num_nodes - 1);
        int64_t cc = c % (num_nodes - 1);
        if (r <= cc) cc += 1;
        out[pos] = (int32_t)r;
        out[ld_out + pos] = (int32_t)cc;
      }
      ++pos;
    }
  }
  // the last workgroup: the count (the last tile's inclusive prefix) and the next call's epoch
  if (llp_arrive_last(&ctl[1], gridDim.x) && threadIdx.x == 0) {
    // a failed look-back (ctl[2] set) left the last tile's prefix unpublished: no negatives
    const bool failed = __hip_atomic_load(&ctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    const unsigned long long all =
        failed ? 0ull
               : __hip_atomic_load(&incl[tile_lo + gridDim.x - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *count = (int32_t)(all < (unsigned long long)num_neg ? all : (unsigned long long)num_neg);
    // the table tags entries with the epoch's low 24 bits, and entries still zero from the initial
    // clear carry tag 0: skip the epochs whose low 24 bits are 0, so no call ever reads those
    // entries as claimed (the next call uses ctl[0] + 1)
    if (advance) {
      const uint32_t next = ((epoch + 1u) & 0xFFFFFFu) == 0u ? epoch + 1u : epoch;
      __hip_atomic_store(&ctl[0], next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ void zero_u32_kernel(int64_t n, uint32_t* __restrict__ p) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0u;
}

// ia/ib for the full-batch predictor rows: B*C context pairs (anchor, context)
// then P positive and n_neg negative label pairs (train_edges, src/main.py:212).
__global__ void fullbatch_pairs_kernel(int64_t B, int64_t C1, const int32_t* __restrict__ samples,
                                       const int32_t* __restrict__ pairs, const int32_t* __restrict__ perm, int64_t P,
                                       const int32_t* __restrict__ neg, int64_t ld_neg, int64_t n_neg,
                                       const int32_t* __restrict__ neg_count, int64_t neg_offset,
                                       int32_t* __restrict__ ia, int32_t* __restrict__ ib) {
  const int64_t C = C1 - 1;
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t BC = B * C;
  if (t < BC) {
    const int64_t b = t / C, c = t % C;
    ia[t] = samples[b * C1];
    ib[t] = samples[b * C1 + 1 + c];
    return;
  }
  const int64_t u = t - BC;
  if (u < P) {
    const int64_t e = perm[u];
    ia[t] = pairs[2 * e];
    ib[t] = pairs[2 * e + 1];
  } else if (u < P + n_neg) {
    // negative slot u - P: past the sampler's device count (neg_offset + slot >= *neg_count) it is
    // an inert pair (node 0, node 0) whose logit the loss ignores (llp_llp_loss with a count)
    const bool live = !neg_count || neg_offset + (u - P) < (int64_t)*neg_count;
    ia[t] = live ? neg[u - P] : 0;
    ib[t] = live ? neg[ld_neg + u - P] : 0;
  }
}

// KD_LM: mse(sigmoid(z), t) mean over n_total label rows; adds the gradient.
__global__ __launch_bounds__(256) void kd_lm_kernel(int64_t n, const float* __restrict__ logit,
                                                    const float* __restrict__ t_prob, double n_total, float w,
                                                    float loss_scale, float* __restrict__ dlogit,
                                                    float* __restrict__ partial) {
  __shared__ float red[4];
  const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  float l = 0.f;
  if (r < n) {
    const float z = logit[r];
    const float o = 1.f / (1.f + __expf(-z));
    const float d = o - t_prob[r];
    l = d * d;
    dlogit[r] += loss_scale * w * (2.f * d / (float)n_total) * o * (1.f - o);
  }
  l = wave_sum(l);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = l;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1] + red[2] + red[3]) / (float)n_total;
}

// KD_RM: 1 - mean_b cos(h[idx_b], t_h[idx_b]) (torch cosine_similarity, eps 1e-8
// clamp on each norm); one wave per row; dh[idx_b] += d/dh.
template <typename T>
__global__ __launch_bounds__(256) void kd_rm_kernel(int64_t B, int64_t H, const T* __restrict__ h, int64_t ldh,
                                                    const T* __restrict__ t_h, int64_t ldt,
                                                    const int32_t* __restrict__ idx, double B_total, float w,
                                                    float loss_scale, float* __restrict__ dh, int64_t lddh,
                                                    float* __restrict__ partial) {
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t b = blockIdx.x * 4 + wv;
  float cosv = 0.f;
  if (b < B) {
    const int64_t row = idx[b];
    const T* hr = h + row * ldh;
    const T* tr = t_h + row * ldt;
    float dot = 0.f, n1 = 0.f, n2 = 0.f;
    for (int64_t j = lane; j < H; j += 64) {
      float a, c;
      if constexpr (sizeof(T) == 2) { a = bf2f(hr[j]); c = bf2f(tr[j]); } else { a = hr[j]; c = tr[j]; }
      dot += a * c; n1 += a * a; n2 += c * c;
    }
    dot = wave_sum(dot); n1 = wave_sum(n1); n2 = wave_sum(n2);
    const float na = fmaxf(sqrtf(n1), 1e-8f), nb = fmaxf(sqrtf(n2), 1e-8f);
    cosv = dot / (na * nb);
    if (dh) {
      const float g = -loss_scale * w / (float)B_total;
      float* dr = dh + row * lddh;
      for (int64_t j = lane; j < H; j += 64) {
        float a, c;
        if constexpr (sizeof(T) == 2) { a = bf2f(hr[j]); c = bf2f(tr[j]); } else { a = hr[j]; c = tr[j]; }
        atomicAdd(&dr[j], g * (c / (na * nb) - cosv * a / (na * na)));
      }
    }
    cosv = 1.f - cosv;   // this row's (1 - cos); summed / B_total = its share of the loss
  }
  if (lane == 0) red[wv] = cosv;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1] + red[2] + red[3]) / (float)B_total;
}

__global__ void kd_finalize(const float* __restrict__ partial, int64_t n_rm, int64_t n_lm, float w_rm, float w_lm,
                            float* __restrict__ terms) {
  __shared__ double red[2][256];
  double a = 0, c = 0;
  for (int64_t i = threadIdx.x; i < n_rm; i += blockDim.x) a += (double)partial[i];
  for (int64_t i = threadIdx.x; i < n_lm; i += blockDim.x) c += (double)partial[n_rm + i];
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = c;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      red[0][threadIdx.x] += red[0][threadIdx.x + s];
      red[1][threadIdx.x] += red[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float rm = (float)red[0][0], lm = (float)red[1][0];
    terms[4] = rm;
    terms[5] = lm;
    terms[0] += w_rm * rm + w_lm * lm;
  }
}

int64_t pow2_at_least(int64_t v) {
  int64_t t = 1;
  while (t < v) t <<= 1;
  return t;
}

}  // namespace

extern "C" int64_t llp_neg_sample_dense_workspace_bytes(int64_t max_candidates) {
  const int64_t T = pow2_at_least(2 * max_candidates);
  const int64_t ntiles = (max_candidates + NC_TILE - 1) / NC_TILE;
  return T * 8 + T * 4 + max_candidates * 8 + max_candidates * 4 + ntiles * 4 + 64;
}

extern "C" int64_t llp_edge_table_size(int64_t n_keys) { return pow2_at_least(2 * (n_keys > 0 ? n_keys : 1)); }

extern "C" int llp_edge_table_build(const int64_t* edge_keys, int64_t n_keys, uint64_t* table, int64_t table_size,
                                    void* stream) {
  LLP_CHECK_ARG(table && (n_keys == 0 || edge_keys), "llp_edge_table_build: null pointer");
  LLP_CHECK_ARG(n_keys >= 0 && table_size >= llp_edge_table_size(n_keys) && (table_size & (table_size - 1)) == 0,
                "llp_edge_table_build: table_size must be a power of two >= llp_edge_table_size(n_keys)");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(edge_table_fill, dim3(ceil_div_u(table_size, 256)), dim3(256), 0, s, table, table_size);
  if (n_keys > 0)
    hipLaunchKernelGGL(edge_table_insert, dim3(ceil_div_u(n_keys, 256)), dim3(256), 0, s, edge_keys, n_keys, table,
                       table_size);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_neg_sample_dense(int64_t num_nodes, const int64_t* edge_keys, int64_t n_keys,
                                    const uint64_t* edge_table, int64_t edge_table_size,
                                    int64_t num_neg, int64_t sample_size, int rounds, uint64_t seed,
                                    const int64_t* step_ctr, int64_t stream_offset, int32_t* out, int64_t ld_out,
                                    int32_t* count, void* workspace, int64_t workspace_bytes, void* stream) {
  LLP_CHECK_ARG(out && count && workspace && step_ctr, "llp_neg_sample_dense: null pointer");
  LLP_CHECK_ARG(num_nodes >= 2 && num_nodes < (1ll << 31), "llp_neg_sample_dense: num_nodes out of range");
  LLP_CHECK_ARG(n_keys == 0 || edge_keys || edge_table, "llp_neg_sample_dense: null edge keys");
  LLP_CHECK_ARG(!edge_table || (edge_table_size > 0 && (edge_table_size & (edge_table_size - 1)) == 0),
                "llp_neg_sample_dense: edge_table_size must be a power of two");
  LLP_CHECK_ARG(rounds >= 1 && sample_size >= 0 && num_neg >= 0 && ld_out >= num_neg,
                "llp_neg_sample_dense: bad sizes");
  hipStream_t s = (hipStream_t)stream;
  const uint64_t population = (uint64_t)num_nodes * (uint64_t)(num_nodes - 1);
  const int enumerate_all = population <= (uint64_t)sample_size;
  // population <= sample_size: every round enumerates range(population); the
  // later rounds can add nothing, so one pass suffices.
  const int64_t M = enumerate_all ? (int64_t)population : (int64_t)rounds * sample_size;
  LLP_CHECK_ARG(workspace_bytes >= llp_neg_sample_dense_workspace_bytes(M), "llp_neg_sample_dense: workspace too small");
  LLP_CHECK_ARG(M < (1ll << 31), "llp_neg_sample_dense: too many candidates");
  const int64_t T = pow2_at_least(2 * M);
  char* w = reinterpret_cast<char*>(workspace);
  uint64_t* tkeys = reinterpret_cast<uint64_t*>(w);
  int32_t* tmin = reinterpret_cast<int32_t*>(w + T * 8);
  int64_t* cand = reinterpret_cast<int64_t*>(w + T * 12);
  int32_t* slot = reinterpret_cast<int32_t*>(w + T * 12 + M * 8);
  if (M > 0) {
    hipLaunchKernelGGL(neg_table_init, dim3(ceil_div_u(T, 256)), dim3(256), 0, s, tkeys, tmin, T);
    LLP_LAUNCH_CHECK();
    hipLaunchKernelGGL(neg_candidates, dim3(ceil_div_u(M, 256)), dim3(256), 0, s, M, enumerate_all, population, seed,
                       step_ctr, stream_offset, edge_keys, n_keys, edge_table, edge_table_size, cand, slot, tkeys,
                       tmin, T);
    LLP_LAUNCH_CHECK();
  }
  const int64_t ntiles = (M + NC_TILE - 1) / NC_TILE;
  int32_t* tbase = reinterpret_cast<int32_t*>(w + T * 12 + M * 12);
  if (ntiles > 0) {
    hipLaunchKernelGGL(neg_tile_count, dim3((unsigned)ntiles), dim3(256), 0, s, M, slot, tmin, tbase);
    LLP_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(neg_tile_scan, dim3(1), dim3(256), 0, s, ntiles, num_neg, tbase, count);
  LLP_LAUNCH_CHECK();
  if (ntiles > 0) {
    hipLaunchKernelGGL(neg_tile_scatter, dim3((unsigned)ntiles), dim3(256), 0, s, M, num_nodes, num_neg, cand, slot,
                       tmin, tbase, out, ld_out);
    LLP_LAUNCH_CHECK();
  }
  return LLP_OK;
}

static int64_t al256b(int64_t b) { return (b + 255) & ~(int64_t)255; }

static int64_t neg2_state_bytes(int64_t M) {
  const int64_t T = pow2_at_least(2 * (M > 0 ? M : 1));
  const int64_t ntiles = (M + NC_TILE - 1) / NC_TILE;
  return al256b(T * 8) + al256b(ntiles * 4) + 256;
}

extern "C" int64_t llp_neg_sample_dense2_state_bytes(int64_t max_candidates) { return neg2_state_bytes(max_candidates); }

extern "C" int64_t llp_neg_sample_dense2_workspace_bytes(int64_t max_candidates) {
  const int64_t ntiles = (max_candidates + NC_TILE - 1) / NC_TILE;
  return neg2_state_bytes(max_candidates) + 2 * al256b(ntiles * 8) + al256b(max_candidates * 8) +
         al256b(max_candidates * 4);
}

extern "C" int llp_neg_sample_dense2(int64_t num_nodes, const int64_t* edge_keys, int64_t n_keys,
                                     const uint64_t* edge_table, int64_t edge_table_size, int64_t num_neg,
                                     int64_t sample_size, int rounds, uint64_t seed, const int64_t* step_ctr,
                                     int64_t stream_offset, int32_t* out, int64_t ld_out, int32_t* count,
                                     int state_clean, void* workspace, int64_t workspace_bytes, void* stream) {
  LLP_CHECK_ARG(out && count && workspace && step_ctr, "llp_neg_sample_dense2: null pointer");
  LLP_CHECK_ARG(num_nodes >= 2 && num_nodes < (1ll << 31), "llp_neg_sample_dense2: num_nodes out of range");
  LLP_CHECK_ARG(n_keys == 0 || edge_keys || edge_table, "llp_neg_sample_dense2: null edge keys");
  LLP_CHECK_ARG(!edge_table || (edge_table_size > 0 && (edge_table_size & (edge_table_size - 1)) == 0),
                "llp_neg_sample_dense2: edge_table_size must be a power of two");
  LLP_CHECK_ARG(rounds >= 1 && sample_size >= 0 && num_neg >= 0 && ld_out >= num_neg,
                "llp_neg_sample_dense2: bad sizes");
  const uint64_t population = (uint64_t)num_nodes * (uint64_t)(num_nodes - 1);
  LLP_CHECK_ARG(population <= NEG2_VALUE_MASK, "llp_neg_sample_dense2: N(N-1) >= 2^40 (use llp_neg_sample_dense)");
  hipStream_t s = (hipStream_t)stream;
  const int enumerate_all = population <= (uint64_t)sample_size;
  const int64_t M = enumerate_all ? (int64_t)population : (int64_t)rounds * sample_size;
  LLP_CHECK_ARG(M < (1ll << 31), "llp_neg_sample_dense2: too many candidates");
  LLP_CHECK_ARG(workspace_bytes >= llp_neg_sample_dense2_workspace_bytes(M), "llp_neg_sample_dense2: workspace");
  const int64_t T = pow2_at_least(2 * (M > 0 ? M : 1));
  const int64_t ntiles = (M + NC_TILE - 1) / NC_TILE;
  char* w = reinterpret_cast<char*>(workspace);
  if (!state_clean) {
    const int64_t n32 = neg2_state_bytes(M) / 4;
    hipLaunchKernelGGL(zero_u32_kernel, dim3(ceil_div_u(n32, 256)), dim3(256), 0, s, n32, (uint32_t*)w);
    LLP_LAUNCH_CHECK();
  }
  uint64_t* tkeys = reinterpret_cast<uint64_t*>(w);
  w += al256b(T * 8);
  uint32_t* flags = reinterpret_cast<uint32_t*>(w);
  w += al256b(ntiles * 4);
  uint32_t* ctl = reinterpret_cast<uint32_t*>(w);
  w += 256;
  unsigned long long* agg = reinterpret_cast<unsigned long long*>(w);
  w += al256b(ntiles * 8);
  unsigned long long* incl = reinterpret_cast<unsigned long long*>(w);
  w += al256b(ntiles * 8);
  int64_t* cand = reinterpret_cast<int64_t*>(w);
  w += al256b(M * 8);
  int32_t* slot = reinterpret_cast<int32_t*>(w);
  if (M == 0) {   // nothing to draw: no negatives
    hipLaunchKernelGGL(zero_u32_kernel, dim3(1), dim3(256), 0, s, (int64_t)1, (uint32_t*)count);
    LLP_LAUNCH_CHECK();
    return LLP_OK;
  }
  // Round-gated: PyG's sampler stops after the first round of sample_size candidates whenever it
  // holds num_neg valid ones, which at sample_size = 1.1 num_neg / prob is practically always.
  // The first round's tiles are drawn and compacted first; the later rounds' launches read that
  // count on the device and do nothing when it suffices (no host read, graph-capturable).  The
  // result is the same as compacting all rounds at once: the first num_neg valid first
  // occurrences in draw order (the later rounds' candidates come after, and their repeats of
  // first-round values lose the slot to the lower index).  Round 1 ends on a tile boundary.
  int64_t M1 = M;
#ifndef LLP_NEG_ONE_PHASE   // A/B build: every round's candidates in one pass (round 4)
  if (!enumerate_all && rounds > 1) {
    M1 = (sample_size + NC_TILE - 1) / NC_TILE * NC_TILE;
    if (M1 >= M) M1 = M;
  }
#endif
  const int64_t nt1 = (M1 + NC_TILE - 1) / NC_TILE;
  hipLaunchKernelGGL(neg_candidates2, dim3(ceil_div_u(M1, 256)), dim3(256), 0, s, (int64_t)0, M1, enumerate_all,
                     population, seed, step_ctr, stream_offset, edge_keys, n_keys, edge_table, edge_table_size, cand,
                     slot, tkeys, T, (const uint32_t*)ctl, (const int32_t*)nullptr, num_neg);
  LLP_LAUNCH_CHECK();
  hipLaunchKernelGGL(neg_compact2, dim3((unsigned)nt1), dim3(256), 0, s, M, num_nodes, num_neg, cand, slot, tkeys,
                     flags, agg, incl, ctl, out, ld_out, count, (int64_t)0, M1 == M ? 1 : 0, (const int32_t*)nullptr);
  LLP_LAUNCH_CHECK();
  if (M1 < M) {
    hipLaunchKernelGGL(neg_candidates2, dim3(ceil_div_u(M - M1, 256)), dim3(256), 0, s, M1, M, enumerate_all,
                       population, seed, step_ctr, stream_offset, edge_keys, n_keys, edge_table, edge_table_size,
                       cand, slot, tkeys, T, (const uint32_t*)ctl, (const int32_t*)count, num_neg);
    LLP_LAUNCH_CHECK();
    hipLaunchKernelGGL(neg_compact2, dim3((unsigned)(ntiles - nt1)), dim3(256), 0, s, M, num_nodes, num_neg, cand, slot,
                       tkeys, flags, agg, incl, ctl, out, ld_out, count, nt1, 1, (const int32_t*)count);
    LLP_LAUNCH_CHECK();
  }
  return LLP_OK;
}

extern "C" int llp_fullbatch_pairs(int64_t B, int64_t C1, const int32_t* samples, const int32_t* pairs,
                                   const int32_t* perm, int64_t P, const int32_t* neg, int64_t ld_neg, int64_t n_neg,
                                   const int32_t* neg_count, int64_t neg_offset, int32_t* ia, int32_t* ib,
                                   void* stream) {
  LLP_CHECK_ARG(B == 0 || (samples && C1 >= 2), "llp_fullbatch_pairs: null samples");
  LLP_CHECK_ARG(P == 0 || (pairs && perm), "llp_fullbatch_pairs: null pairs");
  LLP_CHECK_ARG(n_neg == 0 || neg, "llp_fullbatch_pairs: null negatives");
  const int64_t n = B * (C1 > 0 ? C1 - 1 : 0) + P + n_neg;
  if (n == 0) return LLP_OK;   // an empty batch: nothing to write (the outputs may be empty tensors)
  LLP_CHECK_ARG(ia && ib, "llp_fullbatch_pairs: null output");
  hipLaunchKernelGGL(fullbatch_pairs_kernel, dim3(ceil_div_u(n, 256)), dim3(256), 0, (hipStream_t)stream, B, C1,
                     samples, pairs, perm, P, neg, ld_neg, n_neg, neg_count, neg_offset, ia, ib);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int64_t llp_kd_terms_workspace_bytes(int64_t B_rm, int64_t n_lab) {
  return ((B_rm + 3) / 4 + (n_lab + 255) / 256 + 2) * (int64_t)sizeof(float);
}

extern "C" int llp_kd_terms(int dtype, int64_t n_lab, const float* out_logit, const float* t_prob_lab,
                            double n_lab_total, float w_lm, int64_t B_rm, int64_t H, const void* h, int64_t ldh,
                            const void* t_h, int64_t ldt, const int32_t* idx_rm, double B_rm_total, float w_rm,
                            float loss_scale, float* dlogit_lab, float* dh, int64_t lddh, float* terms_out,
                            void* workspace, int64_t workspace_bytes, void* stream) {
  LLP_CHECK_ARG(terms_out && workspace, "llp_kd_terms: null terms/workspace");
  LLP_CHECK_ARG(workspace_bytes >= llp_kd_terms_workspace_bytes(B_rm, n_lab), "llp_kd_terms: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  float* partial = reinterpret_cast<float*>(workspace);
  const int64_t nrm = B_rm > 0 ? (B_rm + 3) / 4 : 0;
  const int64_t nlm = n_lab > 0 ? (n_lab + 255) / 256 : 0;
  if (nrm > 0) {
    LLP_CHECK_ARG(h && t_h && idx_rm, "llp_kd_terms: null KD_RM buffers");
    if (dtype == LLP_BF16)
      hipLaunchKernelGGL(kd_rm_kernel<bf16_t>, dim3((unsigned)nrm), dim3(256), 0, s, B_rm, H, (const bf16_t*)h, ldh,
                         (const bf16_t*)t_h, ldt, idx_rm, B_rm_total, w_rm, loss_scale, dh, lddh, partial);
    else
      hipLaunchKernelGGL(kd_rm_kernel<float>, dim3((unsigned)nrm), dim3(256), 0, s, B_rm, H, (const float*)h, ldh,
                         (const float*)t_h, ldt, idx_rm, B_rm_total, w_rm, loss_scale, dh, lddh, partial);
    LLP_LAUNCH_CHECK();
  }
  if (nlm > 0) {
    LLP_CHECK_ARG(out_logit && t_prob_lab && dlogit_lab, "llp_kd_terms: null KD_LM buffers");
    hipLaunchKernelGGL(kd_lm_kernel, dim3((unsigned)nlm), dim3(256), 0, s, n_lab, out_logit, t_prob_lab, n_lab_total,
                       w_lm, loss_scale, dlogit_lab, partial + nrm);
    LLP_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(kd_finalize, dim3(1), dim3(256), 0, s, partial, nrm, nlm, w_rm, w_lm, terms_out);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}
