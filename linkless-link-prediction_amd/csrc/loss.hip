// Fused distillation losses and the link-predictor head.
//
//   llp_llp_loss : one wavefront per anchor — sigmoid, softmax/KL (LLP_D),
//                  all-pairs margin rank (LLP_R), plus the label BCE rows, and
//                  d(loss)/d(logit) for every predictor row.  Replaces
//                  src/main.py:98-130 (which materialises B x C(C-1)/2 pair
//                  tensors and a host-built numpy pair index every step).
//   llp_head_fwd / llp_head_bwd : last Linear(H,1)+sigmoid of LinkPredictor
//                  (src/models.py:146,150) as a row-dot, and its backward with
//                  the ReLU of the layer below fused.
#include "llp_common.h"

namespace {

constexpr int MAXC = 1024;
constexpr int WAVES = 4;

__device__ __forceinline__ float sigmoidf_(float z) { return 1.f / (1.f + expf(-z)); }

// The Linear(H, 1) head's finish (head_finish_kernel, gemm.hip) inside the loss: logit of
// predictor row m = bias + the per-256-column GEMM partials part[t * ld + m] in column order --
// the same fp32 sum, so the logits are bit-identical to a separate head_finish launch.
struct HeadIn {
  const float* part;   // [parts][ld] partials of gemm_nt_head, or NULL: logits read as given
  const float* bias;   // [1] or NULL
  int64_t parts, ld;
};
__device__ __forceinline__ float head_sum(const HeadIn& h, int64_t m) {
  float s = h.bias ? h.bias[0] : 0.f;
  for (int64_t t = 0; t < h.parts; ++t) s += h.part[t * h.ld + m];
  return s;
}

// partial sums per block: [bce, kl, rank].  CMAX: the LDS row per wave (64 for C <= 64, the
// collab / physics shapes: 2 KiB of LDS per block instead of 32 KiB, so a CU holds 8x the waves)
// With hs.part / ht.part the student logits (rows b*C + c of the predictor) and the teacher's
// probabilities are finished here from the head partials and written to s_logit / t_prob.
template <int CMAX>
__device__ __forceinline__ void llp_anchor_block(int64_t blk, int64_t B, int64_t C, float* __restrict__ s_logit,
                                                 float* __restrict__ t_prob, const HeadIn& hs, const HeadIn& ht,
                                                 double B_total, float margin, float T, float w_d, float w_r,
                                                 float loss_scale, float* __restrict__ dlogit,
                                                 float* __restrict__ partial, int64_t tb0, int64_t tb1) {
  __shared__ float ss[WAVES][CMAX];
  __shared__ float tt[WAVES][CMAX];
  __shared__ float red[WAVES][2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b = blk * WAVES + w;
  float kl_acc = 0.f, rk_acc = 0.f;
  if (b < B) {
    float* sl = s_logit + b * C;
    float* tp = t_prob + b * C;
    float* sw = ss[w];
    float* tw = tt[w];
    // sigmoid probabilities (Q4) and the softmax statistics of s/T and t/T
    float ms = -INFINITY, mt = -INFINITY;
    for (int c = lane; c < C; c += 64) {
      float z = 0.f, t = 0.f;
      if (hs.part) {
        z = head_sum(hs, b * C + c);
        sl[c] = z;
      } else {
        z = sl[c];
      }
      if (ht.part) {
        t = 1.f / (1.f + expf(-head_sum(ht, b * C + c)));
        tp[c] = t;
      } else {
        t = tp[c];
      }
      const float s = sigmoidf_(z);
      sw[c] = s;
      tw[c] = t;
      ms = fmaxf(ms, s / T);
      mt = fmaxf(mt, t / T);
    }
    ms = wave_max(ms);
    mt = wave_max(mt);
    float zs = 0.f, zt = 0.f;
    for (int c = lane; c < C; c += 64) {
      zs += expf(sw[c] / T - ms);
      zt += expf(tw[c] / T - mt);
    }
    zs = wave_sum(zs);
    zt = wave_sum(zt);
    const float lse_s = logf(zs) + ms, lse_t = logf(zt) + mt;
    const float inv_b = (float)(1.0 / B_total);
    const double npairs = (double)C * (double)(C - 1) / 2.0;
    const float inv_bp = npairs > 0 ? (float)(1.0 / (B_total * npairs)) : 0.f;
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < C; i += 64) {
      const float si = sw[i], ti = tw[i];
      // KL(p_t || q_s) pointwise, kl_div(log q, p, 'sum') = p (log p - log q)
      const float logq = si / T - lse_s, logp = ti / T - lse_t;
      const float pt = expf(logp), qs = expf(logq);
      kl_acc += pt * (logp - logq);
      const float dkl = T * (qs - pt) * inv_b;  // d/ds of KL * T^2 / B
      // rank: pairs (i, j) lexicographic, i < j  (itertools.combinations)
      float gi = 0.f;
      for (int j = 0; j < C; ++j) {
        if (j == i) continue;
        const float sj = sw[j], tj = tw[j];
        if (j > i) {
          const float y = ti > tj + margin ? 1.f : (ti < tj - margin ? -1.f : 0.f);
          const float h = -y * (si - sj) + margin;
          rk_acc += fmaxf(h, 0.f);
          if (h >= 0.f) gi -= y;
        } else {
          const float y = tj > ti + margin ? 1.f : (tj < ti - margin ? -1.f : 0.f);
          const float h = -y * (sj - si) + margin;
          if (h >= 0.f) gi += y;
        }
      }
      const float ds = w_d * dkl + w_r * gi * inv_bp;
      dlogit[b * C + i] = loss_scale * ds * si * (1.f - si);  // through the sigmoid
    }
    kl_acc = wave_sum(kl_acc) * (T * T) * inv_b;
    rk_acc = wave_sum(rk_acc) * inv_bp;
    if (b < tb0 || b >= tb1) kl_acc = rk_acc = 0.f;   // another rank reports this anchor's terms
  }
  if (lane == 0) {
    red[w][0] = kl_acc;
    red[w][1] = rk_acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float k = 0.f, r = 0.f;
    for (int i = 0; i < WAVES; ++i) {
      k += red[i][0];
      r += red[i][1];
    }
    llp_store_handed(partial + blk * 3 + 0, 0.f);   // (read by the last workgroup of the launch)
    llp_store_handed(partial + blk * 3 + 1, k);
    llp_store_handed(partial + blk * 3 + 2, r);
  }
}

// neg_count (device, may be NULL): the label rows are n_pos positives then negative slots of
// which those with neg_offset + slot < *neg_count are live; the others get a zero gradient and
// no loss, and the mean is over pos_total + *neg_count labels (the whole batch's).
// With hl.part the label logits (predictor rows lab_row0 + r) are finished from the head partials
// and written to logit[r].
__device__ __forceinline__ void bce_block(int64_t blk, int64_t n, int64_t n_pos, float* __restrict__ logit,
                                          const HeadIn& hl, int64_t lab_row0, double n_total,
                                          const int32_t* __restrict__ neg_count, int64_t neg_offset,
                                          double pos_total, float w_label, float loss_scale,
                                          float* __restrict__ dlogit, float* __restrict__ partial) {
  __shared__ float red[4];
  const int64_t r = blk * (int64_t)blockDim.x + threadIdx.x;
  int64_t n_live = n;
  if (neg_count) {
    const int64_t c = *neg_count;
    const int64_t nl = c - neg_offset;
    n_live = n_pos + (nl < 0 ? 0 : (nl > n - n_pos ? n - n_pos : nl));
    n_total = pos_total + (double)c;
  }
  float l = 0.f;
  if (r < n && hl.part) logit[r] = head_sum(hl, lab_row0 + r);   // every slot, inert ones too
  if (r < n && r >= n_live) dlogit[r] = 0.f;
  if (r < n_live) {
    const float o = sigmoidf_(logit[r]);
    const float y = r < n_pos ? 1.f : 0.f;
    // nn.BCELoss: -(y*max(log o, -100) + (1-y)*max(log(1-o), -100)), mean
    const float lo = fmaxf(logf(o), -100.f), l1o = fmaxf(logf(1.f - o), -100.f);
    l = -(y * lo + (1.f - y) * l1o);
    const float go = (o - y) / fmaxf((1.f - o) * o, 1e-12f) / (float)n_total;
    dlogit[r] = loss_scale * w_label * go * o * (1.f - o);
  }
  l = wave_sum(l);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = l;
  __syncthreads();
  if (threadIdx.x == 0) {
    llp_store_handed(partial + blk * 3 + 0, (red[0] + red[1] + red[2] + red[3]) / (float)n_total);
    llp_store_handed(partial + blk * 3 + 1, 0.f);
    llp_store_handed(partial + blk * 3 + 2, 0.f);
  }
}

// the three terms from the per-block partials: a fixed tree in double (deterministic)
template <bool HANDOFF>
__device__ __forceinline__ void loss_finalize_block(const float* partial, int64_t nblocks, float w_label, float w_d,
                                                    float w_r, float* __restrict__ terms, int accumulate) {
  __shared__ double red[3][256];
  double a[3] = {0, 0, 0};
  // partials of other workgroups of this launch (write-through loads, never the scalar path):
  // eight blocks' worth issued before any is summed -- the compiler does not batch atomic loads
  // across iterations, and one round trip per block cost ~20 us of the physics step
  constexpr int U = 8;
  for (int64_t i0 = threadIdx.x; i0 < nblocks; i0 += (int64_t)U * blockDim.x) {
    float v[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * blockDim.x;
#pragma unroll
      for (int k = 0; k < 3; ++k)
        v[u][k] = i < nblocks ? (HANDOFF ? llp_load_handed(partial + i * 3 + k) : partial[i * 3 + k]) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + (int64_t)u * blockDim.x < nblocks)
#pragma unroll
        for (int k = 0; k < 3; ++k) a[k] += (double)v[u][k];
  }
  for (int k = 0; k < 3; ++k) red[k][threadIdx.x] = a[k];
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
      for (int k = 0; k < 3; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float bce = (float)red[0][0], kl = (float)red[1][0], rk = (float)red[2][0];
    const float loss = w_label * bce + w_d * kl + w_r * rk;
    if (accumulate) {
      terms[0] += loss; terms[1] += bce; terms[2] += kl; terms[3] += rk;
    } else {
      terms[0] = loss; terms[1] = bce; terms[2] = kl; terms[3] = rk;
    }
  }
}

struct LossArgs {
  int64_t B, C, n_lab, n_pos, nba, nbl;
  float* s_logit; float* t_prob; HeadIn hs, ht;
  float* out_logit; int64_t lab_row0;
  double B_total, n_lab_total, pos_total;
  float margin, T, w_label, w_d, w_r, loss_scale;
  float* dlogit_ctx; float* dlogit_lab;
  const int32_t* neg_count; int64_t neg_offset;
  int64_t tb0, tb1;
  float* partial; float* terms; int accumulate;
  uint32_t* ticket;   // NULL: loss_finalize_kernel follows; else zero on entry, left zero
};

// The whole loss in one launch: blocks [0, nba) are the anchors' (llp_anchor_block), the
// rest the label rows' (bce_block); the workgroup that arrives last on the ticket sums every
// block's partials (the same tree as loss_finalize_kernel) and returns the ticket to zero.
// Hand-off: each block's partials are stored by one lane with write-through atomic stores and
// drained (vmcnt(0)) before its ticket add; the last arriver reads them with write-through
// atomic loads (llp_common.h: llp_store_handed / llp_arrive_last_tree / llp_load_handed).
template <int CMAX>
__global__ __launch_bounds__(256) void llp_loss_kernel(LossArgs a) {
  const int64_t blk = blockIdx.x;
  if (blk < a.nba)
    llp_anchor_block<CMAX>(blk, a.B, a.C, a.s_logit, a.t_prob, a.hs, a.ht, a.B_total, a.margin, a.T, a.w_d, a.w_r,
                           a.loss_scale, a.dlogit_ctx, a.partial, a.tb0, a.tb1);
  else
    bce_block(blk - a.nba, a.n_lab, a.n_pos, a.out_logit, a.hs, a.lab_row0, a.n_lab_total, a.neg_count,
              a.neg_offset, a.pos_total, a.w_label, a.loss_scale, a.dlogit_lab, a.partial + a.nba * 3);
  if (!a.ticket) return;
  if (!llp_arrive_last_tree(a.ticket, blockIdx.x, (uint32_t)(a.nba + a.nbl))) return;
  loss_finalize_block<true>(a.partial, a.nba + a.nbl, a.w_label, a.w_d, a.w_r, a.terms, a.accumulate);
}

__global__ void loss_finalize_kernel(const float* __restrict__ partial, int64_t nblocks, float w_label, float w_d,
                                     float w_r, float* __restrict__ terms, int accumulate) {
  loss_finalize_block<false>(partial, nblocks, w_label, w_d, w_r, terms, accumulate);
}

// ------------------------------------------------------------------ head
template <typename T>
__device__ __forceinline__ float ldf(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ldf<float>(const float* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ldf<bf16_t>(const bf16_t* p, int64_t i) { return bf2f(p[i]); }

// one wave per row
template <typename T>
__global__ __launch_bounds__(256) void head_fwd_kernel(int64_t R, int64_t H, const T* __restrict__ Z, int64_t ldz,
                                                       const T* __restrict__ Z2, int64_t ldz2,
                                                       const int32_t* __restrict__ iz, const int32_t* __restrict__ iz2,
                                                       const float* __restrict__ w, const float* __restrict__ b,
                                                       float* __restrict__ logit, float* __restrict__ prob) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const T* z = Z + (iz ? (int64_t)iz[r] : r) * ldz;
  const T* z2 = Z2 ? Z2 + (iz2 ? (int64_t)iz2[r] : r) * ldz2 : nullptr;
  float acc = 0.f;
  constexpr int E = 16 / sizeof(T);
  const bool vec = (H % E == 0) && ((uintptr_t)z % 16 == 0) && (!z2 || (uintptr_t)z2 % 16 == 0) &&
                   (!w || (uintptr_t)w % 16 == 0);
  if (vec) {
    // 16-byte chunks of the row per lane (the row is streamed once, 1 KiB per wave-instruction)
    for (int64_t c = lane; c < H / E; c += 64) {
      const uint4 raw = *reinterpret_cast<const uint4*>(z + c * E);
      float v[E];
      if constexpr (sizeof(T) == 2) {
        const uint32_t u[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[2 * i] = __uint_as_float(u[i] << 16);
          v[2 * i + 1] = __uint_as_float(u[i] & 0xFFFF0000u);
        }
      } else {
        v[0] = __uint_as_float(raw.x); v[1] = __uint_as_float(raw.y);
        v[2] = __uint_as_float(raw.z); v[3] = __uint_as_float(raw.w);
      }
      if (z2) {
        const uint4 r2 = *reinterpret_cast<const uint4*>(z2 + c * E);
        if constexpr (sizeof(T) == 2) {
          const uint32_t u[4] = {r2.x, r2.y, r2.z, r2.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[2 * i] *= __uint_as_float(u[i] << 16);
            v[2 * i + 1] *= __uint_as_float(u[i] & 0xFFFF0000u);
          }
        } else {
          v[0] *= __uint_as_float(r2.x); v[1] *= __uint_as_float(r2.y);
          v[2] *= __uint_as_float(r2.z); v[3] *= __uint_as_float(r2.w);
        }
      }
#pragma unroll
      for (int i = 0; i < E; ++i) acc += w ? v[i] * w[c * E + i] : v[i];
    }
  } else {
    for (int64_t n = lane; n < H; n += 64) {
      float v = ldf<T>(z, n);
      if (z2) v *= ldf<T>(z2, n);
      acc += w ? v * w[n] : v;
    }
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    const float lg = acc + (b ? b[0] : 0.f);
    if (logit) logit[r] = lg;
    if (prob) prob[r] = sigmoidf_(lg);
  }
}

// Rows per colsum block (host and device agree: the grid and each block's range derive from
// R alone).  The vector kernel holds 140 VGPRs, so a CU keeps 3 of its blocks resident (768
// on the chip): up to 524,288 rows the grid is ~512 blocks (one resident round, no tail round),
// each a whole number of 64-row batches (LLP_COLSUM_INFLIGHT x rows per pass is 64 at H = 256
// bf16, 16 at H = 1024, so only the grid's last block runs the row-at-a-time tail); beyond, 512
// rows per block over several rounds.  Head backward (tools/colsum_probe.py,
// profiles/r06_colsum_blocks.txt), us, round 5 -> this rule: 603,032 x 1024 508 -> 501,
// 225,000 x 1024 220 -> 200, 400,000 x 256 108 -> 92, 130,000 x 256 42 -> 31, 100,000 x 256 32 -> 26.
#ifndef COLSUM_BLOCKS
#define COLSUM_BLOCKS 512
#endif
#ifndef COLSUM_MIN_ROWS
#define COLSUM_MIN_ROWS 64
#endif
__host__ __device__ inline int64_t colsum_rows(int64_t R) {
  int64_t hb = (R + COLSUM_BLOCKS - 1) / COLSUM_BLOCKS;
  if (hb > 1024) return 512;
  hb = hb < COLSUM_MIN_ROWS ? COLSUM_MIN_ROWS : hb;
  return (hb + 63) / 64 * 64;
}

// Column sums (weighted: sum_r weight[r] * Z[r, n]) with the head backward's dZ
// write fused in.  Vector form: a row is cpr 16-byte chunks; 256 threads
// cover rpp = 256 / cpr rows per pass and a block walks HB_ROWS rows; the rpp
// partial rows are combined in LDS and one slab row [blk][H] is written.
#ifndef LLP_COLSUM_MINB
#define LLP_COLSUM_MINB 1
#endif
template <typename T, bool HAS_W>
__global__ __launch_bounds__(256, LLP_COLSUM_MINB) void colsum_vec_kernel(int64_t R, int64_t H, const T* __restrict__ Z, int64_t ldz,
                                                         const float* __restrict__ weight,
                                                         const float* __restrict__ w, int relu_mask, float alpha,
                                                         T* __restrict__ dZ, int64_t lddz, float* __restrict__ slab,
                                                         float* __restrict__ slab_b, const int32_t* __restrict__ r_dev) {
  constexpr int CH = 16 / sizeof(T);
  __shared__ float part[256 * CH];
  __shared__ float partb[256];
  const int cpr = (int)(H / CH);
  const int rpp = 256 / cpr;
  const int t = threadIdx.x;
  const int c = t % cpr, rl = t / cpr;
  const bool active = rl < rpp;
  const int64_t hb = colsum_rows(R);   // the grid's split (host R); rows past *r_dev are not live
  const int64_t r0 = (int64_t)blockIdx.x * hb;
  const int64_t r1 = min(r_dev ? min(R, (int64_t)*r_dev) : R, r0 + hb);
  float acc[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) acc[i] = 0.f;
  float accb = 0.f;
  float wv[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) wv[i] = (w && active) ? alpha * w[c * CH + i] : alpha;
  // LLP_COLSUM_INFLIGHT rows in flight per lane: issue the loads, then consume them in order.
  // The rows' weights are loaded BEFORE their chunks: a weight load issued after them (the
  // round-5 form, weight[r] read inside the row's step) made every row wait for vmcnt(0) --
  // all chunks in flight and the previous rows' dZ stores -- which serialised the stores.
  auto consume = [&](int64_t r, const uint4 raw, const float g) {
    float z[CH];
    if constexpr (sizeof(T) == 2) {
      const uint32_t u[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        z[2 * i] = __uint_as_float(u[i] << 16);
        z[2 * i + 1] = __uint_as_float(u[i] & 0xFFFF0000u);
      }
    } else {
      z[0] = __uint_as_float(raw.x); z[1] = __uint_as_float(raw.y);
      z[2] = __uint_as_float(raw.z); z[3] = __uint_as_float(raw.w);
    }
    accb += g;
#pragma unroll
    for (int i = 0; i < CH; ++i) acc[i] += g * z[i];
    if (dZ) {
      float d[CH];
#pragma unroll
      for (int i = 0; i < CH; ++i) d[i] = (relu_mask && !(z[i] > 0.f)) ? 0.f : g * wv[i];
      uint4 o;
      if constexpr (sizeof(T) == 2) {
        o.x = (uint32_t)f2bf(d[0]) | ((uint32_t)f2bf(d[1]) << 16);
        o.y = (uint32_t)f2bf(d[2]) | ((uint32_t)f2bf(d[3]) << 16);
        o.z = (uint32_t)f2bf(d[4]) | ((uint32_t)f2bf(d[5]) << 16);
        o.w = (uint32_t)f2bf(d[6]) | ((uint32_t)f2bf(d[7]) << 16);
      } else {
        o = make_uint4(__float_as_uint(d[0]), __float_as_uint(d[1]), __float_as_uint(d[2]), __float_as_uint(d[3]));
      }
      *reinterpret_cast<uint4*>(dZ + r * lddz + (int64_t)c * CH) = o;
    }
  };
  if (active) {
    int64_t r = r0 + rl;
#ifndef LLP_COLSUM_INFLIGHT
#define LLP_COLSUM_INFLIGHT 8
#endif
    constexpr int NF = LLP_COLSUM_INFLIGHT;   // rows in flight per lane (16 B each)
    for (; r + (NF - 1) * rpp < r1; r += NF * rpp) {
      float gw[NF];
#pragma unroll
      for (int j = 0; j < NF; ++j) gw[j] = HAS_W ? weight[r + j * rpp] : 1.f;
      uint4 raw[NF];
#pragma unroll
      for (int j = 0; j < NF; ++j) raw[j] = *reinterpret_cast<const uint4*>(Z + (r + j * rpp) * ldz + (int64_t)c * CH);
#pragma unroll
      for (int j = 0; j < NF; ++j) consume(r + j * rpp, raw[j], gw[j]);
    }
    for (; r < r1; r += rpp) {
      const float g = HAS_W ? weight[r] : 1.f;
      consume(r, *reinterpret_cast<const uint4*>(Z + r * ldz + (int64_t)c * CH), g);
    }
  }
  // combine the rpp row-lanes (fixed order -> deterministic)
  if (active)
#pragma unroll
    for (int i = 0; i < CH; ++i) part[rl * (cpr * CH) + c * CH + i] = acc[i];
  partb[t] = active ? accb : 0.f;
  __syncthreads();
  for (int n = t; n < H; n += 256) {
    float s = 0.f;
    for (int k = 0; k < rpp; ++k) s += part[k * (cpr * CH) + n];
    slab[blockIdx.x * H + n] = s;
  }
  if (slab_b && t == 0) {
    float s = 0.f;
    for (int k = 0; k < rpp; ++k) s += partb[k * cpr];
    slab_b[blockIdx.x] = s;
  }
}

// Scalar fallback for widths that are not a multiple of 16 bytes / wider than 256 chunks.
template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(int64_t R, int64_t H, const T* __restrict__ Z, int64_t ldz,
                                                     const float* __restrict__ weight, const float* __restrict__ w,
                                                     int relu_mask, float alpha, T* __restrict__ dZ, int64_t lddz,
                                                     float* __restrict__ slab, float* __restrict__ slab_b,
                                                     const int32_t* __restrict__ r_dev) {
  const int64_t hb = colsum_rows(R);   // the grid's split (host R); rows past *r_dev are not live
  const int64_t r0 = (int64_t)blockIdx.x * hb;
  const int64_t r1 = min(r_dev ? min(R, (int64_t)*r_dev) : R, r0 + hb);
  for (int64_t n = threadIdx.x; n < H; n += blockDim.x) {
    const float wn = w ? w[n] : 1.f;
    float acc = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
      const float z = ldf<T>(Z + r * ldz, n);
      const float g = weight ? weight[r] : 1.f;
      acc += g * z;
      if (dZ) {
        float d = alpha * g * wn;
        if (relu_mask && !(z > 0.f)) d = 0.f;
        if constexpr (sizeof(T) == 2)
          dZ[r * lddz + n] = f2bf(d);
        else
          dZ[r * lddz + n] = d;
      }
    }
    slab[blockIdx.x * H + n] = acc;
  }
  if (slab_b && threadIdx.x == 0) {
    float s = 0.f;
    for (int64_t r = r0; r < r1; ++r) s += weight ? weight[r] : 1.f;
    slab_b[blockIdx.x] = s;
  }
}

// out[n] (+)= sum_i slab[i][n] in a fixed order: SUM_CB columns x (256 / SUM_CB)
// slab-lanes per block (one column and 256 lanes when H == 1), four independent
// partial sums per lane so four loads are in flight, then an LDS tree over the
// lanes.  (One column chain of ~1,000 dependent loads per 16 lanes took ~20 us.)
constexpr int SUM_CB = 4;
struct SumJob { const float* slab; int64_t nslab, H; float* out; };
// blocks [0, nblk0) take job 0 (the weight-gradient columns), the rest job 1 (the bias)
__global__ __launch_bounds__(256) void slab_sum_kernel(SumJob j0, SumJob j1, int64_t nblk0, int accumulate) {
  __shared__ float red[256];
  const bool second = (int64_t)blockIdx.x >= nblk0;
  const SumJob& j = second ? j1 : j0;
  const float* __restrict__ slab = j.slab;
  const int64_t nslab = j.nslab, H = j.H;
  const int cb = H >= SUM_CB ? SUM_CB : 1;
  const int nl = 256 / cb;
  const int cl = threadIdx.x % cb, sl = threadIdx.x / cb;
  const int64_t n = ((int64_t)blockIdx.x - (second ? nblk0 : 0)) * cb + cl;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (n < H) {
    int64_t i = sl;
    for (; i + 3 * nl < nslab; i += 4 * nl) {
      s0 += slab[i * H + n];
      s1 += slab[(i + nl) * H + n];
      s2 += slab[(i + 2 * nl) * H + n];
      s3 += slab[(i + 3 * nl) * H + n];
    }
    for (; i < nslab; i += nl) s0 += slab[i * H + n];
  }
  red[threadIdx.x] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  for (int st = nl / 2; st > 0; st >>= 1) {
    if (sl < st) red[sl * cb + cl] += red[(sl + st) * cb + cl];
    __syncthreads();
  }
  if (sl == 0 && n < H) {
    const float v = red[cl];
    j.out[n] = accumulate ? j.out[n] + v : v;
  }
}

}  // namespace

extern "C" int64_t llp_llp_loss_workspace_bytes(int64_t B, int64_t n_lab) {
  const int64_t nb = (B + WAVES - 1) / WAVES + (n_lab + 255) / 256 + 1;
  return nb * 3 * (int64_t)sizeof(float);
}

extern "C" int llp_llp_loss_heads(int64_t B, int64_t C, float* s_logit, float* t_prob, int64_t n_lab,
                                  int64_t n_pos, float* out_logit, double B_total, double n_lab_total, float margin,
                                  float T, float w_label, float w_d, float w_r, float loss_scale, float* dlogit_ctx,
                                  float* dlogit_lab, float* terms_out, int accumulate, const int32_t* neg_count,
                                  int64_t neg_offset, double pos_total, int64_t term_b0, int64_t term_b1,
                                  const llp_head_parts* s_head, const llp_head_parts* t_head, uint32_t* ticket,
                                  void* workspace, int64_t workspace_bytes, void* stream) {
  LLP_CHECK_ARG(C <= MAXC, "llp_llp_loss: contexts per anchor C=%lld > %d", (long long)C, MAXC);
  LLP_CHECK_ARG(terms_out && workspace, "llp_llp_loss: null terms/workspace");
  LLP_CHECK_ARG(workspace_bytes >= llp_llp_loss_workspace_bytes(B, n_lab), "llp_llp_loss: workspace too small");
  LLP_CHECK_ARG(!s_head || (s_head->part && s_head->ld >= B * C + n_lab && s_head->parts >= 1),
                "llp_llp_loss: student head partials must cover the B*C + n_lab predictor rows");
  LLP_CHECK_ARG(!t_head || (t_head->part && t_head->ld >= B * C && t_head->parts >= 1),
                "llp_llp_loss: teacher head partials must cover the B*C context rows");
  hipStream_t s = (hipStream_t)stream;
  LossArgs a = {};
  a.B = B; a.C = C; a.n_lab = n_lab; a.n_pos = n_pos;
  a.nba = B > 0 ? (B + WAVES - 1) / WAVES : 0;
  a.nbl = (n_lab + 255) / 256;
  if (a.nba > 0) LLP_CHECK_ARG(s_logit && t_prob && dlogit_ctx, "llp_llp_loss: null context buffers");
  if (a.nbl > 0) LLP_CHECK_ARG(out_logit && dlogit_lab, "llp_llp_loss: null label buffers");
  a.s_logit = s_logit; a.t_prob = t_prob; a.out_logit = out_logit;
  if (s_head) a.hs = {s_head->part, s_head->bias, s_head->parts, s_head->ld};
  if (t_head) a.ht = {t_head->part, t_head->bias, t_head->parts, t_head->ld};
  a.lab_row0 = B * C;
  a.B_total = B_total; a.n_lab_total = n_lab_total; a.pos_total = pos_total;
  a.margin = margin; a.T = T; a.w_label = w_label; a.w_d = w_d; a.w_r = w_r; a.loss_scale = loss_scale;
  a.dlogit_ctx = dlogit_ctx; a.dlogit_lab = dlogit_lab;
  a.neg_count = neg_count; a.neg_offset = neg_offset;
  a.tb0 = term_b0; a.tb1 = term_b1;
  a.partial = reinterpret_cast<float*>(workspace);
  a.terms = terms_out; a.accumulate = accumulate;
  a.ticket = ticket;
  const int64_t nb = a.nba + a.nbl;
  if (nb > 0) {
    if (C <= 64) hipLaunchKernelGGL(llp_loss_kernel<64>, dim3((unsigned)nb), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(llp_loss_kernel<MAXC>, dim3((unsigned)nb), dim3(256), 0, s, a);
    LLP_LAUNCH_CHECK();
  }
  if (!ticket || nb == 0) {
    hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, s, a.partial, nb, w_label, w_d, w_r, terms_out,
                       accumulate);
    LLP_LAUNCH_CHECK();
  }
  return LLP_OK;
}

// the round-3 signature (every anchor's terms reported), kept for existing callers
extern "C" int llp_llp_loss(int64_t B, int64_t C, const float* s_logit, const float* t_prob, int64_t n_lab,
                            int64_t n_pos, const float* out_logit, double B_total, double n_lab_total, float margin,
                            float T, float w_label, float w_d, float w_r, float loss_scale, float* dlogit_ctx,
                            float* dlogit_lab, float* terms_out, int accumulate, const int32_t* neg_count,
                            int64_t neg_offset, double pos_total, void* workspace, int64_t workspace_bytes,
                            void* stream) {
  return llp_llp_loss_heads(B, C, const_cast<float*>(s_logit), const_cast<float*>(t_prob), n_lab, n_pos,
                            const_cast<float*>(out_logit), B_total, n_lab_total, margin, T, w_label, w_d, w_r,
                            loss_scale, dlogit_ctx, dlogit_lab, terms_out, accumulate, neg_count, neg_offset,
                            pos_total, 0, B, nullptr, nullptr, nullptr, workspace, workspace_bytes, stream);
}

extern "C" int llp_llp_loss_range(int64_t B, int64_t C, const float* s_logit, const float* t_prob, int64_t n_lab,
                                  int64_t n_pos, const float* out_logit, double B_total, double n_lab_total,
                                  float margin, float T, float w_label, float w_d, float w_r, float loss_scale,
                                  float* dlogit_ctx, float* dlogit_lab, float* terms_out, int accumulate,
                                  const int32_t* neg_count, int64_t neg_offset, double pos_total, int64_t term_b0,
                                  int64_t term_b1, void* workspace, int64_t workspace_bytes, void* stream) {
  return llp_llp_loss_heads(B, C, const_cast<float*>(s_logit), const_cast<float*>(t_prob), n_lab, n_pos,
                            const_cast<float*>(out_logit), B_total, n_lab_total, margin, T, w_label, w_d, w_r,
                            loss_scale, dlogit_ctx, dlogit_lab, terms_out, accumulate, neg_count, neg_offset,
                            pos_total, term_b0, term_b1, nullptr, nullptr, nullptr, workspace, workspace_bytes,
                            stream);
}

extern "C" int llp_head_fwd(int dtype, int64_t R, int64_t H, const void* Z, int64_t ldz, const void* Z2, int64_t ldz2,
                            const int32_t* iz, const int32_t* iz2, const float* w, const float* b, float* logit,
                            float* prob, void* stream) {
  LLP_CHECK_ARG(Z || R == 0, "llp_head_fwd: null Z");
  if (R == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(ceil_div_u(R, 4));
  if (dtype == LLP_BF16)
    hipLaunchKernelGGL(head_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, R, H, (const bf16_t*)Z, ldz,
                       (const bf16_t*)Z2, ldz2, iz, iz2, w, b, logit, prob);
  else
    hipLaunchKernelGGL(head_fwd_kernel<float>, grid, dim3(256), 0, s, R, H, (const float*)Z, ldz, (const float*)Z2,
                       ldz2, iz, iz2, w, b, logit, prob);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

static int64_t colsum_slabs(int64_t R) { return (R + colsum_rows(R) - 1) / colsum_rows(R); }

// workspace: a bound on colsum_slabs that grows with R (the slab count itself does not: 33,280
// rows take 260 blocks of 128, 32,768 take 512 of 64), so a workspace sized for the largest R a
// call site sees fits every smaller one
static int64_t colsum_slabs_bound(int64_t R) {
  const int64_t lo = std::min<int64_t>(512, (R + 63) / 64), hi = (R + 511) / 512;
  return std::max(lo, hi);
}

extern "C" int64_t llp_head_bwd_workspace_bytes(int64_t R, int64_t H) {
  return colsum_slabs_bound(R) * (H + 1) * (int64_t)sizeof(float);
}
extern "C" int64_t llp_colsum_workspace_bytes(int64_t M, int64_t N) { return llp_head_bwd_workspace_bytes(M, N); }

static int colsum_launch(int dtype, int64_t R, int64_t H, const void* Z, int64_t ldz, const float* weight,
                         const float* w, int relu_mask, float alpha, void* dZ, int64_t lddz, float* dw, float* db,
                         int accumulate,
                         void* workspace, int64_t workspace_bytes, hipStream_t s, const int32_t* r_dev = nullptr) {
  LLP_CHECK_ARG(workspace_bytes >= llp_head_bwd_workspace_bytes(R, H), "colsum: workspace too small");
  const int64_t ns = colsum_slabs(R);
  float* slab = reinterpret_cast<float*>(workspace);
  float* slab_b = slab + ns * H;
  if (ns > 0) {
    const int ch = dtype == LLP_BF16 ? 8 : 4;
    const int es = dtype == LLP_BF16 ? 2 : 4;
    const bool vec = (H % ch == 0) && (H / ch <= 256) && ((uintptr_t)Z % 16 == 0) && ((ldz * es) % 16 == 0) &&
                     (!dZ || (((uintptr_t)dZ % 16 == 0) && ((lddz * es) % 16 == 0)));
    if (dtype == LLP_BF16) {
      if (vec) {
        auto* kern = weight ? colsum_vec_kernel<bf16_t, true> : colsum_vec_kernel<bf16_t, false>;
        hipLaunchKernelGGL(kern, dim3((unsigned)ns), dim3(256), 0, s, R, H, (const bf16_t*)Z, ldz, weight, w, relu_mask,
                           alpha, (bf16_t*)dZ, lddz, slab, db ? slab_b : nullptr, r_dev);
      } else
        hipLaunchKernelGGL(colsum_kernel<bf16_t>, dim3((unsigned)ns), dim3(256), 0, s, R, H, (const bf16_t*)Z, ldz,
                           weight, w, relu_mask, alpha, (bf16_t*)dZ, lddz, slab, db ? slab_b : nullptr, r_dev);
    } else {
      if (vec) {
        auto* kern = weight ? colsum_vec_kernel<float, true> : colsum_vec_kernel<float, false>;
        hipLaunchKernelGGL(kern, dim3((unsigned)ns), dim3(256), 0, s, R, H, (const float*)Z, ldz, weight, w, relu_mask,
                           alpha, (float*)dZ, lddz, slab, db ? slab_b : nullptr, r_dev);
      } else
        hipLaunchKernelGGL(colsum_kernel<float>, dim3((unsigned)ns), dim3(256), 0, s, R, H, (const float*)Z, ldz,
                           weight, w, relu_mask, alpha, (float*)dZ, lddz, slab, db ? slab_b : nullptr, r_dev);
    }
    LLP_LAUNCH_CHECK();
  }
  if (dw || db) {   // the dw columns and the db scalar in one launch
    const SumJob jw{slab, ns, H, dw}, jb{slab_b, ns, (int64_t)1, db};
    const int64_t nbw = dw ? ceil_div_u(H, H >= SUM_CB ? SUM_CB : 1) : 0;
    hipLaunchKernelGGL(slab_sum_kernel, dim3((unsigned)(nbw + (db ? 1 : 0))), dim3(256), 0, s, dw ? jw : jb, jb,
                       nbw > 0 ? nbw : (int64_t)1, accumulate);
    LLP_LAUNCH_CHECK();
  }
  return LLP_OK;
}

extern "C" int llp_head_bwd(int dtype, int64_t R, int64_t H, const float* dlogit, const void* Z, int64_t ldz,
                            const float* w, int relu_mask, float alpha, void* dZ, int64_t lddz, float* dw,
                            float* db, int accumulate, void* workspace, int64_t workspace_bytes, void* stream) {
  LLP_CHECK_ARG(R == 0 || (dlogit && Z), "llp_head_bwd: null input");   // R = 0: dw, db = the empty sum
  LLP_CHECK_ARG(!dZ || w, "llp_head_bwd: dZ needs w");
  return colsum_launch(dtype, R, H, Z, ldz, dlogit, w, relu_mask, alpha, dZ, lddz, dw, db, accumulate, workspace,
                       workspace_bytes, (hipStream_t)stream);
}

extern "C" int llp_colsum(int dtype, int64_t M, int64_t N, const void* Y, int64_t ldy, float* out, int accumulate,
                          void* workspace, int64_t workspace_bytes, void* stream) {
  LLP_CHECK_ARG(out && (Y || M == 0), "llp_colsum: null input");   // M = 0: out = the empty sum
  return colsum_launch(dtype, M, N, Y, ldy, nullptr, nullptr, 0, 1.f, nullptr, 0, out, nullptr, accumulate, workspace,
                       workspace_bytes, (hipStream_t)stream);
}

// llp_colsum over min(M, *m_dev) live rows (grid sized by M): the bias
// gradient of a GEMM whose row count is device-resident (gemm.hip).
namespace llp {
int colsum_rows_dev(int dtype, int64_t M, int64_t N, const void* Y, int64_t ldy, float* out, int accumulate,
                    void* workspace, int64_t workspace_bytes, const int32_t* m_dev, void* stream) {
  LLP_CHECK_ARG(out && (Y || M == 0), "llp_colsum: null input");   // M = 0: out = the empty sum
  return colsum_launch(dtype, M, N, Y, ldy, nullptr, nullptr, 0, 1.f, nullptr, 0, out, nullptr, accumulate, workspace,
                       workspace_bytes, (hipStream_t)stream, m_dev);
}
}  // namespace llp
