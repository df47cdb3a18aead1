// Device-side samplers and per-step index builders.
//
// The reference samples on the host: torch_cluster random_walk on CPU for the
// minibatch path (src/main.py:93 -> :33-50, then .to("cuda") at :50) and
// torch.randint (src/main.py:47,84).  Here everything is drawn on the GPU from
// a counter-based Philox stream keyed by a DEVICE step counter, so a captured
// hipGraph replays a fresh sample every step and no host sync is needed.  Draw
// indices are global (b + b_offset), so a rank holding a shard of the anchors
// draws exactly what one GPU would draw for those anchors.
#include "llp_common.h"

namespace {

// One thread per (anchor, walk).  Walk semantics: torch_cluster random_walk,
// p = q = 1: next = col[rowptr[cur] + floor(u * deg(cur))]; deg 0 -> stay.
__global__ void context_walk_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                    const int32_t* __restrict__ start, int64_t B, int64_t b_offset, int n_walks,
                                    int walk_len, int ps_nb, int64_t C1, uint64_t seed,
                                    const int64_t* __restrict__ step_ctr, int64_t stream_offset,
                                    int32_t* __restrict__ samples) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= B * n_walks) return;
  const int64_t b = t % B;
  const int w = (int)(t / B);
  const uint64_t stream = (uint64_t)(LLP_STREAMS_PER_STEP * (*step_ctr) + stream_offset + w);
  const int64_t bg = b + b_offset;
  int32_t cur = start[b];
  int32_t* out = samples + b * C1;
  if (w == 0) out[0] = cur;
  // column of step l (1-based) of walk w: rw -> l ; nb -> w*hops + l
  const int64_t colbase = ps_nb ? (int64_t)w * walk_len : 0;
  for (int l = 0; l < walk_len; ++l) {
    const uint32_t x = philox_u32(seed, stream, (uint64_t)(bg * walk_len + l));
    const int32_t lo = rowptr[cur];
    const int32_t deg = rowptr[cur + 1] - lo;
    if (deg > 0) cur = col[lo + uniform_index(x, deg)];
    out[colbase + l + 1] = cur;
  }
}

__global__ void context_neg_kernel(int64_t B, int64_t b_offset, int64_t nneg, int64_t num_nodes, int64_t col0,
                                   int64_t C1, uint64_t seed, const int64_t* __restrict__ step_ctr,
                                   int64_t stream_rel, int32_t* __restrict__ samples) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= B * nneg) return;
  const uint64_t stream = (uint64_t)(LLP_STREAMS_PER_STEP * (*step_ctr) + stream_rel);
  const int64_t b = t / nneg, q = t % nneg;
  const uint32_t x = philox_u32(seed, stream, (uint64_t)((b + b_offset) * nneg + q));
  samples[b * C1 + col0 + q] = (int32_t)randint_index(x, num_nodes);
}

__global__ void randint_pairs_kernel(int64_t num_nodes, int64_t n, int64_t n_total, int64_t offset, uint64_t seed,
                                     const int64_t* __restrict__ step_ctr, int64_t stream_offset,
                                     int32_t* __restrict__ out) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= 2 * n) return;
  const uint64_t stream = (uint64_t)(LLP_STREAMS_PER_STEP * (*step_ctr) + stream_offset);
  const int64_t side = t / n, i = t % n;
  const uint64_t draw = (uint64_t)(side * n_total + offset + i);
  out[t] = (int32_t)randint_index(philox_u32(seed, stream, draw), num_nodes);
}

__global__ void build_targets_kernel(int64_t BC1, const int32_t* __restrict__ samples,
                                     const int32_t* __restrict__ pairs, const int32_t* __restrict__ perm,
                                     const int64_t* __restrict__ step_ctr, int64_t perm_stride, int64_t P,
                                     const int32_t* __restrict__ neg, int64_t n_neg, int64_t ld_neg,
                                     int32_t* __restrict__ target) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t n_lab = P + n_neg;     // train_edges columns (main.py:86)
  const int64_t total = BC1 + 2 * n_lab;
  if (t >= total) return;
  if (t < BC1) {
    target[t] = samples[t];
    return;
  }
  const int64_t u = t - BC1;           // [0, 2 n_lab): src(n_lab) then dst(n_lab)
  const int64_t side = u / n_lab;      // 0 = src (train_edges[0]), 1 = dst
  const int64_t i = u % n_lab;
  int32_t v;
  if (i < P) {
    const int64_t e = perm[(step_ctr ? *step_ctr : 0) * perm_stride + i];
    v = pairs[2 * e + side];           // pos_train_edge[link_perm].t() (main.py:78)
  } else {
    v = neg[side * ld_neg + (i - P)];  // neg_edge[side] (main.py:81-84)
  }
  target[t] = v;
}

__global__ void pair_index_kernel(int64_t B, int64_t C, const int32_t* __restrict__ samples,
                                  int32_t* __restrict__ ia, int32_t* __restrict__ ib) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= B * C) return;
  const int64_t b = t / C, c = t % C;
  ia[t] = samples[b * (C + 1)];
  ib[t] = samples[b * (C + 1) + 1 + c];
}

// All of one minibatch step's index building in one launch (the collab path: device
// walks + randint negatives): the thread ranges do exactly what context_walk_kernel,
// context_neg_kernel, randint_pairs_kernel, build_targets_kernel and pair_index_kernel
// do, with the same Philox draws, and each writes every array slot its value lands in
// (samples, target, the teacher's pair index) instead of a later kernel copying it.
struct MbSample {
  const int32_t* rowptr; const int32_t* col; int64_t num_nodes;
  const int32_t* start; int64_t B, b_offset; int n_walks, walk_len, ps_nb, rw_step; int64_t nneg, C, C1;
  uint64_t seed; const int64_t* step_ctr; int64_t stream_offset;
  const int32_t* pairs; const int32_t* perm; int64_t P, P_total, p_offset, neg_stream;
  int32_t* samples; int32_t* neg; int32_t* target; int32_t* t_ia; int32_t* t_ib;
};

__global__ void minibatch_sample_kernel(MbSample a) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t nw = a.B * a.n_walks, nn = a.B * a.nneg, BC1 = a.B * a.C1, n_lab = 2 * a.P;
  const int64_t step = *a.step_ctr;
  if (t < nw) {   // walk w of anchor b (context_walk_kernel)
    const int64_t b = t % a.B;
    const int w = (int)(t / a.B);
    const uint64_t stream = (uint64_t)(LLP_STREAMS_PER_STEP * step + a.stream_offset + w);
    const int64_t bg = b + a.b_offset;
    const int32_t anchor = a.start[b];
    int32_t cur = anchor;
    if (w == 0) { a.samples[b * a.C1] = anchor; a.target[b * a.C1] = anchor; }
    const int64_t colbase = a.ps_nb ? (int64_t)w * a.walk_len : 0;
    for (int l = 0; l < a.walk_len; ++l) {
      const uint32_t x = philox_u32(a.seed, stream, (uint64_t)(bg * a.walk_len + l));
      const int32_t lo = a.rowptr[cur];
      const int32_t deg = a.rowptr[cur + 1] - lo;
      if (deg > 0) cur = a.col[lo + uniform_index(x, deg)];
      const int64_t c = colbase + l;          // context column c + 1 of row b
      a.samples[b * a.C1 + c + 1] = cur;
      a.target[b * a.C1 + c + 1] = cur;
      if (a.t_ia) {
        a.t_ia[b * a.C + c] = anchor;
        a.t_ib[b * a.C + c] = cur;
      }
    }
    return;
  }
  int64_t u = t - nw;
  if (u < nn) {   // context negative q of anchor b (context_neg_kernel)
    const uint64_t stream = (uint64_t)(LLP_STREAMS_PER_STEP * step + a.stream_offset + a.rw_step);
    const int64_t b = u / a.nneg, q = u % a.nneg;
    const uint32_t x = philox_u32(a.seed, stream, (uint64_t)((b + a.b_offset) * a.nneg + q));
    const int32_t v = (int32_t)randint_index(x, a.num_nodes);
    const int64_t c = a.C - a.nneg + q;       // negatives follow the walk columns
    a.samples[b * a.C1 + c + 1] = v;
    a.target[b * a.C1 + c + 1] = v;
    if (a.t_ia) {
      a.t_ia[b * a.C + c] = a.start[b];
      a.t_ib[b * a.C + c] = v;
    }
    return;
  }
  u -= nn;
  if (u < 2 * a.P) {   // label negative (randint_pairs_kernel) -> neg[side][i], target
    const uint64_t stream = (uint64_t)(LLP_STREAMS_PER_STEP * step + a.neg_stream);
    const int64_t side = u / a.P, i = u % a.P;
    const uint64_t draw = (uint64_t)(side * a.P_total + a.p_offset + i);
    const int32_t v = (int32_t)randint_index(philox_u32(a.seed, stream, draw), a.num_nodes);
    a.neg[u] = v;
    a.target[BC1 + side * n_lab + a.P + i] = v;
    return;
  }
  u -= 2 * a.P;
  if (u < 2 * a.P) {   // label positive pos_train_edge[link_perm] (build_targets_kernel)
    const int64_t side = u / a.P, i = u % a.P;
    a.target[BC1 + side * n_lab + i] = a.pairs[2 * (int64_t)a.perm[i] + side];
  }
}

// The j-th batch of an epoch's permutations, j = (*step_ctr + ctr_offset) mod n_batches
// (llp_batch_slices): thread i < n_a copies perm_a[j stride_a + off_a + i], thread i < n_b perm_b's.
__global__ void batch_slices_kernel(const int32_t* __restrict__ pa, int64_t sa, int64_t oa, int64_t na,
                                    const int32_t* __restrict__ pb, int64_t sb, int64_t ob, int64_t nb,
                                    int64_t n_batches, const int64_t* __restrict__ step_ctr, int64_t ctr_offset,
                                    int32_t* __restrict__ out_a, int32_t* __restrict__ out_b) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  int64_t j = (*step_ctr + ctr_offset) % n_batches;
  j = j < 0 ? j + n_batches : j;
  if (i < na) out_a[i] = pa[j * sa + oa + i];
  if (i < nb) out_b[i] = pb[j * sb + ob + i];
}

}  // namespace

extern "C" int llp_minibatch_sample(const int32_t* rowptr, const int32_t* col, int64_t num_nodes,
                                    const int32_t* start, int64_t B, int64_t b_offset, int ps_method, int rw_step,
                                    int hops, int ns_rate, uint64_t seed, const int64_t* step_ctr,
                                    int64_t stream_offset, const int32_t* pairs, const int32_t* perm, int64_t P,
                                    int64_t P_total, int64_t p_offset, int64_t neg_stream_offset, int32_t* samples,
                                    int32_t* neg, int32_t* target, int32_t* t_ia, int32_t* t_ib, void* stream) {
  LLP_CHECK_ARG(rowptr && col && start && samples && step_ctr && target && (!t_ia == !t_ib) &&
                    (P == 0 || (pairs && perm && neg)),
                "llp_minibatch_sample: null pointer");
  LLP_CHECK_ARG(ps_method == 0 || ps_method == 1, "llp_minibatch_sample: ps_method must be 0 (rw) or 1 (nb)");
  // walks take streams 0 .. rw_step-1 of a step and the negatives stream rw_step, below the
  // PyG-dense (S-2) and randint (S-1) negatives
  LLP_CHECK_ARG(rw_step >= 1 && hops >= 1 && ns_rate >= 0 && rw_step <= LLP_STREAMS_PER_STEP - 3,
                "llp_minibatch_sample: rw_step %d (1..%d), hops %d, ns_rate %d", rw_step, (int)(LLP_STREAMS_PER_STEP - 3),
                hops, ns_rate);
  LLP_CHECK_ARG(p_offset + P <= P_total, "llp_minibatch_sample: shard out of range");
  MbSample a;
  a.rowptr = rowptr; a.col = col; a.num_nodes = num_nodes; a.start = start; a.B = B; a.b_offset = b_offset;
  a.n_walks = ps_method == 1 ? rw_step : 1;
  a.walk_len = ps_method == 1 ? hops : rw_step * hops;
  a.ps_nb = ps_method;
  a.rw_step = rw_step;
  a.nneg = (int64_t)rw_step * hops * ns_rate;
  a.C = (int64_t)rw_step * hops * (1 + ns_rate);
  a.C1 = a.C + 1;
  a.seed = seed; a.step_ctr = step_ctr; a.stream_offset = stream_offset;
  a.pairs = pairs; a.perm = perm; a.P = P; a.P_total = P_total; a.p_offset = p_offset;
  a.neg_stream = neg_stream_offset;
  a.samples = samples; a.neg = neg; a.target = target; a.t_ia = t_ia; a.t_ib = t_ib;
  const int64_t total = B * a.n_walks + B * a.nneg + 4 * P;
  if (total == 0) return LLP_OK;
  hipLaunchKernelGGL(minibatch_sample_kernel, dim3(ceil_div_u(total, 256)), dim3(256), 0, (hipStream_t)stream, a);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_context_sampler(const int32_t* rowptr, const int32_t* col, int64_t num_nodes,
                                   const int32_t* start, int64_t B, int64_t b_offset, int ps_method, int rw_step,
                                   int hops, int ns_rate, uint64_t seed, const int64_t* step_ctr,
                                   int64_t stream_offset, int32_t* samples, void* stream) {
  LLP_CHECK_ARG((B == 0) || (rowptr && col && start && samples && step_ctr), "llp_context_sampler: null pointer");
  LLP_CHECK_ARG(ps_method == 0 || ps_method == 1, "llp_context_sampler: ps_method must be 0 (rw) or 1 (nb)");
  // walks take streams 0 .. rw_step-1 of a step and the negatives stream rw_step, below the
  // PyG-dense (S-2) and randint (S-1) negatives
  LLP_CHECK_ARG(rw_step >= 1 && hops >= 1 && ns_rate >= 0 && rw_step <= LLP_STREAMS_PER_STEP - 3,
                "llp_context_sampler: rw_step %d (1..%d), hops %d, ns_rate %d", rw_step, (int)(LLP_STREAMS_PER_STEP - 3),
                hops, ns_rate);
  if (B == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  const int64_t C1 = 1 + (int64_t)rw_step * hops * (1 + ns_rate);
  const int n_walks = ps_method == 1 ? rw_step : 1;
  const int walk_len = ps_method == 1 ? hops : rw_step * hops;
  const int64_t nt = B * n_walks;
  hipLaunchKernelGGL(context_walk_kernel, dim3(ceil_div_u(nt, 256)), dim3(256), 0, s, rowptr, col, start, B, b_offset,
                     n_walks, walk_len, ps_method, C1, seed, step_ctr, stream_offset, samples);
  LLP_LAUNCH_CHECK();
  const int64_t nneg = (int64_t)rw_step * hops * ns_rate;
  if (nneg > 0) {
    hipLaunchKernelGGL(context_neg_kernel, dim3(ceil_div_u(B * nneg, 256)), dim3(256), 0, s, B, b_offset, nneg,
                       num_nodes, 1 + (int64_t)rw_step * hops, C1, seed, step_ctr, stream_offset + rw_step, samples);
    LLP_LAUNCH_CHECK();
  }
  return LLP_OK;
}

extern "C" int llp_randint_pairs(int64_t num_nodes, int64_t n, int64_t n_total, int64_t offset, uint64_t seed,
                                 const int64_t* step_ctr, int64_t stream_offset, int32_t* out, void* stream) {
  LLP_CHECK_ARG((n == 0) || (out && step_ctr), "llp_randint_pairs: null pointer");
  LLP_CHECK_ARG(offset + n <= n_total, "llp_randint_pairs: shard out of range");
  if (n == 0) return LLP_OK;
  hipLaunchKernelGGL(randint_pairs_kernel, dim3(ceil_div_u(2 * n, 256)), dim3(256), 0, (hipStream_t)stream,
                     num_nodes, n, n_total, offset, seed, step_ctr, stream_offset, out);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_build_targets(int64_t B, int64_t C1, const int32_t* samples, const int32_t* pairs,
                                 const int32_t* perm, const int64_t* step_ctr, int64_t perm_stride, int64_t P,
                                 const int32_t* neg, int64_t n_neg, int64_t ld_neg, int32_t* target, void* stream) {
  LLP_CHECK_ARG(samples && pairs && perm && target && (neg || n_neg == 0), "llp_build_targets: null pointer");
  LLP_CHECK_ARG(n_neg >= 0 && ld_neg >= n_neg, "llp_build_targets: bad negative layout");
  const int64_t total = B * C1 + 2 * (P + n_neg);
  if (total == 0) return LLP_OK;
  hipLaunchKernelGGL(build_targets_kernel, dim3(ceil_div_u(total, 256)), dim3(256), 0, (hipStream_t)stream,
                     B * C1, samples, pairs, perm, step_ctr, perm_stride, P, neg, n_neg, ld_neg, target);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_pair_index_from_samples(int64_t B, int64_t C, const int32_t* samples, int32_t* ia, int32_t* ib,
                                           void* stream) {
  LLP_CHECK_ARG((B * C == 0) || (samples && ia && ib), "llp_pair_index_from_samples: null pointer");
  if (B * C == 0) return LLP_OK;
  hipLaunchKernelGGL(pair_index_kernel, dim3(ceil_div_u(B * C, 256)), dim3(256), 0, (hipStream_t)stream, B, C,
                     samples, ia, ib);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_batch_slices(const int32_t* perm_a, int64_t stride_a, int64_t off_a, int64_t n_a,
                                const int32_t* perm_b, int64_t stride_b, int64_t off_b, int64_t n_b,
                                int64_t n_batches, int64_t len_a, int64_t len_b, const int64_t* step_ctr,
                                int64_t ctr_offset, int32_t* out_a, int32_t* out_b, void* stream) {
  LLP_CHECK_ARG(n_a >= 0 && n_b >= 0 && n_batches >= 1, "llp_batch_slices: bad sizes");
  LLP_CHECK_ARG(step_ctr && (n_a == 0 || (perm_a && out_a)) && (n_b == 0 || (perm_b && out_b)),
                "llp_batch_slices: null pointer");
  // every batch j < n_batches must lie inside its permutation (len_a / len_b elements)
  LLP_CHECK_ARG(n_a == 0 || (off_a >= 0 && stride_a >= 0 && (n_batches - 1) * stride_a + off_a + n_a <= len_a),
                "llp_batch_slices: slice a past its permutation");
  LLP_CHECK_ARG(n_b == 0 || (off_b >= 0 && stride_b >= 0 && (n_batches - 1) * stride_b + off_b + n_b <= len_b),
                "llp_batch_slices: slice b past its permutation");
  const int64_t n = n_a > n_b ? n_a : n_b;
  if (n == 0) return LLP_OK;
  hipLaunchKernelGGL(batch_slices_kernel, dim3(ceil_div_u(n, 256)), dim3(256), 0, (hipStream_t)stream, perm_a,
                     stride_a, off_a, n_a, perm_b, stride_b, off_b, n_b, n_batches, step_ctr, ctr_offset, out_a, out_b);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}
