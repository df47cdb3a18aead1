// Owner decomposition of a multi-rank minibatch step (train_minibatch, src/main.py:86-130,
// sharded over ranks).
//
// The reference step is single-GPU.  Its N-rank form here gives every predictor pair to
// one rank: a context pair (anchor b, context c) to the owner of the context node, a label
// pair to the owner of its source node (owner = owner_tab[node], a locality order's contiguous
// ranges, or node / ceil(N / world)), balanced so that
// rank r receives exactly cap_r = (r+1)n/W - rn/W pairs of each category: an owner keeps
// its first cap pairs in item order, and the owners' overflow, ordered by (owner, rank in
// the owner's list), fills the ranks' free positions in rank order.  A rank then runs the
// student only on the unique endpoints of its pairs (the i.i.d. context negatives are
// computed where they live, not once per anchor shard).  oracle/llp_oracle.py
// pair_owner_assign is the same rule; the assignment is integer work and bit-exact.
//
// Three launches for up to three categories (context, positive, negative pairs):
//   owner_hist_kernel    per 1,024-item block: items per owner (hist[owner][block])
//   owner_scan_kernel    one block, a wave per (category, owner): per-block offsets, then the
//                        caps, overflow and free-position bases
//   owner_place_kernel   per item: (rank, position) -> sel / gpos, and this rank's pairs'
//                        node ids into target = [ia | ib] (the student's rows)
// Every thread loads its items' ends up front (four loads in flight), so a block is one
// memory latency plus its ranking passes (collab, 603k items on 8 ranks: the round-4 first
// version with 4,096-item blocks and one pass after another took 75 us for the three).
#include "llp_common.h"

namespace {

constexpr int OW_T = 256;
constexpr int OW_PASS = 4;                        // passes of 256 items per block
constexpr int OW_ITEMS = OW_T * OW_PASS;          // items per block
constexpr int OW_MAXW = 64;

struct Cat {
  // node id of item i's ends: base[(i / kc) * kld + koff + (i % kc) * kstep]
  const int32_t* a; int64_t a_kc, a_kld, a_koff, a_kstep;
  const int32_t* b; int64_t b_kc, b_kld, b_koff, b_kstep;
  int key_b;          // the key (owner) node is the b end (context pairs), else the a end
  int64_t n;          // items
  int64_t blk0;       // first block of this category
  int64_t sel0;       // first slot of this category in sel / its items' gpos base
  int64_t row0;       // first row of this category in this rank's pair list
};

struct OwnerArgs {
  Cat c[3];
  int ncat;
  int64_t nblk;
  int64_t num_nodes, n_loc;
  int world, rank;
  const int32_t* owner_tab;   // node -> owner rank, or NULL: node / ceil(N / world)
  int64_t R2;                 // this rank's pairs (all categories): target = [ia (R2) | ib (R2)]
  int32_t* hist;              // [world][nblk] items per owner and block, then exclusive offsets (in place)
  int64_t* meta;              // [3][OW_MAXW][4]: cap, kept, overflow base, free base
  int32_t* sel;               // [sum n]: rank r's items of category c at sel[sel0 + off_r ...]
  int32_t* gpos;              // [sum n] or NULL: item -> its slot in sel (minus sel0)
  int32_t* target;            // [2 R2] or NULL
};

__device__ __forceinline__ int32_t node_at(const int32_t* base, int64_t kc, int64_t kld, int64_t koff, int64_t kstep,
                                           int64_t i) {
  const int64_t q = i / kc;
  return base[q * kld + koff + (i - q * kc) * kstep];
}

__device__ __forceinline__ int owner_of(const OwnerArgs& a, int32_t v) {
  const int64_t o = v < 0 ? 0 : (a.owner_tab ? (int64_t)a.owner_tab[v] : (int64_t)v / a.n_loc);
  return (int)(o < a.world ? o : a.world - 1);
}

__device__ __forceinline__ int cat_of_block(const OwnerArgs& a, int64_t blk) {
  int c = 0;
  while (c + 1 < a.ncat && blk >= a.c[c + 1].blk0) ++c;
  return c;
}

__global__ __launch_bounds__(OW_T) void owner_hist_kernel(OwnerArgs a) {
  __shared__ int32_t cnt[OW_MAXW];
  const int64_t blk = blockIdx.x;
  const Cat& c = a.c[cat_of_block(a, blk)];
  if (threadIdx.x < a.world) cnt[threadIdx.x] = 0;
  const int64_t i0 = (blk - c.blk0) * OW_ITEMS;
  int32_t v[OW_PASS];
#pragma unroll
  for (int p = 0; p < OW_PASS; ++p) {   // all loads first
    const int64_t i = i0 + p * OW_T + threadIdx.x;
    v[p] = i < c.n ? (c.key_b ? node_at(c.b, c.b_kc, c.b_kld, c.b_koff, c.b_kstep, i)
                              : node_at(c.a, c.a_kc, c.a_kld, c.a_koff, c.a_kstep, i))
                   : -1;
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < OW_PASS; ++p)
    if (i0 + p * OW_T + threadIdx.x < c.n) atomicAdd(&cnt[owner_of(a, v[p])], 1);
  __syncthreads();
  if (threadIdx.x < a.world) a.hist[threadIdx.x * a.nblk + blk] = cnt[threadIdx.x];
}

// one block of 1024 threads, one wave per (category, owner) sequence of per-block counts: an
// exclusive scan in place (256 counts per round, four per lane), then thread 0 derives the
// balancing bases from the totals
__global__ __launch_bounds__(1024) void owner_scan_kernel(OwnerArgs a) {
  __shared__ int64_t tot[3][OW_MAXW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int npair = a.ncat * a.world;
  for (int q = wv; q < npair; q += 16) {
    const int ci = q / a.world, o = q % a.world;
    const Cat& c = a.c[ci];
    const int64_t nb = (c.n + OW_ITEMS - 1) / OW_ITEMS;
    int32_t* h = a.hist + (int64_t)o * a.nblk + c.blk0;
    int64_t carry = 0;
    for (int64_t j0 = 0; j0 < nb; j0 += 256) {
      int32_t x[4];
      int32_t s = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t j = j0 + 4 * lane + k;
        x[k] = j < nb ? h[j] : 0;
        s += x[k];
      }
      int32_t inc = s;   // inclusive scan of the lanes' sums
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int32_t y = __shfl_up(inc, d, 64);
        if (lane >= d) inc += y;
      }
      int64_t run = carry + inc - s;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t j = j0 + 4 * lane + k;
        if (j < nb) h[j] = (int32_t)run;
        run += x[k];
      }
      carry += __shfl(inc, 63, 64);
    }
    if (lane == 0) tot[ci][o] = carry;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int ci = 0; ci < a.ncat; ++ci) {
      const int64_t n = a.c[ci].n, W = a.world;
      int64_t ov = 0, fr = 0;
      for (int o = 0; o < a.world; ++o) {
        const int64_t cap = (o + 1) * n / W - o * n / W;
        const int64_t kept = tot[ci][o] < cap ? tot[ci][o] : cap;
        int64_t* m = a.meta + ((int64_t)ci * OW_MAXW + o) * 4;
        m[0] = cap; m[1] = kept; m[2] = ov; m[3] = fr;
        ov += tot[ci][o] - kept;
        fr += cap - kept;
      }
    }
  }
}

__global__ __launch_bounds__(OW_T) void owner_place_kernel(OwnerArgs a) {
  __shared__ int32_t base[OW_MAXW];       // this block's running offset per owner
  __shared__ int32_t wcnt[OW_T / 64][OW_MAXW];
  __shared__ int64_t meta[OW_MAXW][4];
  const int64_t blk = blockIdx.x;
  const int ci = cat_of_block(a, blk);
  const Cat& c = a.c[ci];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int W = a.world;
  const int64_t i0 = (blk - c.blk0) * OW_ITEMS;
  int32_t va[OW_PASS], vb[OW_PASS];
#pragma unroll
  for (int p = 0; p < OW_PASS; ++p) {   // all loads first
    const int64_t i = i0 + p * OW_T + t;
    const bool live = i < c.n;
    va[p] = live ? node_at(c.a, c.a_kc, c.a_kld, c.a_koff, c.a_kstep, i) : 0;
    vb[p] = live ? node_at(c.b, c.b_kc, c.b_kld, c.b_koff, c.b_kstep, i) : 0;
  }
  if (t < W) {
    base[t] = a.hist[(int64_t)t * a.nblk + blk];
#pragma unroll
    for (int k = 0; k < 4; ++k) meta[t][k] = a.meta[((int64_t)ci * OW_MAXW + t) * 4 + k];
  }
  __syncthreads();
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int p = 0; p < OW_PASS; ++p) {
    const int64_t i = i0 + p * OW_T + t;
    const bool live = i < c.n;
    const int o = live ? owner_of(a, c.key_b ? vb[p] : va[p]) : -1;
    // rank among this pass's items of the same owner: lanes below in the wave, then earlier waves
    int in_wave = 0;
    for (int q = 0; q < W; ++q) {
      const uint64_t m = __ballot(o == q);
      if (o == q) in_wave = __popcll(m & below);
      if (lane == 0) wcnt[w][q] = __popcll(m);
    }
    __syncthreads();
    if (live) {
      int g = base[o] + in_wave;
      for (int k = 0; k < w; ++k) g += wcnt[k][o];
      const int64_t cap = meta[o][0];
      int r;
      int64_t pos;
      if (g < cap) {
        r = o;
        pos = g;
      } else {
        const int64_t j = meta[o][2] + g - cap;     // overflow index
        r = 0;
        while (r + 1 < W && meta[r + 1][3] <= j) ++r;
        pos = meta[r][1] + j - meta[r][3];
      }
      const int64_t off = (int64_t)r * c.n / W;
      a.sel[c.sel0 + off + pos] = (int32_t)i;
      if (a.gpos) a.gpos[c.sel0 + i] = (int32_t)(off + pos);
      if (a.target && r == a.rank) {
        const int64_t k = c.row0 + pos;
        a.target[k] = va[p];
        a.target[a.R2 + k] = vb[p];
      }
    }
    __syncthreads();
    if (t < W) {
      int s = 0;
      for (int k = 0; k < OW_T / 64; ++k) s += wcnt[k][t];
      base[t] += s;
    }
    __syncthreads();
  }
}

// S_full[i] = logit of slot i when this rank holds it (its gpos in [lo, hi)), else 0; the same
// for T_full (either may be NULL)
__global__ void owner_scatter_kernel(int64_t n, const int32_t* __restrict__ gpos, int64_t lo, int64_t hi,
                                     const float* __restrict__ s_loc, const float* __restrict__ t_loc,
                                     float* __restrict__ s_full, float* __restrict__ t_full) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t g = gpos[i];
  const bool mine = g >= lo && g < hi;
  if (s_full) s_full[i] = mine ? s_loc[g - lo] : 0.f;
  if (t_full) t_full[i] = mine ? t_loc[g - lo] : 0.f;
}

}  // namespace

extern "C" int64_t llp_pair_owner_workspace_bytes(int64_t n0, int64_t n1, int64_t n2, int world) {
  const int64_t nb = (n0 + OW_ITEMS - 1) / OW_ITEMS + (n1 + OW_ITEMS - 1) / OW_ITEMS + (n2 + OW_ITEMS - 1) / OW_ITEMS;
  return (int64_t)3 * OW_MAXW * 4 * (int64_t)sizeof(int64_t) + nb * (int64_t)(world > 0 ? world : 1) * 4 + 64;
}

extern "C" int llp_pair_owner_assign(int ncat, const llp_owner_cat* cats, int64_t num_nodes, int world, int rank,
                                     const int32_t* owner_tab, int32_t* sel, int32_t* gpos, int32_t* target,
                                     int64_t R2, void* workspace, int64_t workspace_bytes, void* stream) {
  LLP_CHECK_ARG(ncat >= 1 && ncat <= 3 && cats, "llp_pair_owner_assign: 1..3 categories");
  LLP_CHECK_ARG(world >= 1 && world <= OW_MAXW && rank >= 0 && rank < world,
                "llp_pair_owner_assign: world %d (1..%d), rank %d", world, OW_MAXW, rank);
  LLP_CHECK_ARG(num_nodes > 0 && sel && workspace, "llp_pair_owner_assign: null sel / workspace or no nodes");
  OwnerArgs a = {};
  a.ncat = ncat;
  a.num_nodes = num_nodes;
  a.n_loc = (num_nodes + world - 1) / world;
  a.world = world;
  a.rank = rank;
  a.owner_tab = owner_tab;
  a.R2 = R2;
  int64_t blk = 0, sel0 = 0, row0 = 0, n[3] = {0, 0, 0};
  for (int i = 0; i < ncat; ++i) {
    const llp_owner_cat& s = cats[i];
    LLP_CHECK_ARG(s.n >= 0 && (s.n == 0 || (s.a && s.b && s.a_kc > 0 && s.b_kc > 0)),
                  "llp_pair_owner_assign: category %d: null ends or bad stride", i);
    LLP_CHECK_ARG(s.n < (1ll << 31), "llp_pair_owner_assign: category %d too large", i);
    Cat& c = a.c[i];
    c.a = s.a; c.a_kc = s.a_kc; c.a_kld = s.a_kld; c.a_koff = s.a_koff; c.a_kstep = s.a_kstep;
    c.b = s.b; c.b_kc = s.b_kc; c.b_kld = s.b_kld; c.b_koff = s.b_koff; c.b_kstep = s.b_kstep;
    c.key_b = s.key_b;
    c.n = s.n;
    c.blk0 = blk;
    c.sel0 = sel0;
    c.row0 = row0;
    blk += (s.n + OW_ITEMS - 1) / OW_ITEMS;
    sel0 += s.n;
    row0 += (int64_t)(rank + 1) * s.n / world - (int64_t)rank * s.n / world;
    n[i] = s.n;
  }
  LLP_CHECK_ARG(!target || row0 == R2, "llp_pair_owner_assign: R2 %lld != this rank's pairs %lld", (long long)R2,
                (long long)row0);
  LLP_CHECK_ARG(workspace_bytes >= llp_pair_owner_workspace_bytes(n[0], n[1], n[2], world),
                "llp_pair_owner_assign: workspace too small");
  a.nblk = blk;
  a.meta = reinterpret_cast<int64_t*>(workspace);
  a.hist = reinterpret_cast<int32_t*>(a.meta + 3 * OW_MAXW * 4);
  a.sel = sel;
  a.gpos = gpos;
  a.target = target;
  if (blk == 0) return LLP_OK;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(owner_hist_kernel, dim3((unsigned)blk), dim3(OW_T), 0, s, a);
  LLP_LAUNCH_CHECK();
  hipLaunchKernelGGL(owner_scan_kernel, dim3(1), dim3(1024), 0, s, a);
  LLP_LAUNCH_CHECK();
  hipLaunchKernelGGL(owner_place_kernel, dim3((unsigned)blk), dim3(OW_T), 0, s, a);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_pair_owner_scatter(int64_t n, const int32_t* gpos, int64_t lo, int64_t hi, const float* s_loc,
                                      const float* t_loc, float* s_full, float* t_full, void* stream) {
  LLP_CHECK_ARG(n == 0 || gpos, "llp_pair_owner_scatter: null gpos");
  LLP_CHECK_ARG((!s_full || s_loc || hi == lo) && (!t_full || t_loc || hi == lo), "llp_pair_owner_scatter: null src");
  if (n == 0) return LLP_OK;
  hipLaunchKernelGGL(owner_scatter_kernel, dim3(ceil_div_u(n, 256)), dim3(256), 0, (hipStream_t)stream, n, gpos, lo,
                     hi, s_loc, t_loc, s_full, t_full);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}
