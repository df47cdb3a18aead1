// Shared device/host helpers for libllp_hip.so (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/llp_hip.h"

// ---------------------------------------------------------------- errors
namespace llp {
extern thread_local char g_err[512];
int set_error(int code, const char* fmt, ...);
// records (thread-local) the name of the NT GEMM kernel a launch chose: llp_last_gemm_kernel()
void note_kernel(const char* name);
// dropout code of p in (0, 1): the keep threshold and draw width (see drop_keep below)
inline uint32_t drop_code(float p) {
  const double s = (double)p * 256.0;
  if (s == (double)(int64_t)s) return 0x80000000u | (uint32_t)s;
  const double t = (double)p * 65536.0;
  const uint32_t ti = (uint32_t)t;
  return (double)ti == t ? ti : ti + 1u;   // ceil
}
}  // namespace llp

#define LLP_CHECK_ARG(cond, ...)                                        \
  do {                                                                  \
    if (!(cond)) return ::llp::set_error(LLP_E_ARG, __VA_ARGS__);       \
  } while (0)

#define LLP_LAUNCH_CHECK()                                                          \
  do {                                                                              \
    hipError_t _e = hipGetLastError();                                              \
    if (_e != hipSuccess)                                                           \
      return ::llp::set_error((int)_e, "%s: %s", __func__, hipGetErrorString(_e));  \
  } while (0)

// ---------------------------------------------------------------- types
typedef uint16_t bf16_t;  // raw bf16 bits in global memory

typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef float float4_t __attribute__((ext_vector_type(4)));
typedef float float16_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// round-to-nearest-even f32 -> bf16 (NaN-preserving via the hardware cvt at -O3)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&h);
}

// Philox streams per training step: a draw of step s at offset o uses stream
// LLP_STREAMS_PER_STEP * s + o (walks 0 .. rw_step-1, context negatives rw_step, PyG-dense
// negatives STREAMS-2 under their own key, randint negatives STREAMS-1; dropout layers 1 + l
// under per-module keys).  Must match oracle/llp_oracle.py:STREAMS_PER_STEP.
constexpr int64_t LLP_STREAMS_PER_STEP = 64;

// ---------------------------------------------------------------- Philox4x32-10
// Counter = (idx>>2 lo, idx>>2 hi, stream lo, stream hi), key = seed; word idx&3.
// Must match oracle/llp_oracle.py:philox_u32 bit for bit.
__device__ __forceinline__ void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                             uint32_t k0, uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
  const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
  c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
}

__device__ __forceinline__ uint4 philox4(uint64_t blk, uint64_t stream, uint64_t seed) {
  uint32_t c0 = (uint32_t)blk, c1 = (uint32_t)(blk >> 32);
  uint32_t c2 = (uint32_t)stream, c3 = (uint32_t)(stream >> 32);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c0, c1, c2, c3, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

__device__ __forceinline__ uint32_t philox_u32(uint64_t seed, uint64_t stream, uint64_t idx) {
  uint4 r = philox4(idx >> 2, stream, seed);
  switch (idx & 3) {
    case 0: return r.x;
    case 1: return r.y;
    case 2: return r.z;
    default: return r.w;
  }
}

// ---------------------------------------------------------------- dropout draws
// One Philox block serves 16 (8-bit draws) or 8 (16-bit draws) elements of a row, laid
// out so that the 256-tile GEMM epilogues' per-thread column sets (columns jn*16 + g*4 + r
// of a 64-column group, jn, r < 4) take one or two blocks per row instead of one per four
// elements (round 5: the teacher's dropout layers spent ~2/3 of their GEMM on Philox).
// The drop code (llp::drop_code) is thr | (1 << 31) with 8-bit draws (p * 256 an integer,
// e.g. 0.5: thr = p * 256 exactly), else ceil(p * 65536) with 16-bit draws; keep iff the
// draw >= thr.  Element (r, c) of a [rows, N] tensor, NG = ceil(N / 64), q = c >> 6,
// g = (c >> 2) & 3:
//   8-bit:  block (r NG + q) 4 + g,                        word (c >> 4) & 3,                      byte c & 3
//   16-bit: block ((r NG + q) 4 + g) 2 + ((c >> 5) & 1),  word ((c >> 4) & 1) 2 + ((c >> 1) & 1), half c & 1
// Must match oracle/llp_oracle.py:dropout_keep bit for bit.
constexpr uint32_t LLP_DROP_8BIT = 0x80000000u;
__device__ __forceinline__ uint64_t drop_group(int64_t r, int64_t c, int64_t N) {
  return (uint64_t)((r * ((N + 63) >> 6) + (c >> 6)) * 4 + ((c >> 2) & 3));
}
__device__ __forceinline__ uint32_t u4_word(const uint4& x, int w) {
  return w == 0 ? x.x : w == 1 ? x.y : w == 2 ? x.z : x.w;
}
__device__ __forceinline__ bool drop_keep(uint32_t code, uint64_t seed, uint64_t stream, int64_t r, int64_t c,
                                          int64_t N) {
  const uint64_t grp = drop_group(r, c, N);
  uint32_t u;
  if (code & LLP_DROP_8BIT) {
    u = (u4_word(philox4(grp, stream, seed), (int)((c >> 4) & 3)) >> (8 * (c & 3))) & 0xFFu;
  } else {
    const uint4 x = philox4(grp * 2 + ((c >> 5) & 1), stream, seed);
    u = (u4_word(x, (int)(((c >> 4) & 1) * 2 + ((c >> 1) & 1))) >> (16 * (c & 1))) & 0xFFFFu;
  }
  return u >= (code & ~LLP_DROP_8BIT);
}
// keep flags of the 16 elements (jn, r) at columns c0 + 16 jn + r of row r (c0 = a 64-column
// group's base + 4 g): bit 4 jn + r
__device__ __forceinline__ uint32_t drop_keep16(uint32_t code, uint64_t seed, uint64_t stream, int64_t row,
                                                int64_t c0, int64_t N) {
  const uint64_t grp = drop_group(row, c0, N);
  const uint32_t thr = code & ~LLP_DROP_8BIT;
  uint32_t bits = 0;
  if (code & LLP_DROP_8BIT) {
    const uint4 x = philox4(grp, stream, seed);
#pragma unroll
    for (int jn = 0; jn < 4; ++jn)
#pragma unroll
      for (int r = 0; r < 4; ++r) bits |= (((u4_word(x, jn) >> (8 * r)) & 0xFFu) >= thr ? 1u : 0u) << (4 * jn + r);
  } else {
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      const uint4 x = philox4(grp * 2 + jp, stream, seed);
#pragma unroll
      for (int j1 = 0; j1 < 2; ++j1)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          bits |= (((u4_word(x, j1 * 2 + (r >> 1)) >> (16 * (r & 1))) & 0xFFFFu) >= thr ? 1u : 0u)
                  << (4 * (2 * jp + j1) + r);
    }
  }
  return bits;
}

// floor(u*n), u = (x>>8)*2^-24, exact integer form (oracle: uniform_index)
__device__ __forceinline__ int64_t uniform_index(uint32_t x, int64_t n) {
  return (int64_t)((((uint64_t)(x >> 8)) * (uint64_t)n) >> 24);
}
// (x*n)>>32 (oracle: randint_index)
__device__ __forceinline__ int64_t randint_index(uint32_t x, int64_t n) {
  return (int64_t)(((uint64_t)x * (uint64_t)n) >> 32);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

static inline unsigned ceil_div_u(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

// Workgroups are dealt to the 8 XCDs round-robin (workgroup b runs on XCD b % 8): this bijection
// gives each XCD a contiguous range of logical blocks instead, so neighbouring work (rows of a
// locality-ordered graph) shares one XCD's L2 (cdna_hip_programming.md, XCD-aware mapping).
__device__ __forceinline__ int64_t llp_xcd_block(int64_t bid, int64_t nblocks) {
  if (nblocks < 8) return bid;
  const int64_t q = nblocks / 8, r = nblocks % 8;
  const int64_t xcd = bid % 8, loc = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// Hand-offs inside one launch (cdna_hip_programming.md Guideline 16, the write-through form): a
// word another workgroup of the launch reads is stored with llp_store_handed (an agent-scope
// atomic store: write-through, sc1) and read with llp_load_handed (an sc1 load), so no release
// or acquire fence is needed -- an agent-scope release fence in every workgroup (an L2
// write-back each) cost 0.4 ms over the 16k workgroups of a one-launch Adam.
__device__ __forceinline__ void llp_store_handed(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float llp_load_handed(const float* p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}

// One workgroup's arrival on a launch-wide ticket block (LLP_TICKET_WORDS uint32, include/llp_hip.h):
// returns true in the LAST workgroup to arrive.  Two levels, so the arrivals do not all
// serialise on one word (thousands of adds on a single address cost 0.2 ms in a one-launch
// Adam): arrival b (0 .. n_blocks-1, dense: each arriving workgroup passes its own) adds to
// sub-ticket b % 64, the last arriver there adds to the main word.
// Each word is returned to zero by its last arriver, so a block zeroed once at allocation stays
// valid call after call, graph replays included.  Every word this workgroup hands to the last
// arriver must have been stored by its thread 0 with llp_store_handed; thread 0 drains its
// stores (vmcnt(0)) before its add.  Called by every thread.
constexpr int LLP_TICKET_SUBS = 64, LLP_TICKET_STRIDE = 32;   // sub-tickets 128 B apart

__device__ __forceinline__ bool llp_arrive_last_tree(uint32_t* tk, uint32_t b, uint32_t n_blocks) {
  __shared__ int last;
  if (threadIdx.x == 0) {
    const uint32_t sub = b % LLP_TICKET_SUBS;
    const uint32_t n_sub = (n_blocks - sub + LLP_TICKET_SUBS - 1) / LLP_TICKET_SUBS;   // arrivals on it
    const uint32_t n_main = n_blocks < (uint32_t)LLP_TICKET_SUBS ? n_blocks : (uint32_t)LLP_TICKET_SUBS;
    uint32_t* st = tk + LLP_TICKET_STRIDE * (1 + sub);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int l = 0;
    if (__hip_atomic_fetch_add(st, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n_sub - 1) {
      __hip_atomic_store(st, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n_main - 1) {
        __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        l = 1;
      }
    }
    last = l;
  }
  __syncthreads();
  return last != 0;
}

// The one-word form (the compaction scans' state blocks hold one ticket word): the same
// contract as llp_arrive_last_tree on tk[0] alone.
__device__ __forceinline__ bool llp_arrive_last(uint32_t* tk, uint32_t n_blocks) {
  __shared__ int last;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == n_blocks - 1;
    if (last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return last != 0;
}

// ---------------------------------------------------------------- single-pass scan (decoupled look-back)
// Workgroup b of a launch publishes its aggregate, looks back over its predecessors' published
// aggregates / inclusive prefixes (64 per window, one wave) and publishes its inclusive prefix
// (values and flags are agent-scope atomic stores and loads: write-through, no fences);
// returns its exclusive prefix to every thread.  flags[b] = (epoch << 2) | status (1 aggregate,
// 2 inclusive): the epoch tags one call, so the flags never need resetting (the caller advances
// the epoch once per call).  Waits only on lower-numbered workgroups, which the dispatcher starts
// first on each XCD; spins are bounded.  A publisher never seen sets *err, and the workgroup
// publishes LLP_LB_FAIL instead of its prefix, so its successors fail at once instead of spinning
// out in turn; every failed workgroup gets the exclusive prefix 0, which keeps the callers'
// prefix-indexed writes inside their buffers (a prefix is at most the total, so 0 plus the
// workgroup's own part is too).  The results are then invalid but in bounds, and the caller
// checks *err (llp_hip.py error_word, DistillEngine.check_device_errors).  u64 sums: any
// association gives the same result.
constexpr uint32_t LLP_LB_AGG = 1u, LLP_LB_INC = 2u, LLP_LB_FAIL = 3u;

__device__ __forceinline__ uint32_t llp_lb_wait(const uint32_t* flag, uint32_t epoch, uint32_t* err) {
  uint32_t f = 0;
  for (uint32_t it = 0;; ++it) {
    f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((f >> 2) == (epoch & 0x3FFFFFFFu) && (f & 3u)) break;
    if (it > (1u << 22)) {
      __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return LLP_LB_FAIL;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: keeps the value loads below
  return f & 3u;
}

__device__ __forceinline__ unsigned long long llp_lookback_u64(uint32_t* flags, unsigned long long* agg,
                                                               unsigned long long* incl, int64_t b,
                                                               unsigned long long blk_sum, uint32_t epoch,
                                                               uint32_t* err) {
  __shared__ unsigned long long lb_excl;
  const int t = threadIdx.x;
  if (t == 0) {
    __hip_atomic_store(b == 0 ? &incl[0] : &agg[b], blk_sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the write-through value before its flag
    __hip_atomic_store(&flags[b], (epoch << 2) | (b == 0 ? LLP_LB_INC : LLP_LB_AGG), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    if (b == 0) lb_excl = 0ull;
  }
  if (b > 0 && t < 64) {   // wave 0: 64 predecessors per window, nearest first
    unsigned long long acc = 0;
    bool failed = false;
    for (int64_t j0 = b - 1;; j0 -= 64) {
      const int64_t j = j0 - t;
      uint32_t st = 0;
      unsigned long long val = 0;
      if (j >= 0) {
        st = llp_lb_wait(&flags[j], epoch, err);
        val = __hip_atomic_load(st == LLP_LB_INC ? &incl[j] : &agg[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (__ballot(j >= 0 && st == LLP_LB_FAIL)) {   // a predecessor timed out or failed: so does this one
        failed = true;
        break;
      }
      // the nearest predecessor holding an inclusive prefix (workgroup 0 always does) ends it
      const unsigned long long inc_mask = __ballot(j >= 0 && st == LLP_LB_INC);
      const int stop = inc_mask ? __builtin_ctzll(inc_mask) : 64;
      unsigned long long part = (t <= stop && j >= 0) ? val : 0ull;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
      acc += part;
      if (inc_mask || j0 - 64 < 0) break;
    }
    if (t == 0) {
      lb_excl = failed ? 0ull : acc;
      if (!failed) {
        __hip_atomic_store(&incl[b], acc + blk_sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __hip_atomic_store(&flags[b], (epoch << 2) | (failed ? LLP_LB_FAIL : LLP_LB_INC), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  return lb_excl;
}
