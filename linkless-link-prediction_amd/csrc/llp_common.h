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

// One workgroup's agent-scope arrival on a launch-wide ticket (cdna_hip_programming.md §5 "In-launch
// split-K reduction", Guideline 16): every store of this workgroup that the last arriver reads must
// have been made by its thread 0 (drained and released here).  Returns true in the LAST workgroup
// to arrive, which has acquired and returned the ticket to zero (so a ticket zeroed once at
// allocation stays valid call after call, graph replays included).  Called by every thread.
__device__ __forceinline__ bool llp_arrive_last(uint32_t* ticket, uint32_t n_blocks) {
  __shared__ int last;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == n_blocks - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  return last != 0;
}

// a 32-bit word another workgroup of this launch stored: a vector load behind the acquire
// (never the scalar path, Guideline 16 Pitfall 6)
__device__ __forceinline__ float llp_load_handed(const float* p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}
