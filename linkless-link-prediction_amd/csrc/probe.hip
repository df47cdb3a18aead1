// Practical bf16 MFMA ceiling of the device on random operands, timed by bench.py next to
// the dominant GEMM (roofline.practical_peak).  Every CU runs one 512-thread workgroup (two
// waves per SIMD) that issues v_mfma_f32_16x16x32_bf16 back to back on register operands
// drawn from random bf16 data (4 x 4 operand pairs), eight accumulators per wave: the loop shape of
// MI355X_MICROARCH.md's bare-MFMA measurement.  Under dense MFMA load on random data the
// chip lowers its clock (DVFS give-back), so this loop's FLOP/s, not the 2.5 PF/s spec, is
// what any GEMM on such data can approach; the spec peak stays the roofline's `peak`.
#include "llp_common.h"

int llp_cu_count();

namespace {

constexpr int PROBE_THREADS = 512;
constexpr int PROBE_ACC = 8;

// Four A and four B fragments per lane, all random: consecutive MFMAs take different
// operands (a loop on one fixed operand pair barely toggles the multipliers and holds a
// higher clock than any GEMM can).  One iteration = 16 MFMAs over the 4 x 4 operand pairs
// into 8 accumulators.
__global__ __launch_bounds__(PROBE_THREADS) void mfma_probe_kernel(const uint4* __restrict__ data, int64_t n_u4,
                                                                   int64_t iters, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * PROBE_THREADS + threadIdx.x;
  short8 a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint4 ra = data[(8 * t + i) % n_u4], rb = data[(8 * t + 4 + i) % n_u4];
    a[i] = *reinterpret_cast<const short8*>(&ra);
    b[i] = *reinterpret_cast<const short8*>(&rb);
  }
  float4_t acc[PROBE_ACC];
#pragma unroll
  for (int j = 0; j < PROBE_ACC; ++j) acc[j] = float4_t{0.f, 0.f, 0.f, 0.f};
  for (int64_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      acc[j & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j & 3], b[(j >> 2) ^ (j & 1)], acc[j & 7], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < PROBE_ACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[t] = s;
}

// The f32 counterpart (v_mfma_f32_16x16x4_f32, the fp32 GEMMs' instruction, gemm.hip): four
// random f32 A and B operands per lane, 16 MFMAs per iteration into 8 accumulators.
__global__ __launch_bounds__(PROBE_THREADS) void mfma_probe_f32_kernel(const float* __restrict__ data, int64_t n,
                                                                       int64_t iters, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * PROBE_THREADS + threadIdx.x;
  float a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = data[(8 * t + i) % n];
    b[i] = data[(8 * t + 4 + i) % n];
  }
  float4_t acc[PROBE_ACC];
#pragma unroll
  for (int j = 0; j < PROBE_ACC; ++j) acc[j] = float4_t{0.f, 0.f, 0.f, 0.f};
  for (int64_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      acc[j & 7] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j & 3], b[(j >> 2) ^ (j & 1)], acc[j & 7], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < PROBE_ACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[t] = s;
}

}  // namespace

extern "C" int llp_mfma_probe_f32(const float* data, int64_t n, int64_t iters, float* out, double* flops,
                                  void* stream) {
  LLP_CHECK_ARG(data && out && flops && n >= 8 && iters >= 0, "llp_mfma_probe_f32: arguments");
  const int cus = llp_cu_count();
  *flops = (double)cus * (PROBE_THREADS / 64) * (double)iters * 16 * (16.0 * 16.0 * 4.0 * 2.0);
  hipLaunchKernelGGL(mfma_probe_f32_kernel, dim3((unsigned)cus), dim3(PROBE_THREADS), 0, (hipStream_t)stream, data,
                     n, iters, out);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int llp_mfma_probe(const void* data, int64_t n_u4, int64_t iters, float* out, double* flops,
                              void* stream) {
  LLP_CHECK_ARG(data && out && flops && n_u4 >= 2 && iters >= 0, "llp_mfma_probe: arguments");
  const int cus = llp_cu_count();
  *flops = (double)cus * (PROBE_THREADS / 64) * (double)iters * 16 * (16.0 * 16.0 * 32.0 * 2.0);
  hipLaunchKernelGGL(mfma_probe_kernel, dim3((unsigned)cus), dim3(PROBE_THREADS), 0, (hipStream_t)stream,
                     (const uint4*)data, n_u4, iters, out);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int64_t llp_mfma_probe_out_floats() { return (int64_t)llp_cu_count() * PROBE_THREADS; }

// ---------------------------------------------------------------------------
// Staging-cost probe (round 6; DESIGN.md §4.1, "one wave per SIMD"): what moving a GEMM
// tile's operand bytes costs a wave that is ALONE on its SIMD and issues
// v_mfma_f32_32x32x16_bf16 back to back (16 independent accumulators held in AGPRs by inline
// asm, the structure a 128 x 128-per-wave NT GEMM would have).  Every CU runs one 256-thread
// workgroup (four waves, one per SIMD; 96 KiB of LDS keeps a second one off the CU).  Per
// iteration a wave issues 32 MFMAs and, spread evenly between them, `pieces` 1-KiB operand
// pieces by one of:
//   mode 0  nothing (the MFMA floor)
//   mode 1  global_load_lds_dwordx4 (LDS-DMA, the NT GEMM's staging)
//   mode 2  global_load_dwordx4 into VGPRs, ds_write_b128 of the previous iteration's data
//   mode 3  ds_read_b128 only (fragment reads, no staging)
// Wave 0 of each workgroup records s_memtime around the loop: cycles[blockIdx] / (iters * 32)
// = shader cycles per MFMA.
namespace {
typedef float f32x16_t __attribute__((ext_vector_type(16)));

template <int MODE, int PIECES>
__global__ __launch_bounds__(256, 1) void stage_probe_kernel(const uint4* __restrict__ src, int64_t src_u4,
                                                              int64_t iters, float* __restrict__ out,
                                                              unsigned long long* __restrict__ cycles) {
  __shared__ __attribute__((aligned(16))) uint4 lds[96 * 1024 / 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t pmask = (uint32_t)(src_u4 / 64) - 1u;   // src_u4 / 64 is a power of two (host-checked)
  short8 a[2], b[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const uint4 ra = src[((4 * (blockIdx.x * 256 + tid) + i)) & (src_u4 - 1)];
    const uint4 rb = src[((4 * (blockIdx.x * 256 + tid) + 2 + i)) & (src_u4 - 1)];
    a[i] = *reinterpret_cast<const short8*>(&ra);
    b[i] = *reinterpret_cast<const short8*>(&rb);
  }
  f32x16_t acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j)
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=a"(acc[j]) : "v"(a[j & 1]), "v"(b[(j >> 1) & 1]));
  // this wave's 1-KiB piece window: a slice of src walked per iteration (L2 / MALL-resident
  // when src is a few MB, HBM when larger)
  const uint32_t lds_w = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) void*)lds) + w * 16384u;
  uint4 stg[PIECES > 0 ? PIECES : 1];
#pragma unroll
  for (int q = 0; q < (PIECES > 0 ? PIECES : 1); ++q) stg[q] = make_uint4(0u, 0u, 0u, 0u);
  uint4 rd[PIECES > 0 ? PIECES : 1];
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int64_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc[j & 15]) : "v"(a[j & 1]), "v"(b[(j >> 1) & 1])
                   : "memory");
      if (PIECES > 0 && (j % (32 / (PIECES > 0 ? PIECES : 1))) == 0) {
        const int q = j / (32 / (PIECES > 0 ? PIECES : 1));
        const uint32_t pc = ((uint32_t)(blockIdx.x * 4 + w) * 97u + (uint32_t)it * PIECES + q) & pmask;
        if (MODE == 1) {
          const uint4* g = src + pc * 64 + lane;
          asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g),
                       "s"(__builtin_amdgcn_readfirstlane(lds_w + (uint32_t)((q & 15) * 1024)))
                       : "memory", "m0");
        } else if (MODE == 2) {
          lds[w * 1024 + (q & 15) * 64 + lane] = stg[q];
          stg[q] = src[pc * 64 + lane];
        } else if (MODE == 3) {
          rd[q] = lds[w * 1024 + (q & 15) * 64 + ((lane + q) & 63)];
        }
      }
    }
    if (MODE == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PIECES > 0 ? PIECES : 0) : "memory");
    if (MODE == 3) {
#pragma unroll
      for (int q = 0; q < (PIECES > 0 ? PIECES : 1); ++q) asm volatile("" ::"v"(rd[q].x), "v"(rd[q].y), "v"(rd[q].z), "v"(rd[q].w));
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 15" ::: "memory");
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += acc[j][0] + acc[j][15];
#pragma unroll
  for (int q = 0; q < (PIECES > 0 ? PIECES : 1); ++q) s += __uint_as_float(stg[q].x & 0x3FFFFFFFu) * 1e-30f;
  out[blockIdx.x * 256 + tid] = s;
  if (tid == 0) cycles[blockIdx.x] = t1 - t0;
}

template <int MODE>
void launch_stage_probe(int pieces, dim3 g, hipStream_t s, const uint4* src, int64_t n, int64_t iters, float* out,
                        unsigned long long* cyc) {
  switch (pieces) {
    case 0: hipLaunchKernelGGL((stage_probe_kernel<MODE, 0>), g, dim3(256), 0, s, src, n, iters, out, cyc); break;
    case 4: hipLaunchKernelGGL((stage_probe_kernel<MODE, 4>), g, dim3(256), 0, s, src, n, iters, out, cyc); break;
    case 8: hipLaunchKernelGGL((stage_probe_kernel<MODE, 8>), g, dim3(256), 0, s, src, n, iters, out, cyc); break;
    default: hipLaunchKernelGGL((stage_probe_kernel<MODE, 16>), g, dim3(256), 0, s, src, n, iters, out, cyc); break;
  }
}
}  // namespace

// mode 0-3 as above; pieces in {0, 4, 8, 16} per 32 MFMAs; src_u4 / 64 a power of two; out: 256 floats
// per CU; cycles: one per CU
extern "C" int llp_stage_probe(int mode, int pieces, const void* src, int64_t src_u4, int64_t iters, float* out,
                               unsigned long long* cycles, void* stream) {
  LLP_CHECK_ARG(src && out && cycles && src_u4 >= 64 * 64 && ((src_u4 / 64) & (src_u4 / 64 - 1)) == 0 &&
                    src_u4 % 64 == 0 && iters >= 1 && mode >= 0 && mode <= 3 &&
                    (pieces == 0 || pieces == 4 || pieces == 8 || pieces == 16),
                "llp_stage_probe: arguments");
  const dim3 g((unsigned)llp_cu_count());
  hipStream_t s = (hipStream_t)stream;
  const uint4* p = (const uint4*)src;
  if (mode == 0) launch_stage_probe<0>(0, g, s, p, src_u4, iters, out, cycles);
  else if (mode == 1) launch_stage_probe<1>(pieces, g, s, p, src_u4, iters, out, cycles);
  else if (mode == 2) launch_stage_probe<2>(pieces, g, s, p, src_u4, iters, out, cycles);
  else launch_stage_probe<3>(pieces, g, s, p, src_u4, iters, out, cycles);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}
