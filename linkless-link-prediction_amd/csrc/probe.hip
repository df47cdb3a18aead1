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
