// Link-prediction evaluation metrics on the device:
//   * Hits@K — ogb 1.3.6 Evaluator('ogbl-*')._eval_hits as used at
//     src/train_teacher_gnn.py:121-143: kth = topk(y_pred_neg, K)[-1],
//     hits = #(y_pred_pos > kth) / len(y_pred_pos); len(neg) < K -> 1.0.
//     The K-th largest negative comes from an exact 4-pass LDS radix select
//     (one workgroup per K), so the result is bit-identical to topk's.
//   * AUC — sklearn roc_auc_score as used at src/train_teacher_gnn.py:153:
//     the Mann-Whitney statistic with ties counted 1/2, from the negatives
//     sorted on the device (rocPRIM radix sort) and two binary searches per
//     positive.
#include "llp_common.h"

#include <rocprim/device/device_radix_sort.hpp>

namespace {

__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__global__ __launch_bounds__(1024) void hits_kernel(const float* __restrict__ pos, int64_t n_pos,
                                                    const float* __restrict__ neg, int64_t n_neg,
                                                    const int32_t* __restrict__ Ks, double* __restrict__ out) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_prefix, s_mask;
  __shared__ int64_t s_rank;
  __shared__ unsigned long long s_cnt;
  const int64_t K = Ks[blockIdx.x];
  const int tid = threadIdx.x;
  if (K <= 0 || n_neg < K) {   // ogb: len(y_pred_neg) < K -> 1.0 (K <= 0 is rejected on the host)
    if (tid == 0) out[blockIdx.x] = 1.0;
    return;
  }
  if (tid == 0) {
    s_prefix = 0;
    s_mask = 0;
    s_rank = n_neg - K;   // ascending index of the K-th largest
    s_cnt = 0;
  }
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = tid; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix, mask = s_mask;
    for (int64_t i = tid; i < n_neg; i += blockDim.x) {
      const uint32_t k = f2key(neg[i]);
      if ((k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      int64_t r = s_rank;
      uint32_t b = 0;
      for (; b < 255; ++b) {
        if (r < (int64_t)hist[b]) break;
        r -= hist[b];
      }
      s_rank = r;
      s_prefix = prefix | (b << shift);
      s_mask = mask | (255u << shift);
    }
    __syncthreads();
  }
  const float kth = key2f(s_prefix);
  unsigned long long c = 0;
  for (int64_t i = tid; i < n_pos; i += blockDim.x) c += pos[i] > kth ? 1ull : 0ull;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((tid & 63) == 0) atomicAdd(&s_cnt, c);
  __syncthreads();
  if (tid == 0) out[blockIdx.x] = n_pos > 0 ? (double)s_cnt / (double)n_pos : 0.0;
}

__global__ __launch_bounds__(256) void auc_count_kernel(const float* __restrict__ pos, int64_t n_pos,
                                                        const float* __restrict__ neg_sorted, int64_t n_neg,
                                                        double* __restrict__ partial) {
  __shared__ double red[4];
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  double v = 0.0;
  if (i < n_pos) {
    const float s = pos[i];
    int64_t lo = 0, hi = n_neg;   // lower_bound(s)
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (neg_sorted[m] < s) lo = m + 1; else hi = m;
    }
    int64_t lo2 = lo, hi2 = n_neg;   // upper_bound(s)
    while (lo2 < hi2) {
      const int64_t m = (lo2 + hi2) >> 1;
      if (neg_sorted[m] <= s) lo2 = m + 1; else hi2 = m;
    }
    v = (double)lo + 0.5 * (double)(lo2 - lo);
  }
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void auc_finalize(const double* __restrict__ partial, int64_t nb, int64_t n_pos,
                                                    int64_t n_neg, double* __restrict__ out) {
  __shared__ double red[256];
  double a = 0.0;
  for (int64_t i = threadIdx.x; i < nb; i += blockDim.x) a += partial[i];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = red[0] / ((double)n_pos * (double)n_neg);
}

size_t sort_temp_bytes(int64_t n) {
  size_t tb = 0;
  rocprim::radix_sort_keys(nullptr, tb, (const float*)nullptr, (float*)nullptr, (unsigned int)n);
  return tb;
}

}  // namespace

extern "C" int llp_hits_at_k(const float* pos, int64_t n_pos, const float* neg, int64_t n_neg, const int32_t* Ks,
                             int n_K, double* hits_out, void* stream) {
  LLP_CHECK_ARG(hits_out && Ks && n_K > 0, "llp_hits_at_k: null output / K list");
  LLP_CHECK_ARG((n_pos == 0 || pos) && (n_neg == 0 || neg), "llp_hits_at_k: null scores");
  hipLaunchKernelGGL(hits_kernel, dim3((unsigned)n_K), dim3(1024), 0, (hipStream_t)stream, pos, n_pos, neg, n_neg, Ks,
                     hits_out);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}

extern "C" int64_t llp_auc_workspace_bytes(int64_t n_pos, int64_t n_neg) {
  const int64_t nb = (n_pos + 255) / 256;
  return ((n_neg * 4 + 255) & ~255ll) + ((nb * 8 + 255) & ~255ll) + (int64_t)sort_temp_bytes(n_neg) + 256;
}

extern "C" int llp_auc(const float* pos, int64_t n_pos, const float* neg, int64_t n_neg, double* auc_out,
                       void* workspace, int64_t workspace_bytes, void* stream) {
  LLP_CHECK_ARG(pos && neg && auc_out && workspace, "llp_auc: null pointer");
  LLP_CHECK_ARG(n_pos > 0 && n_neg > 0 && n_neg < (1ll << 32), "llp_auc: needs both classes");
  LLP_CHECK_ARG(workspace_bytes >= llp_auc_workspace_bytes(n_pos, n_neg), "llp_auc: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  size_t tb = sort_temp_bytes(n_neg);
  char* w = reinterpret_cast<char*>(workspace);
  float* sorted = reinterpret_cast<float*>(w);
  const int64_t nb = (n_pos + 255) / 256;
  double* partial = reinterpret_cast<double*>(w + ((n_neg * 4 + 255) & ~255ll));
  void* temp = reinterpret_cast<char*>(partial) + ((nb * 8 + 255) & ~255ll);
  hipError_t e = rocprim::radix_sort_keys(temp, tb, neg, sorted, (unsigned int)n_neg, 0, 32, s);
  if (e != hipSuccess) return ::llp::set_error((int)e, "llp_auc: radix sort: %s", hipGetErrorString(e));
  hipLaunchKernelGGL(auc_count_kernel, dim3((unsigned)nb), dim3(256), 0, s, pos, n_pos, sorted, n_neg, partial);
  LLP_LAUNCH_CHECK();
  hipLaunchKernelGGL(auc_finalize, dim3(1), dim3(256), 0, s, partial, nb, n_pos, n_neg, auc_out);
  LLP_LAUNCH_CHECK();
  return LLP_OK;
}
