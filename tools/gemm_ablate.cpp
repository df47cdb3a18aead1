// Ablation harness for the 256x256 NT GEMM main loop (cdna_hip_programming.md
// §7 "The diagnostic loop": which phase dominates?).  Build three variants:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/gemm_ablate.cpp [-DLLP_ABLATE_NOLOAD|-DLLP_ABLATE_NOMFMA]
// and run each: prints ms and TFLOP/s for M=747214, N=K=1024 (outputs of the
// ablated builds are garbage by construction).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "../linkless-link-prediction_amd/csrc/gemm256.hip"

namespace llp {
thread_local char g_err[512];
int set_error(int code, const char*, ...) { return code; }
}  // namespace llp

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("%s\n", hipGetErrorString(err_)); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int64_t M = argc > 1 ? atoll(argv[1]) : 747214, N = 1024, K = 1024;
  void *A, *B, *C;
  CK(hipMalloc(&A, M * K * 2));
  CK(hipMalloc(&B, N * K * 2));
  CK(hipMalloc(&C, M * N * 2));
  std::vector<uint16_t> h(N * K, 0x3c00);
  CK(hipMemcpy(B, h.data(), N * K * 2, hipMemcpyHostToDevice));
  CK(hipMemset(A, 0x3c, M * K * 2));
  // argv[2] == "small": A rows gathered from a 1024-row (2 MiB) table -> L2-resident A
  int32_t* idx = nullptr;
  if (argc > 2) {
    std::vector<int32_t> hi(M);
    for (int64_t i = 0; i < M; ++i) hi[i] = (int32_t)(i % 1024);
    CK(hipMalloc(&idx, M * 4));
    CK(hipMemcpy(idx, hi.data(), M * 4, hipMemcpyHostToDevice));
  }
  llp_operand a{A, idx, nullptr, nullptr, K, 0}, b{B, nullptr, nullptr, nullptr, K, 0};
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  for (int i = 0; i < 3; ++i)
    llp_gemm_nt_bf16_256(&a, &b, M, N, K, C, N, nullptr, 0, nullptr, 0, 1.f, 0.f, 0, 1.f, 0, nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, 0);
  CK(hipEventRecord(s, 0));
  const int it = 20;
  for (int i = 0; i < it; ++i)
    llp_gemm_nt_bf16_256(&a, &b, M, N, K, C, N, nullptr, 0, nullptr, 0, 1.f, 0.f, 0, 1.f, 0, nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, 0);
  CK(hipEventRecord(e, 0));
  CK(hipEventSynchronize(e));
  float ms;
  CK(hipEventElapsedTime(&ms, s, e));
  ms /= it;
  printf("M=%lld N=%lld K=%lld  %.3f ms  %.1f TFLOP/s\n", (long long)M, (long long)N, (long long)K, ms,
         2.0 * M * N * K / ms / 1e9);
  return 0;
}
