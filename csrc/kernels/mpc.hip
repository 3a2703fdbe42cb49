// Modular matrix product for the TurboAggregate secret-sharing layer (K22): C = (A @ B) mod p on int64 operands
// already reduced to [0, p), p < 2^32.  BGW / LCC encoding of a model-sized update is U [N x K] @ X [K x d]
// (d = parameters, millions; N, K = workers / shards, tens): one thread per output element, B and C rows read and
// written coalesced along d, the K products (< 2^64 each) reduced mod p before the sum, the sum (< K * p) reduced
// once.  Reference: fedml_api/distributed/turboaggregate/mpc_function.py (numpy, host).
#include "common.h"

namespace nidt {

__global__ __launch_bounds__(256) void k_modp_matmul(const int64_t* __restrict__ A, const int64_t* __restrict__ B,
                                                     int64_t* __restrict__ C, int M, int K, int64_t N, uint64_t p) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int i = blockIdx.y;
  if (j >= N) return;
  uint64_t acc = 0;
  for (int k = 0; k < K; ++k) {
    const uint64_t a = (uint64_t)A[(int64_t)i * K + k];
    const uint64_t b = (uint64_t)B[(int64_t)k * N + j];
    acc += (a * b) % p;
  }
  C[(int64_t)i * N + j] = (int64_t)(acc % p);
}

void modp_matmul(uintptr_t A, uintptr_t B, uintptr_t C, int M, int K, int64_t N, int64_t p, uintptr_t stream) {
  NIDT_REQUIRE(p > 1 && p < (1ll << 32), "modp_matmul: 1 < p < 2^32");
  NIDT_REQUIRE(M > 0 && M < 65536 && K > 0 && N > 0, "modp_matmul: shapes");
  hipLaunchKernelGGL(k_modp_matmul, dim3((unsigned)((N + 255) / 256), M), dim3(256), 0, as_stream(stream),
                     ptr<const int64_t>(A), ptr<const int64_t>(B), ptr<int64_t>(C), M, K, N, (uint64_t)p);
  NIDT_CHECK(hipGetLastError());
}

}  // namespace nidt
