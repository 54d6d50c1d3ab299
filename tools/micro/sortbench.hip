// Micro-benchmark: rocprim radix_sort_pairs of n (u32 key of `bits` bits, u64 value) pairs on gfx950,
// default onesweep config (8 bits per pass) vs wider digits.  Diagnostics for the sort phase.
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void gen(uint32_t* k, uint64_t* v, uint32_t n, uint32_t bits, uint32_t seed) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t x = i * 2654435761u ^ seed; x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    // skewed: low keys more likely (crude Zipf-like)
    uint32_t m = (1u << bits) - 1u;
    uint32_t r = x & m;
    k[i] = (x >> 28) < 6 ? (r >> ((x >> 24) & 15)) : r;
    v[i] = ((uint64_t)i << 32) | x;
}

template <unsigned RB, class Cfg, class V>
float run(uint32_t* k0, V* v0, uint32_t* k1, V* v1, uint32_t n, uint32_t bits, int reps) {
    size_t tb = 0;
    CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tb, k0, k1, v0, v1, n, 0u, bits));
    void* tmp; CK(hipMalloc(&tmp, tb));
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, k0, k1, v0, v1, n, 0u, bits));   // warm
    hipEventRecord(a);
    for (int r = 0; r < reps; r++) CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, k0, k1, v0, v1, n, 0u, bits));
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    // check sortedness
    std::vector<uint32_t> h(n);
    CK(hipMemcpy(h.data(), k1, n * 4ull, hipMemcpyDeviceToHost));
    for (uint32_t i = 1; i < n; i++) if (h[i] < h[i - 1]) { printf("NOT SORTED at %u\n", i); exit(1); }
    hipFree(tmp);
    return ms / reps;
}

int main(int argc, char** argv) {
    uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : (1u << 27);
    uint32_t bits = argc > 2 ? (uint32_t)atoi(argv[2]) : 24;
    uint32_t *k0, *k1; uint64_t *v0, *v1;
    CK(hipMalloc(&k0, n * 4ull)); CK(hipMalloc(&k1, n * 4ull));
    CK(hipMalloc(&v0, n * 8ull)); CK(hipMalloc(&v1, n * 8ull));
    gen<<<(n + 255) / 256, 256>>>(k0, v0, n, bits, 12345u);
    CK(hipDeviceSynchronize());
    using C8 = rocprim::default_config;
    const int reps = 5;
    printf("n %u bits %u\n", n, bits);
    printf("u32 key + u64 value  %.3f ms\n", run<8, C8>(k0, v0, k1, v1, n, bits, reps));
    printf("u32 key + u32 value  %.3f ms\n", run<8, C8>(k0, (uint32_t*)v0, k1, (uint32_t*)v1, n, bits, reps));
    printf("u32 key + u64 value, 16-bit keys  %.3f ms\n", run<8, C8>(k0, v0, k1, v1, n, 16, reps));
    return 0;
}
