// Micro-benchmark of the product sort passes (sentinel_amd/csrc/sf_rsort.h)
// against rocprim::radix_sort_pairs on config-3-like keys (Zipf(1.1) ranks
// over 10M resources, scrambled), 8-B payloads.  Build variants with
// -DSF_RS_DB / -DSF_RS_W / -DSF_RS_K (tools/micro/build_rs.sh).
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../sentinel_amd/csrc/sf_rsort.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
using namespace sf;

__device__ __forceinline__ uint64_t hash64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x;
}
__global__ void gen(uint32_t* k, PackedEv* v, uint32_t n, uint32_t R, uint64_t seed) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t h = hash64(i + seed * 0x9e3779b97f4a7c15ull);
    uint64_t rank;
    for (int t = 0;; t++) {
        double u = ((h >> 11) + 0.5) * (1.0 / 9007199254740992.0);
        rank = (uint64_t)pow(u, -10.0) - 1;
        if (rank < R) break;
        h = hash64(h + t + 1);
    }
    k[i] = (uint32_t)((rank * 2654435761ull) % R);
    v[i].idx = i; v[i].meta = (uint32_t)(h >> 40);
}

// rs_sort with an array source for the first pass too (the product's first pass reads the batch, its last
// writes the sorted SoA); middle buffers as the product's (a, b) pair
static void sort_arrays(uint32_t* k0, PackedEv* v0, uint32_t* ka, PackedEv* va, uint32_t* kb_, PackedEv* vb,
                        uint32_t* kf, PackedEv* vf, uint32_t n, uint32_t kb, void* scratch, hipEvent_t* ev) {
    const uint32_t P = (kb + RS_DB - 1) / RS_DB, D = (kb + P - 1) / P, mask = (1u << D) - 1u;
    const uint32_t* ki = k0; const PackedEv* vi = v0;
    for (uint32_t p = 0; p < P; p++) {
        uint32_t* ko = p + 1 == P ? kf : (p & 1) ? kb_ : ka;
        PackedEv* vo = p + 1 == P ? vf : (p & 1) ? vb : va;
        if (ev) hipEventRecord(ev[p]);
        rs_launch_pass<RsArraySrc<PackedEv>, RsSinkKV<PackedEv>, PackedEv>(RsArraySrc<PackedEv>{ki, vi},
                                                                             RsSinkKV<PackedEv>{ko, vo}, n, p * D, mask,
                                                                             scratch, 0);
        ki = ko; vi = vo;
    }
    if (ev) hipEventRecord(ev[P]);
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : (1u << 27);
    const uint32_t R = argc > 2 ? (uint32_t)atol(argv[2]) : 10000000u;
    uint32_t bits = 1; while ((1ull << bits) < R) bits++;
    uint32_t *k0, *k1, *k2, *k3, *rk; PackedEv *v0, *v1, *v2, *v3, *rv; void* scratch;
    CK(hipMalloc(&k0, n * 4ull)); CK(hipMalloc(&k1, n * 4ull)); CK(hipMalloc(&k2, n * 4ull)); CK(hipMalloc(&rk, n * 4ull)); CK(hipMalloc(&k3, n * 4ull)); CK(hipMalloc(&v3, n * 8ull));
    CK(hipMalloc(&v0, n * 8ull)); CK(hipMalloc(&v1, n * 8ull)); CK(hipMalloc(&v2, n * 8ull)); CK(hipMalloc(&rv, n * 8ull));
    CK(hipMalloc(&scratch, rs_scratch_bytes()));
    hipLaunchKernelGGL(gen, dim3((n + 255) / 256), dim3(256), 0, 0, k0, v0, n, R, 7ull);
    CK(hipDeviceSynchronize());
    size_t tb = 0;
    CK(rocprim::radix_sort_pairs(nullptr, tb, k0, rk, v0, rv, n, 0u, bits));
    void* tmp; CK(hipMalloc(&tmp, tb));
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const int reps = 5; float ms;
    CK(rocprim::radix_sort_pairs(tmp, tb, k0, rk, v0, rv, n, 0u, bits));
    hipEventRecord(a);
    for (int r = 0; r < reps; r++) CK(rocprim::radix_sort_pairs(tmp, tb, k0, rk, v0, rv, n, 0u, bits));
    hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    printf("n %u R %u bits %u | DB %d W %d tile %d\n", n, R, bits, RS_DB, RS_W, RsGeom<PackedEv>::TILE);
    printf("rocprim onesweep    %.3f ms\n", ms / reps);
    sort_arrays(k0, v0, k1, v1, k2, v2, k3, v3, n, bits, scratch, nullptr);
    CK(hipDeviceSynchronize());
    hipEventRecord(a);
    for (int r = 0; r < reps; r++) sort_arrays(k0, v0, k1, v1, k2, v2, k3, v3, n, bits, scratch, nullptr);
    hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    std::vector<uint32_t> hk(n), gk(n); std::vector<uint64_t> hv(n), gv(n);
    CK(hipMemcpy(hk.data(), rk, n * 4ull, hipMemcpyDeviceToHost)); CK(hipMemcpy(hv.data(), rv, n * 8ull, hipMemcpyDeviceToHost));
    CK(hipMemcpy(gk.data(), k3, n * 4ull, hipMemcpyDeviceToHost)); CK(hipMemcpy(gv.data(), v3, n * 8ull, hipMemcpyDeviceToHost));
    uint64_t bad = 0; for (uint32_t i = 0; i < n; i++) bad += (gk[i] != hk[i]) | (gv[i] != hv[i]);
    printf("rs_sort passes      %.3f ms  mismatches %llu\n", ms / reps, (unsigned long long)bad);
    hipEvent_t ev[8]; for (auto& e : ev) hipEventCreate(&e);
    sort_arrays(k0, v0, k1, v1, k2, v2, k3, v3, n, bits, scratch, ev);
    CK(hipDeviceSynchronize());
    const uint32_t P = (bits + RS_DB - 1) / RS_DB;
    for (uint32_t p = 0; p < P; p++) {
        float q; hipEventElapsedTime(&q, ev[p], ev[p + 1]);
        printf("  pass %u (count + scan + pass): %.3f ms (%.2f TB/s of 24 B/event)\n", p, q, 24.0 * n / (q * 1e-3) / 1e12);
    }
    return 0;
}
