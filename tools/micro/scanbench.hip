// Micro-benchmark (diagnostics): the sort phase's two rocprim inclusive scans
// on gfx950 -- u32 segment heads (transform over sorted keys) and int64 entry
// acquireCount prefix (transform over count / flags) -- default config vs
// explicit scan_config choices.
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>
#include <cstdio>
#include <cstring>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct HeadFlag {
    const uint32_t* keys;
    __device__ uint32_t operator()(uint32_t j) const { return (j == 0 || keys[j] != keys[j - 1]) ? 1u : 0u; }
};
struct EntryCount {
    const int32_t* cnt; const uint8_t* flags;
    __device__ int64_t operator()(uint32_t j) const { return (flags[j] & 1) ? 0 : (int64_t)cnt[j]; }
};
__global__ void gen(uint32_t* k, int32_t* c, uint8_t* f, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    k[i] = i / 37; c[i] = 1 + (i % 5 == 0); f[i] = (i % 9 == 0);
}

template <class Cfg, class It, class T>
float run(It it, T* out, uint32_t n, int reps) {
    size_t tb = 0;
    CK(rocprim::inclusive_scan<Cfg>(nullptr, tb, it, out, (size_t)n, rocprim::plus<T>()));
    void* tmp; CK(hipMalloc(&tmp, tb));
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    CK(rocprim::inclusive_scan<Cfg>(tmp, tb, it, out, (size_t)n, rocprim::plus<T>()));
    hipEventRecord(a);
    for (int r = 0; r < reps; r++) CK(rocprim::inclusive_scan<Cfg>(tmp, tb, it, out, (size_t)n, rocprim::plus<T>()));
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    hipFree(tmp);
    return ms / reps;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : (1u << 27);
    uint32_t* k; int32_t* c; uint8_t* f; uint32_t* o32; int64_t* o64;
    CK(hipMalloc(&k, n * 4ull)); CK(hipMalloc(&c, n * 4ull)); CK(hipMalloc(&f, n));
    CK(hipMalloc(&o32, n * 4ull)); CK(hipMalloc(&o64, n * 8ull));
    gen<<<(n + 255) / 256, 256>>>(k, c, f, n);
    CK(hipDeviceSynchronize());
    using namespace rocprim;
    auto hit = make_transform_iterator(counting_iterator<uint32_t>(0), HeadFlag{k});
    auto pit = make_transform_iterator(counting_iterator<uint32_t>(0), EntryCount{c, f});
    const int reps = 10;
    using T256x21w = scan_config<256, 21, block_load_method::block_load_transpose, block_store_method::block_store_transpose, block_scan_algorithm::using_warp_scan>;
    using T256x16w = scan_config<256, 16, block_load_method::block_load_transpose, block_store_method::block_store_transpose, block_scan_algorithm::using_warp_scan>;
    using T256x15r = scan_config<256, 15, block_load_method::block_load_transpose, block_store_method::block_store_transpose, block_scan_algorithm::reduce_then_scan>;
    using T256x8r = scan_config<256, 8, block_load_method::block_load_transpose, block_store_method::block_store_transpose, block_scan_algorithm::reduce_then_scan>;
    using T256x12w = scan_config<256, 12, block_load_method::block_load_transpose, block_store_method::block_store_transpose, block_scan_algorithm::using_warp_scan>;
    printf("n %u\n", n);
    printf("u32 heads default      %.3f ms\n", run<default_config>(hit, o32, n, reps));
    printf("u32 heads 256x21 warp  %.3f ms\n", run<T256x21w>(hit, o32, n, reps));
    printf("u32 heads 256x16 warp  %.3f ms\n", run<T256x16w>(hit, o32, n, reps));
    printf("i64 count default      %.3f ms\n", run<default_config>(pit, o64, n, reps));
    printf("i64 count 256x15 rts   %.3f ms\n", run<T256x15r>(pit, o64, n, reps));
    printf("i64 count 256x8 rts    %.3f ms\n", run<T256x8r>(pit, o64, n, reps));
    printf("i64 count 256x12 warp  %.3f ms\n", run<T256x12w>(pit, o64, n, reps));
    printf("i64 count 256x16 warp  %.3f ms\n", run<T256x16w>(pit, o64, n, reps));
    return 0;
}
