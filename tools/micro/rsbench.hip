// Micro-benchmark for the sort phase: a hand-written chunked LSD radix sort of
// (u32 key, u64 value) pairs against rocprim::radix_sort_pairs (onesweep),
// on config-3-like keys (Zipf(1.1) ranks over 10M resources, scrambled).
//
// Chunked LSD pass (no decoupled look-back, no inter-workgroup waiting):
//   count  one workgroup per chunk (a contiguous range of the pass input):
//          digit histogram of the chunk -> h[chunk][bin]
//   scan   per bin, exclusive prefix over the chunks (in place) + bin totals
//   pass   one workgroup per chunk, tiles of W*K*64 elements in order: each
//          wave ranks its K rows of 64 (match-by-ballot on the digit bits, a
//          per-wave running count per bin in LDS), the waves' counts are
//          scanned per bin, and every element goes to
//          start[bin] + h[chunk][bin] + (earlier tiles of the chunk) + rank.
//   Stable: ranks follow (tile, wave, row, lane) = input order.
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint64_t hash64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x;
}
// Zipf(1.1)-like ranks over [0, R): inverse of the continuous power law, truncated; scrambled by a unit mod R
__global__ void gen(uint32_t* k, uint64_t* v, uint32_t n, uint32_t R, uint64_t seed) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t h = hash64(i + seed * 0x9e3779b97f4a7c15ull);
    uint64_t rank;
    for (int t = 0;; t++) {
        double u = ((h >> 11) + 0.5) * (1.0 / 9007199254740992.0);
        double x = pow(u, -10.0);                 // P(X > x) = x^-0.1
        rank = (uint64_t)x - 1;
        if (rank < R) break;
        h = hash64(h + t + 1);
    }
    k[i] = (uint32_t)((rank * 2654435761ull) % R);
    v[i] = ((uint64_t)i << 32) | (uint32_t)(h >> 40);
}

template <int DB>
__device__ __forceinline__ uint64_t match_bits(uint32_t d, uint64_t act) {
    uint64_t m = act;
#pragma unroll
    for (int b = 0; b < DB; b++) {
        const uint64_t x = __ballot((d >> b) & 1u);
        m &= ((d >> b) & 1u) ? x : ~x;
    }
    return m;
}

template <int DB, int T>
__global__ __launch_bounds__(T) void k_count(const uint32_t* key, uint32_t n, uint32_t chunk, uint32_t shift,
                                             uint32_t* h) {
    constexpr int NB = 1 << DB;
    __shared__ uint32_t hist[NB];
    for (int b = threadIdx.x; b < NB; b += T) hist[b] = 0;
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += T) atomicAdd(&hist[(key[i] >> shift) & (NB - 1)], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < NB; b += T) h[(size_t)blockIdx.x * NB + b] = hist[b];
}

// per bin (one workgroup each, one chunk per thread): exclusive prefix over the chunks, bin total
template <int DB>
__global__ __launch_bounds__(1024) void k_scan_chunks(uint32_t* h, uint32_t nchunks, uint32_t* tot) {
    constexpr int NB = 1 << DB;
    __shared__ uint32_t wsum[16];
    const uint32_t b = blockIdx.x, c = threadIdx.x, lane = c & 63, wv = c >> 6;
    const uint32_t x = c < nchunks ? h[(size_t)c * NB + b] : 0u;
    uint32_t inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) { const uint32_t y = __shfl_up(inc, o); if (lane >= (uint32_t)o) inc += y; }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t k = 0; k < wv; k++) base += wsum[k];
    if (c < nchunks) h[(size_t)c * NB + b] = base + inc - x;
    if (c == blockDim.x - 1) tot[b] = base + inc;
}

template <int DB, int W, int K, class V>
__global__ __launch_bounds__(W * 64) void k_pass(const uint32_t* kin, const V* vin, uint32_t* kout, V* vout, uint32_t n,
                                                 uint32_t chunk, uint32_t shift, const uint32_t* h, const uint32_t* tot) {
    constexpr int NB = 1 << DB, T = W * 64, TILE = W * K * 64, BPT = NB / T > 0 ? NB / T : 1;
    __shared__ uint16_t wc[W][NB];
    __shared__ uint16_t ttot[NB];
    __shared__ uint32_t run[NB];
    __shared__ uint32_t part[T];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // start[bin] = exclusive scan of the bin totals; run = start + this chunk's prefix
    {
        uint32_t loc[BPT], s = 0;
#pragma unroll
        for (int j = 0; j < BPT; j++) { const int b = tid * BPT + j; loc[j] = b < NB ? tot[b] : 0; s += loc[j]; }
        part[tid] = s;
        __syncthreads();
        for (int o = 1; o < T; o <<= 1) {           // Hillis-Steele over T partials
            const uint32_t x = tid >= o ? part[tid - o] : 0;
            __syncthreads();
            part[tid] += x;
            __syncthreads();
        }
        uint32_t acc = part[tid] - s;
#pragma unroll
        for (int j = 0; j < BPT; j++) {
            const int b = tid * BPT + j;
            if (b < NB) run[b] = acc + h[(size_t)blockIdx.x * NB + b];
            acc += loc[j];
        }
        for (int b = tid; b < NB; b += T) {
#pragma unroll
            for (int x = 0; x < W; x++) wc[x][b] = 0;
        }
        __syncthreads();
    }
    const uint64_t lo = (uint64_t)blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (uint64_t t0 = lo; t0 < hi; t0 += TILE) {
        uint32_t key[K];
        V val[K];
        uint16_t rk[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint64_t i = t0 + (uint64_t)(w * K + k) * 64 + lane;
            if (i < hi) { key[k] = kin[i]; val[k] = vin[i]; } else key[k] = 0;
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint64_t i = t0 + (uint64_t)(w * K + k) * 64 + lane;
            const bool ok = i < hi;
            const uint64_t act = __ballot(ok);
            if (!act) { rk[k] = 0; continue; }
            const uint32_t d = (key[k] >> shift) & (NB - 1);
            const uint64_t m = match_bits<DB>(d, act);
            const uint32_t before = ok ? wc[w][d] : 0;
            const uint32_t r = (uint32_t)__popcll(m & lt);
            rk[k] = (uint16_t)(before + r);
            if (ok && r == 0) wc[w][d] = (uint16_t)(before + __popcll(m));
        }
        __syncthreads();
        for (int b = tid; b < NB; b += T) {
            uint32_t acc = 0;
#pragma unroll
            for (int x = 0; x < W; x++) { const uint32_t c = wc[x][b]; wc[x][b] = (uint16_t)acc; acc += c; }
            ttot[b] = (uint16_t)acc;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint64_t i = t0 + (uint64_t)(w * K + k) * 64 + lane;
            if (i < hi) {
                const uint32_t d = (key[k] >> shift) & (NB - 1);
                const uint32_t dst = run[d] + wc[w][d] + rk[k];
                kout[dst] = key[k];
                vout[dst] = val[k];
            }
        }
        __syncthreads();
        for (int b = tid; b < NB; b += T) {
            run[b] += ttot[b];
#pragma unroll
            for (int x = 0; x < W; x++) wc[x][b] = 0;
        }
        __syncthreads();
    }
}

// LDS-staged variant: the tile's records are placed in LDS in (bin, rank)
// order first, then written out by consecutive threads, so every store
// instruction writes runs of consecutive addresses (one run per bin).
template <int DB, int W, int K, class V>
__global__ __launch_bounds__(W * 64) void k_pass_st(const uint32_t* kin, const V* vin, uint32_t* kout, V* vout,
                                                    uint32_t n, uint32_t chunk, uint32_t shift, const uint32_t* h,
                                                    const uint32_t* tot) {
    constexpr int NB = 1 << DB, T = W * 64, TILE = W * K * 64, BPT = NB / T > 0 ? NB / T : 1;
    __shared__ uint16_t wc[W][NB];
    __shared__ uint16_t ttot[NB];
    __shared__ uint16_t tstart[NB];
    __shared__ uint32_t run[NB];
    __shared__ uint32_t part[T];
    __shared__ uint32_t skey[TILE];
    __shared__ V sval[TILE];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    {
        uint32_t loc[BPT], s = 0;
#pragma unroll
        for (int j = 0; j < BPT; j++) { const int b = tid * BPT + j; loc[j] = b < NB ? tot[b] : 0; s += loc[j]; }
        part[tid] = s;
        __syncthreads();
        for (int o = 1; o < T; o <<= 1) {
            const uint32_t x = tid >= o ? part[tid - o] : 0;
            __syncthreads();
            part[tid] += x;
            __syncthreads();
        }
        uint32_t acc = part[tid] - s;
#pragma unroll
        for (int j = 0; j < BPT; j++) {
            const int b = tid * BPT + j;
            if (b < NB) run[b] = acc + h[(size_t)blockIdx.x * NB + b];
            acc += loc[j];
        }
        for (int b = tid; b < NB; b += T) {
#pragma unroll
            for (int x = 0; x < W; x++) wc[x][b] = 0;
        }
        __syncthreads();
    }
    const uint64_t lo = (uint64_t)blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (uint64_t t0 = lo; t0 < hi; t0 += TILE) {
        const uint32_t nt = (uint32_t)(hi - t0 < TILE ? hi - t0 : TILE);
        uint32_t key[K];
        V val[K];
        uint16_t rk[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint64_t i = t0 + (uint64_t)(w * K + k) * 64 + lane;
            if (i < hi) { key[k] = kin[i]; val[k] = vin[i]; } else key[k] = 0;
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint64_t i = t0 + (uint64_t)(w * K + k) * 64 + lane;
            const bool ok = i < hi;
            const uint64_t act = __ballot(ok);
            if (!act) { rk[k] = 0; continue; }
            const uint32_t d = (key[k] >> shift) & (NB - 1);
            const uint64_t m = match_bits<DB>(d, act);
            const uint32_t before = ok ? wc[w][d] : 0;
            const uint32_t r = (uint32_t)__popcll(m & lt);
            rk[k] = (uint16_t)(before + r);
            if (ok && r == 0) wc[w][d] = (uint16_t)(before + __popcll(m));
        }
        __syncthreads();
        for (int b = tid; b < NB; b += T) {
            uint32_t acc = 0;
#pragma unroll
            for (int x = 0; x < W; x++) { const uint32_t c = wc[x][b]; wc[x][b] = (uint16_t)acc; acc += c; }
            ttot[b] = (uint16_t)acc;
        }
        __syncthreads();
        {   // tile-local bin starts: exclusive scan of ttot
            uint32_t loc[BPT], s = 0;
#pragma unroll
            for (int j = 0; j < BPT; j++) { const int b = tid * BPT + j; loc[j] = b < NB ? ttot[b] : 0; s += loc[j]; }
            part[tid] = s;
            __syncthreads();
            for (int o = 1; o < T; o <<= 1) {
                const uint32_t x = tid >= o ? part[tid - o] : 0;
                __syncthreads();
                part[tid] += x;
                __syncthreads();
            }
            uint32_t acc = part[tid] - s;
#pragma unroll
            for (int j = 0; j < BPT; j++) {
                const int b = tid * BPT + j;
                if (b < NB) tstart[b] = (uint16_t)acc;
                acc += loc[j];
            }
            __syncthreads();
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint64_t i = t0 + (uint64_t)(w * K + k) * 64 + lane;
            if (i < hi) {
                const uint32_t d = (key[k] >> shift) & (NB - 1);
                const uint32_t p = tstart[d] + wc[w][d] + rk[k];
                skey[p] = key[k];
                sval[p] = val[k];
            }
        }
        __syncthreads();
        for (uint32_t p = tid; p < nt; p += T) {
            const uint32_t kk = skey[p];
            const uint32_t d = (kk >> shift) & (NB - 1);
            const uint32_t dst = run[d] + (p - tstart[d]);
            kout[dst] = kk;
            vout[dst] = sval[p];
        }
        __syncthreads();
        for (int b = tid; b < NB; b += T) {
            run[b] += ttot[b];
#pragma unroll
            for (int x = 0; x < W; x++) wc[x][b] = 0;
        }
        __syncthreads();
    }
}

struct Bufs { uint32_t *k0, *k1, *k2; uint64_t *v0, *v1, *v2; uint32_t *h, *tot; };

template <int DB, int W, int K, bool ST = false>
void lsd(Bufs& B, uint32_t n, uint32_t bits, uint32_t nchunks, hipStream_t s, uint32_t** kres, uint64_t** vres) {
    constexpr int NB = 1 << DB, TILE = W * K * 64;
    const int passes = (bits + DB - 1) / DB;
    uint32_t chunk = (n + nchunks - 1) / nchunks;
    chunk = (chunk + TILE - 1) / TILE * TILE;
    const uint32_t C = (n + chunk - 1) / chunk;
    const uint32_t* kin = B.k0; const uint64_t* vin = B.v0;
    uint32_t* ko[2] = {B.k1, B.k2}; uint64_t* vo[2] = {B.v1, B.v2};
    for (int p = 0; p < passes; p++) {
        const uint32_t shift = p * DB;
        hipLaunchKernelGGL((k_count<DB, 256>), dim3(C), dim3(256), 0, s, kin, n, chunk, shift, B.h);
        hipLaunchKernelGGL((k_scan_chunks<DB>), dim3(NB), dim3(1024), 0, s, B.h, C, B.tot);
        if constexpr (ST)
            hipLaunchKernelGGL((k_pass_st<DB, W, K, uint64_t>), dim3(C), dim3(W * 64), 0, s, kin, vin, ko[p & 1],
                               vo[p & 1], n, chunk, shift, B.h, B.tot);
        else
            hipLaunchKernelGGL((k_pass<DB, W, K, uint64_t>), dim3(C), dim3(W * 64), 0, s, kin, vin, ko[p & 1], vo[p & 1],
                               n, chunk, shift, B.h, B.tot);
        kin = ko[p & 1]; vin = vo[p & 1];
    }
    *kres = (uint32_t*)kin; *vres = (uint64_t*)vin;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : (1u << 27);
    const uint32_t R = argc > 2 ? (uint32_t)atol(argv[2]) : 10000000u;
    const uint32_t nchunks = argc > 3 ? (uint32_t)atol(argv[3]) : 512u;
    uint32_t bits = 1; while ((1ull << bits) < R) bits++;
    Bufs B;
    CK(hipMalloc(&B.k0, n * 4ull)); CK(hipMalloc(&B.k1, n * 4ull)); CK(hipMalloc(&B.k2, n * 4ull));
    CK(hipMalloc(&B.v0, n * 8ull)); CK(hipMalloc(&B.v1, n * 8ull)); CK(hipMalloc(&B.v2, n * 8ull));
    CK(hipMalloc(&B.h, (size_t)8192 * 4096 * 4)); CK(hipMalloc(&B.tot, 4096 * 4));
    hipLaunchKernelGGL(gen, dim3((n + 255) / 256), dim3(256), 0, 0, B.k0, B.v0, n, R, 7ull);
    CK(hipDeviceSynchronize());
    // reference: rocprim
    uint32_t* rk; uint64_t* rv;
    CK(hipMalloc(&rk, n * 4ull)); CK(hipMalloc(&rv, n * 8ull));
    size_t tb = 0;
    CK(rocprim::radix_sort_pairs(nullptr, tb, B.k0, rk, B.v0, rv, n, 0u, bits));
    void* tmp; CK(hipMalloc(&tmp, tb));
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const int reps = 5;
    float ms;
    CK(rocprim::radix_sort_pairs(tmp, tb, B.k0, rk, B.v0, rv, n, 0u, bits));
    hipEventRecord(a);
    for (int r = 0; r < reps; r++) CK(rocprim::radix_sort_pairs(tmp, tb, B.k0, rk, B.v0, rv, n, 0u, bits));
    hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    printf("n %u R %u bits %u chunks %u\n", n, R, bits, nchunks);
    printf("rocprim onesweep          %.3f ms\n", ms / reps);
    std::vector<uint32_t> hk(n), gk(n); std::vector<uint64_t> hv(n), gv(n);
    CK(hipMemcpy(hk.data(), rk, n * 4ull, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hv.data(), rv, n * 8ull, hipMemcpyDeviceToHost));
    {   // key histogram skew
        std::vector<uint32_t> c(R, 0); for (uint32_t i = 0; i < n; i++) c[hk[i]]++;
        uint32_t mx = 0; for (auto x : c) mx = x > mx ? x : mx;
        printf("top resource share %.3f\n", (double)mx / n);
    }
    auto check = [&](const char* name, uint32_t* k, uint64_t* v, float t) {
        CK(hipMemcpy(gk.data(), k, n * 4ull, hipMemcpyDeviceToHost));
        CK(hipMemcpy(gv.data(), v, n * 8ull, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint32_t i = 0; i < n; i++) bad += (gk[i] != hk[i]) | (gv[i] != hv[i]);
        printf("%-25s %.3f ms  mismatches %llu\n", name, t, (unsigned long long)bad);
    };
#define RUN(NAME, DB, W, K, ...)                                                             \
    {                                                                                      \
        uint32_t* ok; uint64_t* ov;                                                        \
        lsd<DB, W, K, ##__VA_ARGS__>(B, n, bits, nchunks, 0, &ok, &ov);                    \
        CK(hipDeviceSynchronize());                                                        \
        hipEventRecord(a);                                                                 \
        for (int r = 0; r < reps; r++) lsd<DB, W, K, ##__VA_ARGS__>(B, n, bits, nchunks, 0, &ok, &ov); \
        hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);         \
        check(NAME, ok, ov, ms / reps);                                                    \
    }
    RUN("lsd 12-bit W8 K16", 12, 8, 16);
    RUN("lsd 8-bit W4 K16", 8, 4, 16);
    RUN("staged 8-bit W8 K8", 8, 8, 8, true);
    RUN("staged 8-bit W8 K16", 8, 8, 16, true);
    RUN("staged 8-bit W4 K16", 8, 4, 16, true);
    RUN("staged 8-bit W16 K4", 8, 16, 4, true);
    RUN("staged 12-bit W4 K16", 12, 4, 16, true);
    // per-kernel breakdown of the 12-bit variant
    {
        uint32_t* ok; uint64_t* ov;
        hipEvent_t ev[8]; for (auto& e : ev) hipEventCreate(&e);
        constexpr int DB = 12, W = 4, K = 32, NB = 1 << DB, TILE = W * K * 64;
        uint32_t chunk = (n + nchunks - 1) / nchunks; chunk = (chunk + TILE - 1) / TILE * TILE;
        const uint32_t C = (n + chunk - 1) / chunk;
        const uint32_t* kin = B.k0; const uint64_t* vin = B.v0;
        uint32_t* ko[2] = {B.k1, B.k2}; uint64_t* vo[2] = {B.v1, B.v2};
        int e = 0;
        for (int p = 0; p < 2; p++) {
            hipEventRecord(ev[e++]);
            hipLaunchKernelGGL((k_count<DB, 256>), dim3(C), dim3(256), 0, 0, kin, n, chunk, p * DB, B.h);
            hipLaunchKernelGGL((k_scan_chunks<DB>), dim3(NB), dim3(1024), 0, 0, B.h, C, B.tot);
            hipEventRecord(ev[e++]);
            hipLaunchKernelGGL((k_pass<DB, W, K, uint64_t>), dim3(C), dim3(W * 64), 0, 0, kin, vin, ko[p], vo[p], n,
                               chunk, (uint32_t)(p * DB), B.h, B.tot);
            kin = ko[p]; vin = vo[p];
        }
        hipEventRecord(ev[e++]);
        CK(hipDeviceSynchronize());
        float t[4];
        for (int i = 0; i < 4; i++) hipEventElapsedTime(&t[i], ev[i], ev[i + 1]);
        printf("12-bit breakdown: count+scan0 %.3f pass0 %.3f count+scan1 %.3f pass1 %.3f ms\n", t[0], t[1], t[2], t[3]);
        (void)ok; (void)ov;
    }
    return 0;
}
