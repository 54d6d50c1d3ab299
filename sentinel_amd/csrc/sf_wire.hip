// sf_wire.hip — gfx950 kernels of sf_serve_frames (product code): the token
// server's inbound C1 frames of many connections decoded, decided and
// answered on the GPU.  See sf_wire.h for the reference pipeline it replaces
// and the three-step framing; sentinel_flow.h for the contract.
#include <cstdint>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "sf_wire.h"

namespace sf {

static inline unsigned wblocks(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

// largest s in [lo, hi] with soff[s] <= pos: the (non-empty) stream holding byte pos
__device__ __forceinline__ uint32_t stream_at(const uint64_t* soff, uint32_t lo, uint32_t hi, uint32_t pos) {
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if ((uint32_t)soff[mid] <= pos) lo = mid; else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ uint32_t rd32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
__device__ __forceinline__ uint64_t rd64(const uint8_t* p) { return ((uint64_t)rd32(p) << 32) | rd32(p + 4); }

// ---------------------------------------------------------------- framing
// (1) For every byte offset i of the tile: where a frame walk from i leaves
// the tile.  nx[i] = next frame start inside the tile, or i itself when the
// next start is outside the tile / past the stream end / the frame is
// incomplete (a root).  13 doublings reach the root (a path inside a
// 16-KiB tile has at most 8192 frames); the exit is the root's target.
constexpr unsigned WX_T = 512;
constexpr int WX_PER = WIRE_TILE / WX_T;

__global__ void __launch_bounds__(WX_T) k_wire_exit(WireBufs w) {
    __shared__ uint8_t b[WIRE_TILE + 4];
    __shared__ uint16_t nx[WIRE_TILE];
    const uint32_t base = blockIdx.x * WIRE_TILE;
    const uint32_t len = min(WIRE_TILE, w.n - base);
    const uint32_t lim = min(len + 1, w.n - base);          // + the byte after the tile (a straddling length field)
    for (uint32_t i = threadIdx.x; i < lim; i += WX_T) b[i] = w.bytes[base + i];
    const uint32_t s0 = stream_at(w.soff, 0, w.S - 1, base);
    const uint32_t s1 = stream_at(w.soff, s0, w.S - 1, base + len - 1);
    __syncthreads();
    uint16_t v[WX_PER];
#pragma unroll
    for (int k = 0; k < WX_PER; k++) {
        const uint32_t i = threadIdx.x + k * WX_T;
        uint16_t nv = (uint16_t)i;
        if (i < len) {
            const uint32_t abs = base + i;
            const uint32_t s = s0 == s1 ? s0 : stream_at(w.soff, s0, s1, abs);
            const uint32_t se = (uint32_t)w.soff[s + 1];
            if (abs + 2 <= se) {
                const uint32_t t = abs + 2 + (((uint32_t)b[i] << 8) | b[i + 1]);
                if (t < se && t < base + len) nv = (uint16_t)(t - base);
            }
        }
        v[k] = nv;
    }
#pragma unroll
    for (int k = 0; k < WX_PER; k++) nx[threadIdx.x + k * WX_T] = v[k];
    __syncthreads();
    for (int r = 0; r < 13; r++) {
#pragma unroll
        for (int k = 0; k < WX_PER; k++) v[k] = nx[nx[threadIdx.x + k * WX_T]];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < WX_PER; k++) nx[threadIdx.x + k * WX_T] = v[k];
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < WX_PER; k++) {
        const uint32_t i = threadIdx.x + k * WX_T;
        if (i >= len) continue;
        const uint32_t root = v[k];
        const uint32_t abs = base + root;
        const uint32_t s = s0 == s1 ? s0 : stream_at(w.soff, s0, s1, abs);
        const uint32_t se = (uint32_t)w.soff[s + 1];
        uint32_t t = WIRE_NONE;
        if (abs + 2 <= se) {
            t = abs + 2 + (((uint32_t)b[root] << 8) | b[root + 1]);
            if (t > se) t = WIRE_NONE;                       // incomplete frame: the walk stops there
        }
        w.exitv[base + i] = t;
    }
}

__global__ void k_wire_init(WireBufs w) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= w.S) return;
    const uint32_t se = (uint32_t)w.soff[s + 1];
    w.consumed[s] = se;
    w.stopoff[s] = se;
}

// (2) one lane per connection: the first frame start in each later tile
__global__ void k_wire_chain(WireBufs w) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= w.S) return;
    uint32_t e = (uint32_t)w.soff[s];
    const uint32_t se = (uint32_t)w.soff[s + 1];
    if (e >= se) return;
    e = w.exitv[e];
    while (e != WIRE_NONE && e < se) {
        w.tentry[e / WIRE_TILE] = e;
        e = w.exitv[e];
    }
}

// (3) walk each tile from its entries (the continuing connection's first
// frame, the starts of connections beginning in the tile), frame starts into
// an LDS bitmap; the incomplete last frame of a connection ends its prefix.
__global__ void __launch_bounds__(64) k_wire_walk(WireBufs w) {
    __shared__ uint8_t b[WIRE_TILE + 4];
    __shared__ uint32_t bm[WIRE_TILE / 32];
    const uint32_t base = blockIdx.x * WIRE_TILE;
    const uint32_t len = min(WIRE_TILE, w.n - base);
    const uint32_t lim = min(len + 1, w.n - base);
    const uint32_t lane = threadIdx.x;
    {   // 16-B loads where aligned, bytes for the tail
        const uint32_t nv = len / 16;
        const uint4* src = (const uint4*)(w.bytes + base);
        uint4* dst = (uint4*)b;
        if ((((uintptr_t)(w.bytes + base)) & 15) == 0) {
            for (uint32_t i = lane; i < nv; i += 64) dst[i] = src[i];
            for (uint32_t i = nv * 16 + lane; i < lim; i += 64) b[i] = w.bytes[base + i];
        } else {
            for (uint32_t i = lane; i < lim; i += 64) b[i] = w.bytes[base + i];
        }
    }
    for (uint32_t i = lane; i < WIRE_TILE / 32; i += 64) bm[i] = 0;
    const uint32_t s0 = stream_at(w.soff, 0, w.S - 1, base);
    const uint32_t s1 = stream_at(w.soff, s0, w.S - 1, base + len - 1);
    __syncthreads();
    const uint32_t first = (uint32_t)w.soff[s0] >= base ? s0 : s0 + 1;
    const uint32_t n_ent = 1 + (s1 >= first ? s1 - first + 1 : 0);
    for (uint32_t k = lane; k < n_ent; k += 64) {
        uint32_t p, s;
        if (k == 0) {
            p = w.tentry[blockIdx.x]; s = s0;
            if (p == WIRE_NONE) continue;
        } else {
            s = first + k - 1; p = (uint32_t)w.soff[s];
            if (p >= (uint32_t)w.soff[s + 1]) continue;     // empty connection
        }
        const uint32_t se = (uint32_t)w.soff[s + 1];
        const uint32_t pe = min(se, base + len);
        while (p < pe) {
            if (p + 2 > se) { w.consumed[s] = p; break; }
            const uint32_t i = p - base;
            const uint32_t t = p + 2 + (((uint32_t)b[i] << 8) | b[i + 1]);
            if (t > se) { w.consumed[s] = p; break; }
            atomicOr(&bm[i >> 5], 1u << (i & 31));
            p = t;
        }
    }
    __syncthreads();
    uint32_t c = 0;
    for (uint32_t i = lane; i < WIRE_TILE / 32; i += 64) {
        const uint32_t x = bm[i];
        w.bitmap[(size_t)blockIdx.x * (WIRE_TILE / 32) + i] = x;
        c += __popc(x);
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0) w.tcount[blockIdx.x] = c;
}

// frame list in offset order: one workgroup per tile, 2 bitmap words per thread
__global__ void __launch_bounds__(256) k_wire_emit(WireBufs w) {
    __shared__ uint32_t wsum[4];
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint32_t* bm = w.bitmap + (size_t)blockIdx.x * (WIRE_TILE / 32);
    const uint32_t x0 = bm[2 * t], x1 = bm[2 * t + 1];
    const uint32_t c = __popc(x0) + __popc(x1);
    uint32_t inc = c;                                        // inclusive wave scan
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t off = w.tbase[blockIdx.x] + inc - c;
    for (uint32_t k = 0; k < wv; k++) off += wsum[k];
    const uint32_t base = blockIdx.x * WIRE_TILE + 64 * t;
    for (uint32_t x = x0; x; x &= x - 1) w.frames[off++] = base + (uint32_t)__ffs(x) - 1;
    for (uint32_t x = x1; x; x &= x - 1) w.frames[off++] = base + 32 + (uint32_t)__ffs(x) - 1;
}

// ---------------------------------------------------------------- decode
// DefaultRequestEntityDecoder + the data decoders + the processor, for one
// frame body of L bytes (ClusterConstants: PING 0, FLOW 1, PARAM_FLOW 2;
// PARAM_TYPE_INTEGER 0, LONG 1, BYTE 2, DOUBLE 3, FLOAT 4, SHORT 5,
// BOOLEAN 6, STRING 7).  WC_HOST where the reference's outcome depends on
// more than this frame (sentinel_flow.h).
// The parameters of a PARAM_FLOW body (q: the data after xid and type, rem
// bytes; amount entries from offset 16): values written to tag / bits when
// given.  Returns how many decodeParam accepted, or -1 where the reference's
// outcome depends on more than the frame (bytes short or left over).
__device__ int wire_params(const uint8_t* q, uint32_t rem, int32_t amount, uint8_t* otag, uint64_t* obits) {
    uint32_t p = 16;
    int n = 0;
    for (int32_t k = 0; k < amount; k++) {
        if (p + 1 > rem) return -1;
        const uint8_t ty = q[p++];
        uint8_t tag = 0; uint64_t bits = 0; bool ok = true;
        switch (ty) {
        case 0: if (p + 4 > rem) return -1; tag = SF_TAG_INT; bits = (uint64_t)(int64_t)(int32_t)rd32(q + p); p += 4; break;
        case 1: if (p + 8 > rem) return -1; tag = SF_TAG_LONG; bits = rd64(q + p); p += 8; break;
        case 2: if (p + 1 > rem) return -1; tag = SF_TAG_BYTE; bits = (uint64_t)(int64_t)(int8_t)q[p]; p += 1; break;
        case 3: {
            if (p + 8 > rem) return -1;
            uint64_t x = rd64(q + p); p += 8;
            if ((x & 0x7ff0000000000000ULL) == 0x7ff0000000000000ULL && (x & 0x000fffffffffffffULL))
                x = 0x7ff8000000000000ULL;                   // Double.equals: doubleToLongBits
            tag = SF_TAG_DOUBLE; bits = x; break;
        }
        case 4: {
            if (p + 4 > rem) return -1;
            uint32_t x = rd32(q + p); p += 4;
            if ((x & 0x7f800000u) == 0x7f800000u && (x & 0x007fffffu)) x = 0x7fc00000u;   // floatToIntBits
            tag = SF_TAG_FLOAT; bits = x; break;
        }
        case 5: if (p + 2 > rem) return -1; tag = SF_TAG_SHORT;
            bits = (uint64_t)(int64_t)(int16_t)(((uint32_t)q[p] << 8) | q[p + 1]); p += 2; break;
        case 6: if (p + 1 > rem) return -1; tag = SF_TAG_BOOL; bits = q[p] != 0; p += 1; break;
        case 7: {
            if (p + 4 > rem) return -1;
            const int32_t sl = (int32_t)rd32(q + p); p += 4;
            if (sl < 0 || (uint32_t)sl > rem - p) return -1;
            uint64_t h = 0xcbf29ce484222325ULL;              // sf_string_key: FNV-1a 64
            for (int32_t j = 0; j < sl; j++) { h ^= q[p + j]; h *= 0x100000001b3ULL; }
            tag = SF_TAG_STRING; bits = h; p += (uint32_t)sl; break;
        }
        default: ok = false;                                 // decodeParam returns false
        }
        if (ok) {
            if (otag) { otag[n] = tag; obits[n] = bits; }
            n++;
        }
    }
    return p == rem ? n : -1;
}

__device__ uint8_t wire_decode_body(const uint8_t* b, uint32_t L, WFrame& f, uint32_t* nval) {
    if (L == 0) return WC_NONE;                              // nothing readable
    if (L < 5) return WC_HOST;                               // decode() null, bytes stay cumulated
    f.xid = (int32_t)rd32(b);
    const int8_t type = (int8_t)b[4];
    f.type = (uint8_t)type;
    const uint8_t* q = b + 5;
    const uint32_t rem = L - 5;
    if (type == 1) {                                         // FlowRequestDataDecoder
        if (rem == 0) return WC_NONE;                        // null data: NPE in FlowRequestProcessor :39
        if (rem < 12 || rem > 13) return WC_HOST;
        f.flow_id = (int64_t)rd64(q);
        f.count = (int32_t)rd32(q + 8);
        f.flags = (rem == 13 && q[12] != 0) ? SF_TOK_PRIORITIZED : 0;
        return WC_REQ;
    }
    if (type == 2) {                                         // ParamFlowRequestDataDecoder
        if (rem == 0) return WC_NONE;
        if (rem < 16) return WC_HOST;
        f.flow_id = (int64_t)rd64(q);
        f.count = (int32_t)rd32(q + 8);
        const int32_t amount = (int32_t)rd32(q + 12);
        if (amount <= 0) return rem == 16 ? WC_NONE : WC_HOST;
        if ((uint32_t)amount > rem - 16) return WC_HOST;    // each parameter reads >= 1 byte
        const int n = wire_params(q, rem, amount, nullptr, nullptr);
        if (n < 0) return WC_HOST;
        if (n == 0) return WC_BAD;                           // requestParamToken: params.isEmpty()
        *nval = (uint32_t)n;                                 // one Collection (the decoder's ArrayList)
        f.flags = SF_TOK_PARAM;
        return WC_REQ;
    }
    if (rem == 0 && type != 0) return WC_NONE;               // no decoder: null message, nothing left
    return WC_HOST;                                          // PING / no decoder with bytes left
}

__global__ void k_wire_class(WireBufs w, uint32_t nf) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nf) return;
    const uint32_t p = w.frames[f];
    const uint32_t s = stream_at(w.soff, 0, w.S - 1, p);
    const uint32_t L = ((uint32_t)w.bytes[p] << 8) | w.bytes[p + 1];
    WFrame x{};
    x.stream = s;
    uint32_t nv = 0;
    x.cls = L + 2 > SF_WIRE_MAX_FRAME ? WC_SKIP : wire_decode_body(w.bytes + p + 2, L, x, &nv);
    w.wf[f] = x;
    w.nval[f] = x.cls == WC_REQ ? nv : 0u;
    if (x.cls == WC_HOST) atomicMin(&w.stopoff[s], p);
}

__global__ void k_wire_flags(WireBufs w, uint32_t nf) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nf) return;
    const WFrame& x = w.wf[f];
    const bool active = w.frames[f] < w.stopoff[x.stream];
    const uint64_t rq = active && x.cls == WC_REQ;
    const uint64_t rs = active && (x.cls == WC_REQ || x.cls == WC_BAD);
    w.fl[f] = (rq << 32) | rs;
}

__global__ void k_wire_compact(WireBufs w, uint32_t nf, int64_t now_ms) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nf || !(w.fl[f] >> 32)) return;
    const uint32_t r = (uint32_t)(w.pos[f] >> 32);
    const WFrame x = w.wf[f];
    w.q_fid[r] = x.flow_id; w.q_cnt[r] = x.count; w.q_flags[r] = x.flags; w.q_ts[r] = now_ms;
    w.q_nval[r] = w.nval[f];
}
// parameters of each PARAM_FLOW request at q_poff[r] (decoded again from its frame)
__global__ void k_wire_values(WireBufs w, uint32_t nf) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nf || !(w.fl[f] >> 32) || !w.nval[f]) return;
    const uint32_t r = (uint32_t)(w.pos[f] >> 32);
    const uint32_t p = w.frames[f];
    const uint32_t L = ((uint32_t)w.bytes[p] << 8) | w.bytes[p + 1];
    const uint8_t* q = w.bytes + p + 2 + 5;
    const uint32_t o = w.q_poff[r];
    wire_params(q, L - 5, (int32_t)rd32(q + 12), w.q_tag + o, w.q_bits + o);
}

// response frames (LengthFieldPrepender(2) + DefaultResponseEntityWriter + FlowResponseDataWriter)
__global__ void k_wire_encode(WireBufs w, uint32_t nf) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nf || !(w.fl[f] & 0xffffffffu)) return;
    const WFrame x = w.wf[f];
    int8_t status = SF_TOKEN_BAD_REQUEST;
    int32_t rem = 0, wait = 0;
    if (x.cls == WC_REQ) {
        const uint32_t r = (uint32_t)(w.pos[f] >> 32);
        status = w.r_status[r]; rem = w.r_rem[r];
        wait = (x.flags & SF_TOK_PARAM) ? 0 : w.r_wait[r];   // ParamFlowRequestProcessor: setWaitInMs(0)
    }
    union { uint8_t c[16]; uint4 v; } o;
    o.c[0] = 0; o.c[1] = 14;
    o.c[2] = (uint8_t)(x.xid >> 24); o.c[3] = (uint8_t)(x.xid >> 16); o.c[4] = (uint8_t)(x.xid >> 8); o.c[5] = (uint8_t)x.xid;
    o.c[6] = x.type; o.c[7] = (uint8_t)status;
    o.c[8] = (uint8_t)(rem >> 24); o.c[9] = (uint8_t)(rem >> 16); o.c[10] = (uint8_t)(rem >> 8); o.c[11] = (uint8_t)rem;
    o.c[12] = (uint8_t)(wait >> 24); o.c[13] = (uint8_t)(wait >> 16); o.c[14] = (uint8_t)(wait >> 8); o.c[15] = (uint8_t)wait;
    ((uint4*)w.resp)[(uint32_t)w.pos[f]] = o.v;
}

// first frame index at or after byte offset p
__device__ __forceinline__ uint32_t frame_lb(const uint32_t* frames, uint32_t nf, uint32_t p) {
    uint32_t lo = 0, hi = nf;
    while (lo < hi) { const uint32_t mid = (lo + hi) >> 1; if (frames[mid] < p) lo = mid + 1; else hi = mid; }
    return lo;
}

// per connection: handled prefix, stop reason, response range, handled frames
__global__ void k_wire_final(WireBufs w, uint32_t nf) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s > w.S) return;
    const uint64_t tot = nf ? w.pos[nf - 1] + w.fl[nf - 1] : 0;
    const uint32_t lo = frame_lb(w.frames, nf, s < w.S ? (uint32_t)w.soff[s] : w.n);
    w.resp_scan[s] = lo < nf ? (uint32_t)w.pos[lo] : (uint32_t)tot;
    if (s == w.S) return;
    const uint32_t ss = (uint32_t)w.soff[s], se = (uint32_t)w.soff[s + 1];
    const uint32_t stop = w.stopoff[s], cons = w.consumed[s];
    w.stop[s] = stop < se ? SF_WIRE_HOST : (cons < se ? SF_WIRE_PARTIAL : SF_WIRE_DONE);
    const uint32_t end = min(stop, cons);
    w.consumed_rel[s] = end - ss;
    const uint32_t hi = frame_lb(w.frames, nf, end);
    if (hi > lo) atomicAdd(&w.counters[0], hi - lo);
}

// ---------------------------------------------------------------- host side
hipError_t wire_query_temp(uint32_t n_tiles, uint32_t S, uint32_t max_frames, size_t* bytes) {
    size_t a = 0, b = 0;
    hipError_t e = rocprim::exclusive_scan(nullptr, a, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)n_tiles + 1,
                                           rocprim::plus<uint32_t>());
    if (e != hipSuccess) return e;
    e = rocprim::exclusive_scan(nullptr, b, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint64_t)0,
                                (size_t)std::max<uint32_t>(max_frames, 1), rocprim::plus<uint64_t>());
    if (e != hipSuccess) return e;
    size_t c = 0;
    e = rocprim::exclusive_scan(nullptr, c, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)max_frames + 1,
                                rocprim::plus<uint32_t>());
    *bytes = std::max(std::max(a, b), c);
    (void)S;
    return e;
}

hipError_t wire_frame(const WireBufs& w, hipStream_t s) {
    hipMemsetAsync(w.tentry, 0xff, (size_t)w.n_tiles * 4, s);
    hipMemsetAsync(w.tcount, 0, ((size_t)w.n_tiles + 1) * 4, s);
    hipMemsetAsync(w.counters, 0, 16, s);
    hipLaunchKernelGGL(k_wire_init, dim3(wblocks(w.S, 256)), dim3(256), 0, s, w);
    hipLaunchKernelGGL(k_wire_exit, dim3(w.n_tiles), dim3(WX_T), 0, s, w);
    hipLaunchKernelGGL(k_wire_chain, dim3(wblocks(w.S, 64)), dim3(64), 0, s, w);
    hipLaunchKernelGGL(k_wire_walk, dim3(w.n_tiles), dim3(64), 0, s, w);
    size_t tb = w.tmp_bytes;
    hipError_t e = rocprim::exclusive_scan(w.tmp, tb, w.tcount, w.tbase, 0u, (size_t)w.n_tiles + 1,
                                           rocprim::plus<uint32_t>(), s);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t wire_decode(const WireBufs& w, uint32_t nf, int64_t now_ms, hipStream_t s) {
    (void)now_ms;
    if (!nf) return hipSuccess;
    hipLaunchKernelGGL(k_wire_emit, dim3(w.n_tiles), dim3(256), 0, s, w);
    hipLaunchKernelGGL(k_wire_class, dim3(wblocks(nf, 256)), dim3(256), 0, s, w, nf);
    hipLaunchKernelGGL(k_wire_flags, dim3(wblocks(nf, 256)), dim3(256), 0, s, w, nf);
    size_t tb = w.tmp_bytes;
    hipError_t e = rocprim::exclusive_scan(w.tmp, tb, w.fl, w.pos, (uint64_t)0, (size_t)nf, rocprim::plus<uint64_t>(), s);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t wire_compact(const WireBufs& w, uint32_t nf, uint32_t n_req, int64_t now_ms, hipStream_t s) {
    if (!nf) return hipSuccess;
    hipMemsetAsync(w.q_nval + n_req, 0, 4, s);
    hipLaunchKernelGGL(k_wire_compact, dim3(wblocks(nf, 256)), dim3(256), 0, s, w, nf, now_ms);
    size_t tb = w.tmp_bytes;
    hipError_t e = rocprim::exclusive_scan(w.tmp, tb, w.q_nval, w.q_poff, 0u, (size_t)n_req + 1,
                                           rocprim::plus<uint32_t>(), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_wire_values, dim3(wblocks(nf, 256)), dim3(256), 0, s, w, nf);
    return hipGetLastError();
}

hipError_t wire_encode(const WireBufs& w, uint32_t nf, hipStream_t s) {
    if (nf) hipLaunchKernelGGL(k_wire_encode, dim3(wblocks(nf, 256)), dim3(256), 0, s, w, nf);
    hipLaunchKernelGGL(k_wire_final, dim3(wblocks((size_t)w.S + 1, 256)), dim3(256), 0, s, w, nf);
    return hipGetLastError();
}

}  // namespace sf
