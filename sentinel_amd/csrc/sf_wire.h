// sf_wire.h — token-server wire path (product code): C1 frames of many
// connections in, TokenService decisions, response frames out (sf_serve_frames).
//
// Reference (CS = sentinel-cluster/sentinel-cluster-server-default/src/main/java/com/alibaba/csp/sentinel/cluster):
//   NettyTransportServer.java:84-101   pipeline: LengthFieldBasedFrameDecoder(1024,0,2,0,2),
//                                      NettyRequestDecoder, LengthFieldPrepender(2), NettyResponseEncoder
//   codec/DefaultRequestEntityDecoder.java:42-63, codec/data/FlowRequestDataDecoder.java:37-48,
//   codec/data/ParamFlowRequestDataDecoder.java:35-90, handler/TokenServerHandler.java:61-82,
//   processor/FlowRequestProcessor.java:36-52, processor/ParamFlowRequestProcessor.java:38-54,
//   codec/DefaultResponseEntityWriter.java:35-52, codec/data/FlowResponseDataWriter.java:30-33
//
// Framing is a pointer chase (each frame's 2-byte length gives the next frame
// start).  It is made parallel in three steps over 16-KiB tiles of the byte
// buffer: (1) k_wire_exit resolves, for EVERY byte offset of a tile at once,
// where a frame walk starting there leaves the tile (pointer doubling in LDS);
// (2) k_wire_chain follows those exits, one lane per connection, one step per
// tile; (3) k_wire_walk walks each tile from its known entries, marking frame
// starts in an LDS bitmap.  Frames are then decoded one per lane, compacted
// into a token batch by one scan, decided by the token service kernels
// (sf_token.hip) and encoded in place.
#pragma once
#include "sf_token.h"

namespace sf {

constexpr uint32_t WIRE_TILE = 16384;           // bytes per framing tile
constexpr uint32_t WIRE_NONE = 0xffffffffu;

enum : uint8_t { WC_NONE = 0, WC_REQ = 1, WC_BAD = 2, WC_HOST = 3, WC_SKIP = 4 };

struct WFrame {                 // one decoded frame, 32 B
    int64_t flow_id;
    uint64_t bits;
    int32_t xid;
    int32_t count;
    uint32_t stream;
    uint8_t cls, type, flags, tag;
};

struct WireBufs {
    const uint8_t* bytes; const uint64_t* soff;   // input (device)
    uint32_t n, S, n_tiles;
    uint32_t* exitv;            // [n]
    uint32_t* tentry;           // [n_tiles]
    uint32_t* bitmap;           // [n_tiles * WIRE_TILE / 32]
    uint32_t* tcount;           // [n_tiles + 1] -> exclusive scan in tbase
    uint32_t* tbase;            // [n_tiles + 1]
    uint32_t* consumed;         // [S] absolute end of the handled prefix (partial frame start or stream end)
    uint32_t* stopoff;          // [S] first frame the host must handle (or stream end)
    uint32_t* resp_cnt;         // [S + 1] -> exclusive scan in resp_scan
    uint32_t* resp_scan;        // [S + 1]
    uint32_t* frames;           // [max frames] frame start offsets, ascending
    WFrame* wf;                 // [max frames]
    uint64_t* fl;               // [max frames] (request << 32 | response) flags, then their exclusive scan in pos
    uint64_t* pos;
    uint32_t* counters;         // [0] frames handled
    // token batch built from the frames (capacity = max frames)
    int64_t* q_fid; int32_t* q_cnt; uint8_t* q_flags; int64_t* q_ts; uint8_t* q_tag; uint64_t* q_bits;
    // parameter Collection of each request: q_poff (exclusive scan of q_nval), values in q_tag / q_bits
    uint32_t* nval;             // [max frames] decoded parameters of a PARAM_FLOW frame (0 otherwise)
    uint32_t* q_nval;           // [max frames + 1]
    uint32_t* q_poff;           // [max frames + 1]
    int8_t* r_status; int32_t* r_rem; int32_t* r_wait;
    uint8_t* resp;              // [max frames * 16]
    uint8_t* stop;              // [S]
    uint64_t* consumed_rel;     // [S]
    void* tmp; size_t tmp_bytes;
};

// scratch bytes rocprim needs for the scans of sf_serve_frames
hipError_t wire_query_temp(uint32_t n_tiles, uint32_t S, uint32_t max_frames, size_t* bytes);
// framing: exits, chains, walks, per-tile counts and their scan (tbase[n_tiles] = frames)
hipError_t wire_frame(const WireBufs& w, hipStream_t s);
// frame list, decode, stop offsets, request/response ranks (pos[nf-1] + fl[nf-1] = totals)
hipError_t wire_decode(const WireBufs& w, uint32_t nf, int64_t now_ms, hipStream_t s);
// token batch arrays of the requests (n_req of them), parameters as one CSR
hipError_t wire_compact(const WireBufs& w, uint32_t nf, uint32_t n_req, int64_t now_ms, hipStream_t s);
// response frames and per-stream results
hipError_t wire_encode(const WireBufs& w, uint32_t nf, hipStream_t s);

}  // namespace sf
