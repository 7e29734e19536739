// rt_codec.hip -- lossless 8x8-tile codec for the band sets shipped to rank 0.
//
// The multi-GPU path gathers every frame to rank 0 over xGMI; at 1080p that transfer, not
// the trace, bounds strong scaling.  Each rank encodes its band sets before
// the gather and rank 0 decodes them straight into the frame.  The format is specified, and
// mirrored on the host, in raytracer_hip/tilecodec.py.  In short, per 8x8 tile of a band set
// (lane l = ry*8 + rx): pixel (0,0) raw in the tile's 4-byte header beside its width code;
// per channel mod 256 the second differences r = dx - dx(row above), dx = p - p(left) (column 0:
// p - p(0,0); row 0: r = dx) -- decoded by a prefix sum over the rows (3 DPP steps across the
// tile's lanes) and one along each row (registers); zigzag; widths rounded up to 0/2/3/4/6/8
// bits, lane-packed.  Tiles are grouped in chunks of 8; a tile's payload lives at its chunk's
// base + the units of the chunk's earlier tiles (a wave scan of the headers).
//
// Encode = two launches per batch of frames (deterministic layout, no atomics), chunks of 8
// tiles = one wave's, contiguous ranges of chunks per workgroup:
//   encode_tiles_kernel  residuals, widths, packed segments (into the context's staging slot
//                        of 48 words per tile, final byte layout), tile headers; chunk totals
//                        -> chunk_base[], range totals -> wg_total[]
//   encode_copy_kernel   range base = sum of the earlier ranges' totals, chunk bases by an LDS
//                        scan, staged segments -> compact offsets (chunk-relative offsets by a
//                        wave scan of the headers); wire header and size
// Decode = one launch for every rank's wire of a batch (decode_tiles_kernel).
// Integer/byte work: the encoder reads each band-set pixel once (4 B), the decoder writes
// each frame pixel once (4 B); both are instruction-lean (DPP row shifts, ballots, inverse
// ballots) so that they stay near those HBM bytes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "rt_codec_common.h"
#include "rt_internal.h"

namespace rtk {

#ifndef RT_ENC_BLOCKS
#define RT_ENC_BLOCKS 2048
#endif
constexpr int CODEC_BLOCKS = RT_ENC_BLOCKS;  // encode grid: 256 CUs x 8 workgroups of 4 waves
constexpr int CODEC_MAX_PER = 1024;  // chunks per workgroup at most (LDS of the copy pass)

// Wave index inside the workgroup, as a scalar: what derives from it stays wave-uniform.
__device__ __forceinline__ int wave_index() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

__device__ __forceinline__ uint32_t* wire_chunk_base(unsigned char* w, const CodecGeom& g) {
    return (uint32_t*)(w + 16 + 4 * (size_t)g.n_tiles);
}
__device__ __forceinline__ const uint32_t* wire_chunk_base(const unsigned char* w, const CodecGeom& g) {
    return (const uint32_t*)(w + 16 + 4 * (size_t)g.n_tiles);
}
__device__ __forceinline__ uint64_t* wire_payload(unsigned char* w, const CodecGeom& g) {
    return (uint64_t*)(w + g.fixed_bytes);
}
__device__ __forceinline__ const uint64_t* wire_payload(const unsigned char* w, const CodecGeom& g) {
    return (const uint64_t*)(w + g.fixed_bytes);
}

// RT_ENC_DPP: the encoder's cross-lane steps without LDS round trips (ds_bpermute): the tile's
// first pixel by a quad broadcast + a 4-lane shift into the upper quad, the tile OR as an
// all-lanes butterfly (quad xor 1, quad xor 2, half-row mirror), the chunk-relative offsets
// as a DPP wave scan (row shifts + row broadcasts) of the group totals.
#ifndef RT_ENC_DPP
#define RT_ENC_DPP 1
#endif

// Local row r of band set `rank` -> frame row.
__device__ __forceinline__ int frame_row(const CodecGeom& g, int rank, int r) {
    return (rank + (r / g.band_rows) * g.world) * g.band_rows + r % g.band_rows;
}

// Both directions use one layout: lane L = 8 j + ry of a wave handles row ry (8 pixels) of
// tile t0 + j of a group of CODEC_TPW = 8 consecutive tiles (= one chunk).  A row's residuals
// of one channel are then the w consecutive bytes [ry*w, ry*w + w) of the channel's segment,
// the left-neighbour prediction / prefix runs in registers, the first column needs only the
// lane above (DPP row shift by one) and the tile's first pixel (one bpermute), and a tile's
// OR of residuals is a 3-step DPP OR inside its 8 lanes.

// Tile position of this lane's tile (t0 + j): t0's by scalar divisions, then stepping
// (tiles_x >= 8 wraps at most once; narrow frames loop).
struct TilePos {
    int f, tr, tc;
};
__device__ __forceinline__ TilePos tile_pos(const CodecGeom& g, int t0, int j) {
    const int f0 = t0 / g.tiles_per_frame;
    const int tt0 = t0 - f0 * g.tiles_per_frame;
    const int tr0 = tt0 / g.tiles_x;
    TilePos p{f0, tr0, tt0 - tr0 * g.tiles_x + j};
    while (p.tc >= g.tiles_x) {
        p.tc -= g.tiles_x;
        if (++p.tr == g.tiles_y) p.tr = 0, ++p.f;
    }
    return p;
}

// Encode one group of CODEC_TPW tiles (one chunk): tile headers with chunk-relative offsets,
// the chunk total into chunk_base[chunk], the non-flat tiles' segments into their staging
// slots (STAGE_WORDS per tile, final byte layout).  Returns the chunk total (units).
// A lane's tile row of a chunk: its 8 pixels (0 outside the frame) and how many exist.
struct EncRow {
    uint32_t p[8];
    int ncols;
};
__device__ __forceinline__ EncRow encode_load(const int32_t* __restrict__ bands, const CodecGeom& g, int chunk,
                                              int lane) {
    const int t0 = chunk * CODEC_TPW;
    const int j = lane >> 3, ry = lane & 7;
    const bool live = t0 + j < g.n_tiles;
    const TilePos tp = tile_pos(g, t0, j);
    const int r = tp.tr * 8 + ry;
    const bool row_ok = live && r < g.n_bands * g.band_rows && frame_row(g, g.rank, r) < g.H;
    const int x0 = tp.tc * 8;
    const int ncols = row_ok ? min(8, g.W - x0) : 0;
    const int32_t* src = bands + (size_t)tp.f * g.frame_stride + (size_t)r * (size_t)g.W + (size_t)x0;
    EncRow e;
    e.ncols = ncols;
    uint32_t* p = e.p;
    if (ncols == 8 && ((uintptr_t)src & 15) == 0) {
        const int4 a = ((const int4*)src)[0], b = ((const int4*)src)[1];
        p[0] = (uint32_t)a.x, p[1] = (uint32_t)a.y, p[2] = (uint32_t)a.z, p[3] = (uint32_t)a.w;
        p[4] = (uint32_t)b.x, p[5] = (uint32_t)b.y, p[6] = (uint32_t)b.z, p[7] = (uint32_t)b.w;
    } else {
#pragma unroll
        for (int rx = 0; rx < 8; ++rx) p[rx] = rx < ncols ? (uint32_t)src[rx] : 0u;
    }
#pragma unroll
    for (int rx = 0; rx < 8; ++rx) p[rx] &= 0xffffffu;  // pixels outside the frame are 0
    return e;
}

__device__ __forceinline__ uint32_t encode_group(unsigned char* __restrict__ wire, uint32_t* __restrict__ stage,
                                                 const CodecGeom& g, int chunk, int lane, const EncRow& e) {
    const int t0 = chunk * CODEC_TPW;
    const int j = lane >> 3, ry = lane & 7;
    const int t = t0 + j;
    const bool live = t < g.n_tiles;
    const int ncols = e.ncols;
    const uint32_t* p = e.p;
    // residuals: second differences (dx along the row, column 0 against the tile's first pixel;
    // then minus the row above's dx, rows >= 1)
    const uint32_t first = RT_ENC_DPP ? group8_first(p[0]) : (uint32_t)__shfl((int)p[0], lane & ~7, 64);
    uint32_t z[8];
#pragma unroll
    for (int rx = 0; rx < 8; ++rx) {
        const uint32_t dx = sub_bytes(p[rx], rx ? p[rx - 1] : first);
        const uint32_t above = row_shr<1>(dx);  // (lane - 1 = the row above for ry >= 1)
        const uint32_t r = ry ? sub_bytes(dx, above) : dx;
        z[rx] = rx < ncols ? zigzag_bytes(r) & 0xffffffu : 0u;
    }
    // tile OR of residuals -> width indices, broadcast over the tile's lanes
    uint32_t o = z[0] | z[1] | z[2] | z[3] | z[4] | z[5] | z[6] | z[7];
    if constexpr (RT_ENC_DPP) {
        o = group8_or(o);
    } else {
        o |= row_shr<1>(o);
        o |= row_shr<2>(o);
        o |= row_shr<4>(o);
        o = (uint32_t)__shfl((int)o, lane | 7, 64);
    }
    const uint32_t iR = width_index((o >> 16) & 0xffu), iG = width_index((o >> 8) & 0xffu),
                   iB = width_index(o & 0xffu);
    const uint32_t code = live ? iR + 6u * iG + 36u * iB : 0u;
    const uint32_t wm = live ? width_at(iR) | (width_at(iG) << 4) | (width_at(iB) << 8) : 0u;
    // chunk total: with each group's units in its lane 8j+7 only, an inclusive wave scan
    const uint32_t u7 = ry == 7 ? units_of(wm) : 0u;
    const uint32_t incl = wave_scan_incl(u7);
    if (live && ry == 0) wire_tile_hdr(wire)[t] = first | (code << 24);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (lane == 63) wire_chunk_base(wire, g)[chunk] = total;  // chunk total, scanned later
    // segments: this row's residuals of channel c = bytes [ry*w, ry*w + w) of the segment
    if (wm & 0xfffu) {
        unsigned char* seg = (unsigned char*)(stage + (size_t)t * STAGE_WORDS);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const uint32_t w = (wm >> (4 * c)) & 15u;
            const int sh = 16 - 8 * c;
            uint64_t acc = 0;
#pragma unroll
            for (int rx = 0; rx < 8; ++rx) acc |= (uint64_t)((z[rx] >> sh) & 0xffu) << (rx * w);
            store_row_bits(seg + ry * w, w, acc);
            seg += 8 * w;
        }
    }
    return total;
}

// Workgroup b owns the contiguous chunks [b * per, (b + 1) * per) (its waves take every 4th),
// and leaves the sum of their totals in wg_total[b]: the copy pass then finds every chunk's
// base from those sums and its own chunks -- no single-workgroup scan of all chunks.
__global__ __launch_bounds__(256) void encode_tiles_kernel(const int32_t* __restrict__ bands,
                                                          unsigned char* __restrict__ wire,
                                                          uint32_t* __restrict__ stage,
                                                          uint32_t* __restrict__ wg_total, CodecGeom g, int per) {
    __shared__ uint32_t s_tot[4];
    const int lane = threadIdx.x & 63, wave = wave_index();
    const int lo = blockIdx.x * per, hi = min(g.n_chunks, lo + per);
    uint32_t mine = 0;
    for (int chunk = lo + wave; chunk < hi; chunk += 4)
        mine += encode_group(wire, stage, g, chunk, lane, encode_load(bands, g, chunk, lane));
    if (lane == 0) s_tot[wave] = mine;
    __syncthreads();
    if (threadIdx.x == 0) wg_total[blockIdx.x] = s_tot[0] + s_tot[1] + s_tot[2] + s_tot[3];
}

// After traces with OUT_TILES (the encoder fused into rt_kernel.hip): the chunk totals from the
// tile headers alone (the encode_tiles_kernel ranges and outputs, no band-set read).  Tile rows
// >= traced_rows of a frame were not traced: their headers are zeroed here.
__global__ __launch_bounds__(256) void chunk_totals_kernel(unsigned char* __restrict__ wire,
                                                          uint32_t* __restrict__ wg_total, CodecGeom g, int per,
                                                          int traced_rows) {
    __shared__ uint32_t s_tot[4];
    const int lane = threadIdx.x & 63, wave = wave_index();
    const int j = lane >> 3, ry = lane & 7;
    const int lo = blockIdx.x * per, hi = min(g.n_chunks, lo + per);
    uint32_t mine = 0;
    for (int chunk = lo + wave; chunk < hi; chunk += 4) {
        const int t = chunk * CODEC_TPW + j;
        uint32_t hdr = 0;
        if (t < g.n_tiles) {
            uint32_t* h = wire_tile_hdr(wire) + t;
            if ((t % g.tiles_per_frame) / g.tiles_x < traced_rows) hdr = *h;
            else if (ry == 0) *h = 0u;
        }
        const uint32_t u7 = ry == 7 ? units_of(widths_of_code(hdr >> 24)) : 0u;
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_incl(u7), 63);
        if (lane == 63) wire_chunk_base(wire, g)[chunk] = total;
        mine += total;
    }
    if (lane == 0) s_tot[wave] = mine;
    __syncthreads();
    if (threadIdx.x == 0) wg_total[blockIdx.x] = s_tot[0] + s_tot[1] + s_tot[2] + s_tot[3];
}

// Inclusive scan of x over the 256 threads (LDS, Hillis-Steele); returns it, *sum = total.
__device__ __forceinline__ uint32_t block_scan256(uint32_t x, uint32_t* s, uint32_t* sum) {
    const int tid = threadIdx.x;
    s[tid] = x;
    __syncthreads();
#pragma unroll
    for (int k = 1; k < 256; k <<= 1) {
        const uint32_t o = tid >= k ? s[tid - k] : 0u;
        __syncthreads();
        s[tid] += o;
        __syncthreads();
    }
    const uint32_t r = s[tid];
    *sum = s[255];
    __syncthreads();
    return r;
}

// One chunk's staged segments -> compact payload: lane 8j + q moves units q, q+8, q+16 of
// tile t0 + j (loads first, then stores).  Converged call (the wave scan).
__device__ __forceinline__ void copy_group(const uint64_t* __restrict__ stage, unsigned char* __restrict__ wire,
                                           const CodecGeom& g, int chunk, uint32_t base, int lane) {
    const int t = chunk * CODEC_TPW + (lane >> 3), q = lane & 7;
    const bool live = t < g.n_tiles;
    const uint32_t u = live ? units_of(widths_of_code(wire_tile_hdr(wire)[t] >> 24)) : 0u;
    // offset inside the chunk: the units of the chunk's earlier tiles (wave scan, as the encoder)
    const uint32_t u7 = q == 7 ? u : 0u;
    const uint32_t incl = wave_scan_incl(u7);
    const uint32_t rel = q == 7 ? incl - u7 : incl;
    uint64_t* pay = wire_payload(wire, g);
    uint64_t v[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) v[k] = q + 8 * k < (int)u ? stage[(size_t)t * STAGE_UNITS + q + 8 * k] : 0ull;
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (q + 8 * k < (int)u) pay[(size_t)base + rel + q + 8 * k] = v[k];
}

// Same workgroup ranges as encode_tiles_kernel: the base of workgroup b's chunks is the sum of
// wg_total[0..b); its chunk totals (in chunk_base[]) are scanned in LDS and replaced by their
// bases; then the staged segments move to their compact offsets.  The last workgroup writes
// the wire header and size.
__global__ __launch_bounds__(256) void encode_copy_kernel(const uint64_t* __restrict__ stage,
                                                         unsigned char* __restrict__ wire,
                                                         const uint32_t* __restrict__ wg_total, CodecGeom g, int per,
                                                         int64_t* __restrict__ wire_bytes) {
    __shared__ uint32_t s_scan[256];
    __shared__ uint32_t s_base[CODEC_MAX_PER];
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_index();
    const int b = blockIdx.x;
    const int lo = b * per, hi = min(g.n_chunks, lo + per);
    uint32_t pre = 0;  // sum of the earlier workgroups' totals
    for (int i = tid; i < b; i += 256) pre += wg_total[i];
    uint32_t sum;
    block_scan256(pre, s_scan, &sum);
    uint32_t run = sum;
    uint32_t* cb = wire_chunk_base(wire, g);
    for (int k0 = lo; k0 < hi; k0 += 256) {
        const int c = k0 + tid;
        const uint32_t x = c < hi ? cb[c] : 0u;
        uint32_t tot;
        const uint32_t incl = block_scan256(x, s_scan, &tot);
        if (c < hi) s_base[c - lo] = run + incl - x;
        run += tot;
    }
    __syncthreads();
    for (int c = lo + tid; c < hi; c += 256) cb[c] = s_base[c - lo];
    for (int chunk = lo + wave; chunk < hi; chunk += 4) copy_group(stage, wire, g, chunk, s_base[chunk - lo], lane);
    if (b == (int)gridDim.x - 1 && tid == 0) {
        const uint32_t total = run;
        uint32_t* h = (uint32_t*)wire;
        h[0] = total;
        h[1] = (uint32_t)g.n_tiles;
        h[2] = (uint32_t)g.n_chunks;
        h[3] = (uint32_t)g.tiles_per_frame;
        if (wire_bytes) *wire_bytes = (int64_t)(g.fixed_bytes + 8 * (size_t)total);
        const size_t used = 16 + 4 * (size_t)g.n_tiles + 4 * (size_t)g.n_chunks;
        if (used < g.fixed_bytes) *(uint32_t*)(wire + used) = 0u;  // padding to 8 bytes
    }
}

// Decoder layout: lane L = 8 j + ry handles row ry (8 pixels) of tile t0 + j, so a row's
// residuals of one channel are the w consecutive bytes [ry*w, ry*w + w) of the segment (one
// aligned 8-byte load), the prefix along the row runs in registers, and the first column
// needs only the lane above (DPP row shift by one).  A wave decodes one chunk.
constexpr int DEC_TPW = CODEC_TPW;
// decode grid: 4096 workgroups of 4 waves (4 per SIMD; 2048 / 8192 / 16384: +7 / +2 / +14 %)
#ifndef RT_DEC_BLOCKS
#define RT_DEC_BLOCKS 4096
#endif
#ifndef RT_DEC_NT
#define RT_DEC_NT 1
#endif
#ifndef RT_DEC_LDS
#define RT_DEC_LDS 1
#endif

// A group's header words, loaded one group ahead of its decode: the header load of group i+1
// overlaps the payload loads and arithmetic of group i.
struct DecHead {
    const unsigned char* wire;
    int rank, t0;
    uint32_t hdr;   // this lane's tile: first pixel | width code << 24
    uint32_t base;  // the chunk's unit offset
};
__device__ __forceinline__ DecHead decode_head(const unsigned char* __restrict__ gathered, size_t rank_stride,
                                               const CodecGeom& g, int groups, size_t gw, int lane) {
    DecHead h;
    const int rel_rank = (int)(gw / (size_t)groups);
    h.t0 = (int)(gw - (size_t)rel_rank * groups) * DEC_TPW;
    h.rank = g.rank + rel_rank;
    h.wire = gathered + (size_t)h.rank * rank_stride;
    const int t = h.t0 + (lane >> 3);
    h.hdr = wire_tile_hdr(h.wire)[t < g.n_tiles ? t : 0];
    h.base = wire_chunk_base(h.wire, g)[h.t0 / CODEC_TPW];  // the wave's chunk
    return h;
}

__device__ __forceinline__ void decode_group(int32_t* __restrict__ frames, const CodecGeom& g, const DecHead& h,
                                             int lane) {
    const int rank = h.rank, t0 = h.t0;
    const unsigned char* wire = h.wire;
    const int total_bands = (g.H + g.band_rows - 1) / g.band_rows;
    const int nb = rank < total_bands ? (total_bands - 1 - rank) / g.world + 1 : 0;
    const int j = lane >> 3, ry = lane & 7;
    const int t = t0 + j;
    const bool live = t < g.n_tiles;
    const uint32_t first = live ? h.hdr & 0xffffffu : 0u;
    const uint32_t wm = live ? widths_of_code(h.hdr >> 24) : 0u;
    const uint32_t u = units_of(wm);
    // the tile's offset inside the chunk: the units of the chunk's earlier tiles (wave scan)
    const uint32_t u7 = ry == 7 ? u : 0u;
    const uint32_t incl = wave_scan_incl(u7);
    const uint32_t rel = ry == 7 ? incl - u7 : incl;
    const TilePos tp = tile_pos(g, t0, j);
    const int f = tp.f, tr = tp.tr, tc = tp.tc;
    const int r = tr * 8 + ry;
    const int y = frame_row(g, rank, r);
    const bool row_ok = live && r < nb * g.band_rows && y < g.H;
    const int x0 = tc * 8;
    const uint64_t* pay = wire_payload(wire, g);
    uint32_t d[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = 0u;
    if (__builtin_amdgcn_ballot_w64(u != 0) != 0) {  // some tile of the wave is not flat
        uint32_t seg = h.base + rel;  // unit offset of the channel's segment
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const uint32_t wc = (wm >> (4 * c)) & 15u;
            uint64_t bits = 0;
            if (wc) {  // this row's wc bytes [ry*wc, ry*wc + wc) of the segment: one or two loads
                const uint32_t byte = (uint32_t)ry * wc, sb = byte & 7u;
                const uint64_t* src = pay + seg + (byte >> 3);
                const uint64_t lo = src[0];
                const uint64_t hi = sb + wc > 8u ? src[1] : 0ull;  // (never past the segment)
                bits = sb ? (lo >> (8 * sb)) | (hi << (64 - 8 * sb)) : lo;
            }
            const uint32_t mask = (1u << wc) - 1u;
#pragma unroll
            for (int rx = 0; rx < 8; ++rx)
                d[rx] |= ((uint32_t)(bits >> (rx * wc)) & mask) << (16 - 8 * c);
            seg += wc;
        }
#pragma unroll
        for (int rx = 0; rx < 8; ++rx) d[rx] = unzigzag_bytes(d[rx]) & 0xffffffu;
        // prefix over the tile's rows (lanes 8j..8j+7): Hillis-Steele, 3 row shifts
#pragma unroll
        for (int rx = 0; rx < 8; ++rx) {
            uint32_t v = d[rx];
            const uint32_t s1 = row_shr<1>(v);
            v = ry >= 1 ? add_bytes(v, s1) : v;
            const uint32_t s2 = row_shr<2>(v);
            v = ry >= 2 ? add_bytes(v, s2) : v;
            const uint32_t s4 = row_shr<4>(v);
            v = ry >= 4 ? add_bytes(v, s4) : v;
            d[rx] = v & 0xffffffu;
        }
    }
    // then along the row: column 0 holds p(0, ry) - first, columns >= 1 p(x) - p(x-1)
    uint32_t px[8];
    px[0] = add_bytes(first, d[0]) & 0xffffffu;
#pragma unroll
    for (int rx = 1; rx < 8; ++rx) px[rx] = add_bytes(px[rx - 1], d[rx]) & 0xffffffu;
    // A group of 8 tiles of one tile row, inside the width, on 16-byte aligned rows (wave-uniform;
    // every group of a frame whose width is a multiple of 64): the wave's 8 rows x 64 pixels go
    // through LDS so that each store instruction writes whole row segments (8 lanes x 16 B =
    // 128 B of one row) instead of 16-byte pieces 32 bytes apart (RT_DEC_LDS).
    if constexpr (RT_DEC_LDS) {
        const int tc0 = __builtin_amdgcn_readfirstlane(tc);  // lane 0: j = 0
        const bool full = t0 + DEC_TPW <= g.n_tiles && tc0 + DEC_TPW <= g.tiles_x && (tc0 + DEC_TPW) * 8 <= g.W &&
                          (g.W & 3) == 0 && (g.frame_stride & 3) == 0 && ((uintptr_t)frames & 15) == 0;
        if (full) {
            __shared__ uint4 xch[4][8][16];  // [wave][row][16 B]
            uint4(*rows)[16] = xch[wave_index()];
            rows[ry][2 * j] = make_uint4(px[0], px[1], px[2], px[3]);
            rows[ry][2 * j + 1] = make_uint4(px[4], px[5], px[6], px[7]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint4 a = rows[ry][j], b = rows[ry][8 + j];
            __builtin_amdgcn_wave_barrier();  // (the next group's writes come after these reads)
            if (row_ok) {
                uint4* dst = (uint4*)(frames + (size_t)f * g.frame_stride + (size_t)y * (size_t)g.W + (size_t)tc0 * 8);
                if constexpr (RT_DEC_NT) {
                    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                    __builtin_nontemporal_store(u32x4{a.x, a.y, a.z, a.w}, (u32x4*)(dst + j));
                    __builtin_nontemporal_store(u32x4{b.x, b.y, b.z, b.w}, (u32x4*)(dst + 8 + j));
                } else {
                    dst[j] = a;
                    dst[8 + j] = b;
                }
            }
            return;
        }
    }
    if (!row_ok) return;
    int32_t* dst = frames + (size_t)f * g.frame_stride + (size_t)y * (size_t)g.W + (size_t)x0;
    if (x0 + 8 <= g.W && ((uintptr_t)dst & 15) == 0) {
        ((int4*)dst)[0] = make_int4((int)px[0], (int)px[1], (int)px[2], (int)px[3]);
        ((int4*)dst)[1] = make_int4((int)px[4], (int)px[5], (int)px[6], (int)px[7]);
    } else {
#pragma unroll
        for (int rx = 0; rx < 8; ++rx)
            if (x0 + rx < g.W) dst[rx] = (int32_t)px[rx];
    }
}

// Decode the wires of ranks g.rank .. world-1 (rank r's at gathered + r * rank_stride) of a
// batch into the frames (frame f at frames + f * frame_stride): a resident grid of 4-wave
// workgroups walks the (rank, 8-tile group) pairs.
__global__ __launch_bounds__(256) void decode_tiles_kernel(const unsigned char* __restrict__ gathered,
                                                          size_t rank_stride, int32_t* __restrict__ frames,
                                                          CodecGeom g) {
    const int lane = threadIdx.x & 63;
    const int groups = (g.n_tiles + DEC_TPW - 1) / DEC_TPW;  // per rank
    const size_t n = (size_t)(g.world - g.rank) * (size_t)groups;  // ranks g.rank .. world-1
    const size_t stride = (size_t)gridDim.x * 4;
    size_t gw = (size_t)blockIdx.x * 4 + wave_index();
    if (gw >= n) return;  // wave-uniform
    DecHead h = decode_head(gathered, rank_stride, g, groups, gw, lane);
    for (;;) {
        const size_t nx = gw + stride;
        DecHead hn = h;
        if (nx < n) hn = decode_head(gathered, rank_stride, g, groups, nx, lane);  // prefetch
        decode_group(frames, g, h, lane);
        if (nx >= n) break;
        gw = nx;
        h = hn;
    }
}

int launch_encode_bands(const int32_t* bands, unsigned char* wire, const CodecGeom& g, int64_t* wire_bytes,
                        void* stage, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    // workgroups of 4 waves over contiguous chunk ranges: a resident-size grid (short waves are
    // launch-rate bound), at most CODEC_MAX_PER chunks per workgroup
    long long blocks = std::min<long long>((g.n_chunks + 3) / 4, CODEC_BLOCKS);
    int per = (int)((g.n_chunks + blocks - 1) / blocks);
    if (per > CODEC_MAX_PER) per = CODEC_MAX_PER;
    blocks = (g.n_chunks + per - 1) / per;
    uint32_t* st = (uint32_t*)stage;
    uint32_t* wg_total = st + (size_t)g.n_chunks * CODEC_TPW * STAGE_WORDS;
    hipLaunchKernelGGL(encode_tiles_kernel, dim3((unsigned)blocks), dim3(256), 0, s, bands, wire, st, wg_total, g, per);
    hipLaunchKernelGGL(encode_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const uint64_t*)st, wire,
                       (const uint32_t*)wg_total, g, per, wire_bytes);
    return (int)hipGetLastError();
}

int launch_finish_wire(unsigned char* wire, const CodecGeom& g, int traced_tile_rows, int64_t* wire_bytes,
                       void* stage, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    long long blocks = std::min<long long>((g.n_chunks + 3) / 4, CODEC_BLOCKS);  // as launch_encode_bands
    int per = (int)((g.n_chunks + blocks - 1) / blocks);
    if (per > CODEC_MAX_PER) per = CODEC_MAX_PER;
    blocks = (g.n_chunks + per - 1) / per;
    uint32_t* st = (uint32_t*)stage;
    uint32_t* wg_total = st + (size_t)g.n_chunks * CODEC_TPW * STAGE_WORDS;
    hipLaunchKernelGGL(chunk_totals_kernel, dim3((unsigned)blocks), dim3(256), 0, s, wire, wg_total, g, per,
                       traced_tile_rows);
    hipLaunchKernelGGL(encode_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const uint64_t*)st, wire,
                       (const uint32_t*)wg_total, g, per, wire_bytes);
    return (int)hipGetLastError();
}

size_t encode_stage_bytes(const CodecGeom& g) {
    const long long blocks = std::max<long long>(1, std::min<long long>((g.n_chunks + 3) / 4, CODEC_BLOCKS));
    const long long per = std::min<long long>(CODEC_MAX_PER, (g.n_chunks + blocks - 1) / blocks);
    const long long nb = (g.n_chunks + per - 1) / per;
    return ((size_t)g.n_chunks * CODEC_TPW * STAGE_WORDS + (size_t)nb) * sizeof(uint32_t);
}

int launch_decode_gathered(const unsigned char* gathered, size_t rank_stride, int32_t* frames, const CodecGeom& g,
                           void* stream) {
    const size_t waves = (size_t)(g.world - g.rank) * (size_t)((g.n_tiles + DEC_TPW - 1) / DEC_TPW);
    if (waves == 0) return (int)hipSuccess;
    hipLaunchKernelGGL(decode_tiles_kernel, dim3((unsigned)std::min<size_t>((waves + 3) / 4, RT_DEC_BLOCKS)), dim3(256), 0,
                       (hipStream_t)stream,
                       gathered, rank_stride, frames, g);
    return (int)hipGetLastError();
}

}  // namespace rtk
