// rt_codec.hip -- lossless 8x8-tile codec for the band sets shipped to rank 0.
//
// The multi-GPU path gathers every frame to rank 0 over xGMI; at 1080p that transfer, not
// the trace, bounds strong scaling.  Each rank encodes its band sets before
// the gather and rank 0 decodes them straight into the frame.  The format is specified, and
// mirrored on the host, in raytracer_hip/tilecodec.py.  In short, per 8x8 tile of a band set
// (lane l = ry*8 + rx of one wave64): pixel (0,0) raw in the tile header; every other pixel
// predicted by its left neighbour, the first column by the pixel above (odd rows) or by the
// tile's first pixel (even rows) -- predictors a DPP row shift or a scalar can deliver; per
// channel residuals mod 256, zigzag; widths rounded up to 0/1/2/4/8 bits, lane-packed.
// Tiles are grouped in chunks of 64; a tile's payload lives at its chunk's base + its offset
// inside the chunk.
//
// Encode = two launches per batch of frames (deterministic layout, no atomics), chunks of 16
// tiles = one wave's, contiguous ranges of chunks per workgroup:
//   encode_tiles_kernel  residuals, widths, packed segments (into the context's staging slot
//                        of 48 words per tile), chunk-relative offsets -> tile headers; chunk
//                        totals -> chunk_base[] (in place), range totals -> wg_total[]
//   encode_copy_kernel   range base = sum of the earlier ranges' totals, chunk bases by an LDS
//                        scan, staged segments -> compact offsets; wire header and size
// Decode = one launch for every rank's wire of a batch (decode_tiles_kernel).
// Integer/byte work: the encoder reads each band-set pixel once (4 B), the decoder writes
// each frame pixel once (4 B); both are instruction-lean (DPP row shifts, ballots, inverse
// ballots) so that they stay near those HBM bytes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "rt_internal.h"

namespace rtk {

constexpr int CODEC_TPW = 16;    // tiles per wave = tiles per chunk
constexpr int CODEC_BLOCKS = 2048;   // resident grid: 256 CUs x 8 workgroups of 4 waves
constexpr int CODEC_MAX_PER = 1024;  // chunks per workgroup at most (LDS of the copy pass)
constexpr int STAGE_WORDS = 48;  // staging words per tile (3 channels x 8 bits x 64 lanes / 32)

// Wave index inside the workgroup, as a scalar: what derives from it stays wave-uniform.
__device__ __forceinline__ int wave_index() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

__device__ __forceinline__ const uint32_t* wire_tile_hdr(const unsigned char* w) { return (const uint32_t*)(w + 16); }
__device__ __forceinline__ uint32_t* wire_tile_hdr(unsigned char* w) { return (uint32_t*)(w + 16); }
__device__ __forceinline__ uint32_t* wire_chunk_base(unsigned char* w, const CodecGeom& g) {
    return (uint32_t*)(w + 16 + 8 * (size_t)g.n_tiles);
}
__device__ __forceinline__ const uint32_t* wire_chunk_base(const unsigned char* w, const CodecGeom& g) {
    return (const uint32_t*)(w + 16 + 8 * (size_t)g.n_tiles);
}
__device__ __forceinline__ uint64_t* wire_payload(unsigned char* w, const CodecGeom& g) {
    return (uint64_t*)(w + g.fixed_bytes);
}
__device__ __forceinline__ const uint64_t* wire_payload(const unsigned char* w, const CodecGeom& g) {
    return (const uint64_t*)(w + g.fixed_bytes);
}

// Byte-wise (mod 256 per byte) add / subtract of packed 0x00RRGGBB values.
__device__ __forceinline__ uint32_t add_bytes(uint32_t a, uint32_t b) {
    return ((a & 0x7f7f7f7fu) + (b & 0x7f7f7f7fu)) ^ ((a ^ b) & 0x80808080u);
}
__device__ __forceinline__ uint32_t sub_bytes(uint32_t a, uint32_t b) {
    return ((a | 0x80808080u) - (b & 0x7f7f7f7fu)) ^ ((a ^ ~b) & 0x80808080u);
}
// zigzag of each byte read as int8: 0, -1, 1, -2, ... -> 0, 1, 2, 3, ...
__device__ __forceinline__ uint32_t zigzag_bytes(uint32_t d) {
    const uint32_t neg = (d >> 7) & 0x01010101u;      // sign bit of each byte
    return ((d << 1) & 0xfefefefeu) ^ (neg * 0xffu);  // (s << 1) ^ (s >> 7) per byte
}
__device__ __forceinline__ uint32_t unzigzag_bytes(uint32_t z) {
    const uint32_t odd = z & 0x01010101u;
    return ((z >> 1) & 0x7f7f7f7fu) ^ (odd * 0xffu);  // (z >> 1) ^ -(z & 1) per byte
}

// DPP row shift right by N lanes inside each 16-lane row (0 shifted in).
template <int N>
__device__ __forceinline__ uint32_t row_shr(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 + N, 0xf, 0xf, true);
}

__device__ __forceinline__ uint32_t bitlen8(uint32_t v) { return v ? 32u - (uint32_t)__builtin_clz(v) : 0u; }
__device__ __forceinline__ uint32_t units_of(uint32_t wm) { return (wm & 15u) + ((wm >> 4) & 15u) + ((wm >> 8) & 15u); }

// Local row r of band set `rank` -> frame row.
__device__ __forceinline__ int frame_row(const CodecGeom& g, int rank, int r) {
    return (rank + (r / g.band_rows) * g.world) * g.band_rows + r % g.band_rows;
}

// Per-tile bookkeeping is lane-parallel: lane j (< CODEC_TPW) of a wave describes tile t0 + j
// of its chunk (frame, tile row / column, where its pixels live, which are inside the frame),
// and the tile loop fetches what it needs with readlane -- so the scalar unit, which all waves
// of a CU share, stays nearly idle.  When band_rows % 8 == 0 (the shipped 8) a tile lies
// inside one band: its frame rows are y0 + ry and a pixel is inside iff rx < x_lim and
// ry < y_lim; otherwise every pixel maps its own row (generic path).
struct TileInfo {
    int tr;        // tile row (generic path)
    int x_lim;     // columns inside the frame: rx < x_lim
    int y_lim;     // rows inside (band_rows % 8 == 0): ry < y_lim
    int64_t src;   // element offset of the tile's pixel (0, 0) in the band sets
    int64_t dst;   // element offset of the tile's pixel (0, 0) in the frames (band_rows % 8 == 0)
    bool live;     // t0 + j < n_tiles
};
__device__ __forceinline__ TileInfo tile_info(const CodecGeom& g, int rank, int nb, int t) {
    TileInfo ti;
    ti.live = t < g.n_tiles;
    const int tc0 = ti.live ? t : 0;
    const int f = tc0 / g.tiles_per_frame;
    const int tt = tc0 - f * g.tiles_per_frame;
    ti.tr = tt / g.tiles_x;
    const int tc = tt - ti.tr * g.tiles_x;
    const int r0 = ti.tr * 8;
    ti.x_lim = g.W - tc * 8;
    ti.src = (int64_t)f * (int64_t)g.frame_stride + (int64_t)r0 * g.W + tc * 8;
    ti.y_lim = 0, ti.dst = 0;
    if ((g.band_rows & 7) == 0) {
        const int k = r0 / g.band_rows;
        const int y0 = (rank + k * g.world) * g.band_rows + (r0 - k * g.band_rows);
        ti.y_lim = min(nb * g.band_rows - r0, g.H - y0);
        ti.dst = (int64_t)f * (int64_t)g.frame_stride + (int64_t)y0 * g.W + tc * 8;
    } else {
        ti.dst = (int64_t)f * (int64_t)g.frame_stride + tc * 8;  // + y * W per pixel
    }
    if (!ti.live) ti.x_lim = 0, ti.y_lim = 0;
    return ti;
}
__device__ __forceinline__ int64_t readlane64(int64_t v, int j) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, j);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), j);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
// This lane's pixel of tile j (lane-parallel info `ti`): inside the frame?  *y_off = the
// element offset of its frame row relative to the tile's dst (generic path: absolute row).
__device__ __forceinline__ bool pixel_inside(const CodecGeom& g, int rank, int nb, const TileInfo& ti, int j, int lane,
                                             int64_t* row_off) {
    const int rx = lane & 7, ry = lane >> 3;
    const int x_lim = __builtin_amdgcn_readlane(ti.x_lim, j);
    if ((g.band_rows & 7) == 0) {
        const int y_lim = __builtin_amdgcn_readlane(ti.y_lim, j);
        *row_off = (int64_t)ry * g.W;
        return rx < x_lim && ry < y_lim;
    }
    const int r = __builtin_amdgcn_readlane(ti.tr, j) * 8 + ry;
    const int y = frame_row(g, rank, r);
    *row_off = (int64_t)y * g.W;
    return rx < x_lim && r < nb * g.band_rows && y < g.H;
}

// Zigzag residuals (packed 0x00RRGGBB) of this lane's pixel v (0 outside the frame; a valid
// pixel's predictor is valid too); converged wave call.
__device__ __forceinline__ uint32_t tile_residual(uint32_t v, bool valid, int lane, uint32_t first) {
    const uint32_t left = row_shr<1>(v), above = row_shr<8>(v);
    const uint32_t pred = (lane & 7) ? left : ((lane & 8) ? above : first);
    return valid ? zigzag_bytes(sub_bytes(v, pred)) & 0xffffffu : 0u;
}

// OR of z over the wave (DPP OR-scan inside each 16-lane row, then the four row totals).
__device__ __forceinline__ uint32_t wave_or(uint32_t z) {
    z |= row_shr<1>(z);
    z |= row_shr<2>(z);
    z |= row_shr<4>(z);
    z |= row_shr<8>(z);
    return (uint32_t)__builtin_amdgcn_readlane((int)z, 15) | (uint32_t)__builtin_amdgcn_readlane((int)z, 31) |
           (uint32_t)__builtin_amdgcn_readlane((int)z, 47) | (uint32_t)__builtin_amdgcn_readlane((int)z, 63);
}
// Width of a channel: bit length of its OR rounded up to 0, 1, 2, 4 or 8.
__device__ __forceinline__ uint32_t width_of(uint32_t o) {
    return o == 0 ? 0u : o < 2 ? 1u : o < 4 ? 2u : o < 16 ? 4u : 8u;
}

// DPP quad permutations (inside each group of 4 lanes).
__device__ __forceinline__ uint32_t quad_swap1(uint32_t v) {  // [1,0,3,2]
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t quad_swap2(uint32_t v) {  // [2,3,0,1]
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false);
}

// Pack channel values x (0..2^w-1, this lane's) of width w into 2w words at seg: lane l's
// bits at l*w of the stream.  A word gathers 32/w lanes (a DPP OR inside the group), the
// group's last lane stores it.  Converged wave call, w in {1, 2, 4, 8} (wave-uniform).
__device__ __forceinline__ void pack_segment(uint32_t* __restrict__ seg, uint32_t x, uint32_t w, int lane) {
    if (w == 1) {
        const uint64_t m = __builtin_amdgcn_ballot_w64(x != 0);
        if (lane < 2) seg[lane] = lane == 0 ? (uint32_t)m : (uint32_t)(m >> 32);
        return;
    }
    uint32_t y = x << ((lane * w) & 31);
    y |= quad_swap1(y);
    y |= quad_swap2(y);  // every lane: its quad's OR (w = 8: one word per quad)
    if (w <= 4) y |= row_shr<4>(y);  // lanes 8k+7: the OR of their 8 lanes (w = 4: one word)
    if (w == 2) y |= row_shr<8>(y);  // lanes 16k+15: the OR of their 16 lanes
    const int group = 32 / (int)w;
    if ((lane & (group - 1)) == group - 1) seg[lane / group] = y;
}

// One wave per chunk of CODEC_TPW consecutive tiles, their loads issued together
// (unconditional loads from a safe address for pixels outside the frame: no branch, no wait).
// Writes the tile headers with chunk-relative offsets, the chunk total into chunk_base[]
// (scanned next) and the non-flat tiles' segments into their staging slots.
__device__ __forceinline__ uint32_t encode_chunk(const int32_t* __restrict__ bands, unsigned char* __restrict__ wire,
                                                 uint32_t* __restrict__ stage, const CodecGeom& g, int chunk, int lane) {
    const int t0 = chunk * CODEC_TPW;
    const TileInfo ti = tile_info(g, g.rank, g.n_bands, t0 + (lane & (CODEC_TPW - 1)));
    uint32_t v[CODEC_TPW];
    bool ok[CODEC_TPW];
    const int64_t lane_off = (int64_t)(lane >> 3) * g.W + (lane & 7);
#pragma unroll
    for (int j = 0; j < CODEC_TPW; ++j) {
        int64_t row_off;
        ok[j] = pixel_inside(g, g.rank, g.n_bands, ti, j, lane, &row_off);
        const int64_t off = readlane64(ti.src, j) + lane_off;
        const uint32_t raw = (uint32_t)bands[ok[j] ? off : 0];
        v[j] = ok[j] ? raw & 0xffffffu : 0u;
    }
    uint32_t z[CODEC_TPW];
    uint32_t lane_first = 0, lane_or = 0;  // lane j: tile j's first pixel / OR of residuals
#pragma unroll
    for (int j = 0; j < CODEC_TPW; ++j) {
        const uint32_t first = (uint32_t)__builtin_amdgcn_readfirstlane((int)v[j]);  // lane 0 (0 if outside)
        z[j] = tile_residual(v[j], ok[j], lane, first);
        const uint32_t o = wave_or(z[j]);
        if (lane == j) lane_first = first, lane_or = o;
    }
    // lane-parallel over the chunk's tiles: widths, units, chunk-relative offsets
    const uint32_t wm = width_of((lane_or >> 16) & 0xffu) | (width_of((lane_or >> 8) & 0xffu) << 4) |
                        (width_of(lane_or & 0xffu) << 8);
    const uint32_t u = lane < CODEC_TPW ? units_of(wm) : 0u;
    uint32_t incl = u;  // inclusive prefix over lanes 0..15 (DPP row 0)
    uint32_t o = row_shr<1>(incl);
    incl += o;
    o = row_shr<2>(incl);
    incl += o;
    o = row_shr<4>(incl);
    incl += o;
    o = row_shr<8>(incl);
    incl += o;
    const uint32_t meta = wm | ((incl - u) << 12);
    if (lane < CODEC_TPW && ti.live) {
        uint32_t* h = wire_tile_hdr(wire) + 2 * (size_t)(t0 + lane);
        h[0] = lane_first;
        h[1] = meta;
    }
    if (lane == CODEC_TPW - 1) wire_chunk_base(wire, g)[chunk] = incl;  // chunk total
    // segments of the non-flat tiles -> staging slot (48 words per tile)
#pragma unroll
    for (int j = 0; j < CODEC_TPW; ++j) {
        const uint32_t mj = (uint32_t)__builtin_amdgcn_readlane((int)meta, j);
        if ((mj & 0xfffu) == 0) continue;  // flat tile (wave-uniform)
        uint32_t* seg = stage + (size_t)(t0 + j) * STAGE_WORDS;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const uint32_t w = (mj >> (4 * c)) & 15u;
            if (w == 0) continue;
            pack_segment(seg, (z[j] >> (16 - 8 * c)) & 0xffu, w, lane);
            seg += 2 * w;
        }
    }
    return (uint32_t)__builtin_amdgcn_readlane((int)incl, CODEC_TPW - 1);
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
    for (int chunk = lo + wave; chunk < hi; chunk += 4) mine += encode_chunk(bands, wire, stage, g, chunk, lane);
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

__device__ __forceinline__ void copy_chunk(const uint32_t* __restrict__ stage, unsigned char* __restrict__ wire,
                                           const CodecGeom& g, int chunk, uint32_t base, int lane) {
    const int t0 = chunk * CODEC_TPW;
    const bool hv = lane < CODEC_TPW && t0 + lane < g.n_tiles;
    const uint32_t meta = hv ? wire_tile_hdr(wire)[2 * (size_t)(t0 + lane) + 1] : 0u;
    uint32_t* pay = (uint32_t*)wire_payload(wire, g);
    uint32_t words[CODEC_TPW];
#pragma unroll
    for (int j = 0; j < CODEC_TPW; ++j) {  // non-flat tiles only; words past a tile's units are unused
        const uint32_t mj = (uint32_t)__builtin_amdgcn_readlane((int)meta, j);
        words[j] = 0u;
        if (mj & 0xfffu) words[j] = stage[(size_t)(t0 + j) * STAGE_WORDS + min(lane, STAGE_WORDS - 1)];
    }
#pragma unroll
    for (int j = 0; j < CODEC_TPW; ++j) {
        const uint32_t mj = (uint32_t)__builtin_amdgcn_readlane((int)meta, j);
        if (lane < 2 * (int)units_of(mj)) pay[2 * ((size_t)base + (mj >> 12)) + lane] = words[j];
    }
}

// Same workgroup ranges as encode_tiles_kernel: the base of workgroup b's chunks is the sum of
// wg_total[0..b); its chunk totals (in chunk_base[]) are scanned in LDS and replaced by their
// bases; then the staged segments move to their compact offsets (one wave per chunk, word q
// of a tile by lane q).  The last workgroup writes the wire header and size.
__global__ __launch_bounds__(256) void encode_copy_kernel(const uint32_t* __restrict__ stage,
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
    for (int chunk = lo + wave; chunk < hi; chunk += 4) copy_chunk(stage, wire, g, chunk, s_base[chunk - lo], lane);
    if (b == (int)gridDim.x - 1 && tid == 0) {
        const uint32_t total = run;
        uint32_t* h = (uint32_t*)wire;
        h[0] = total;
        h[1] = (uint32_t)g.n_tiles;
        h[2] = (uint32_t)g.n_chunks;
        h[3] = (uint32_t)g.tiles_per_frame;
        if (wire_bytes) *wire_bytes = (int64_t)(g.fixed_bytes + 8 * (size_t)total);
        const size_t used = 16 + 8 * (size_t)g.n_tiles + 4 * (size_t)g.n_chunks;
        if (used < g.fixed_bytes) *(uint32_t*)(wire + used) = 0u;  // padding to 8 bytes
    }
}

__device__ __forceinline__ void decode_chunk(const unsigned char* __restrict__ gathered, size_t rank_stride,
                                             int32_t* __restrict__ frames, const CodecGeom& g, size_t gw, int lane) {
    const int rank = (int)(gw / (size_t)g.n_chunks);
    const int chunk = (int)(gw - (size_t)rank * g.n_chunks);
    const int t0 = chunk * CODEC_TPW;
    const unsigned char* wire = gathered + (size_t)rank * rank_stride;
    const int total_bands = (g.H + g.band_rows - 1) / g.band_rows;
    const int nb = rank < total_bands ? (total_bands - 1 - rank) / g.world + 1 : 0;
    const TileInfo ti = tile_info(g, rank, nb, t0 + (lane & (CODEC_TPW - 1)));
    const bool hv = lane < CODEC_TPW && ti.live;
    const uint2 hdr = hv ? ((const uint2*)wire_tile_hdr(wire))[t0 + lane] : make_uint2(0u, 0u);
    const uint32_t base = wire_chunk_base(wire, g)[chunk];
    const uint32_t* pay = (const uint32_t*)wire_payload(wire, g);
    uint32_t words[CODEC_TPW];
#pragma unroll
    for (int j = 0; j < CODEC_TPW; ++j) {  // lanes past a tile's words read something harmless
        const uint32_t mj = (uint32_t)__builtin_amdgcn_readlane((int)hdr.y, j);
        const uint32_t nw = 2 * units_of(mj);
        words[j] = nw ? pay[2 * ((size_t)base + (mj >> 12)) + min((uint32_t)lane, nw - 1)] : *(const uint32_t*)wire;
    }
    const int rx = lane & 7;
#pragma unroll
    for (int j = 0; j < CODEC_TPW; ++j) {
        const uint32_t first = (uint32_t)__builtin_amdgcn_readlane((int)hdr.x, j);
        const uint32_t mj = (uint32_t)__builtin_amdgcn_readlane((int)hdr.y, j);
        int64_t row_off;
        const bool inside = pixel_inside(g, rank, nb, ti, j, lane, &row_off);
        uint32_t px = first;  // flat tile: every pixel is the first one
        if (mj & 0xfffu) {    // wave-uniform
            uint32_t zz = 0;
            int wo = 0;  // word offset of the segment inside the tile's payload
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int w = (int)((mj >> (4 * c)) & 15u);
                if (w == 0) continue;
                const int pos = lane * w;
                const uint32_t word = (uint32_t)__builtin_amdgcn_ds_bpermute((wo + (pos >> 5)) << 2, (int)words[j]);
                zz |= ((word >> (pos & 31)) & ((1u << w) - 1u)) << (16 - 8 * c);
                wo += 2 * w;
            }
            const uint32_t d = unzigzag_bytes(zz) & 0xffffffu;
            // first column: odd rows add the row above's residual, every row adds `first`
            const uint32_t above = row_shr<8>(d);
            const uint32_t col = add_bytes(first, (lane & 8) ? add_bytes(d, above) : d);
            // rows: inclusive prefix inside each 8-lane row, seeded by the first column
            uint32_t v = rx == 0 ? col : d;
            uint32_t o = row_shr<1>(v);
            if (rx >= 1) v = add_bytes(v, o);
            o = row_shr<2>(v);
            if (rx >= 2) v = add_bytes(v, o);
            o = row_shr<4>(v);
            if (rx >= 4) v = add_bytes(v, o);
            px = v & 0xffffffu;
        }
        if (inside) frames[readlane64(ti.dst, j) + row_off + rx] = (int32_t)px;
    }
}

// Decode every rank's wire (rank r's at gathered + r * rank_stride) of a batch into the
// frames (frame f at frames + f * frame_stride).  One wave per chunk (CODEC_TPW tiles of one
// rank): one load of their headers, one load of each tile's payload words (lane q: word q),
// then per tile each lane fetches the word holding its bits (ds_bpermute), shifts and masks;
// prefix sums by DPP; one store.  Flat tiles store their first pixel.
__global__ __launch_bounds__(256) void decode_tiles_kernel(const unsigned char* __restrict__ gathered,
                                                          size_t rank_stride, int32_t* __restrict__ frames,
                                                          CodecGeom g) {
    const int lane = threadIdx.x & 63;
    const size_t n = (size_t)g.world * (size_t)g.n_chunks;
    for (size_t gw = (size_t)blockIdx.x * 4 + wave_index(); gw < n; gw += (size_t)gridDim.x * 4)
        decode_chunk(gathered, rank_stride, frames, g, gw, lane);
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
    hipLaunchKernelGGL(encode_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const uint32_t*)st, wire,
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
    const size_t waves = (size_t)g.world * (size_t)g.n_chunks;
    if (waves == 0) return (int)hipSuccess;
    hipLaunchKernelGGL(decode_tiles_kernel, dim3((unsigned)std::min<size_t>((waves + 3) / 4, CODEC_BLOCKS)), dim3(256), 0,
                       (hipStream_t)stream,
                       gathered, rank_stride, frames, g);
    return (int)hipGetLastError();
}

}  // namespace rtk
