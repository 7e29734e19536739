// rt_codec_common.h -- device helpers of the band-set tile codec shared by its kernels
// (rt_codec.hip) and the trace kernels' fused encoder (rt_kernel.hip, RT_BANDS_TILES): byte-wise
// residual arithmetic, zigzag, the DPP steps inside 8-lane groups, the width code.  The format
// is specified in raytracer_hip/tilecodec.py.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rtk {

constexpr int CODEC_TPW = 8;     // tiles per wave of the codec kernels = tiles per chunk
constexpr int STAGE_WORDS = 48;  // staging words per tile (3 channels x 8 bits x 64 lanes / 32)
constexpr int STAGE_UNITS = STAGE_WORDS / 2;

__device__ __forceinline__ const uint32_t* wire_tile_hdr(const unsigned char* w) { return (const uint32_t*)(w + 16); }
__device__ __forceinline__ uint32_t* wire_tile_hdr(unsigned char* w) { return (uint32_t*)(w + 16); }

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
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf, bool BOUND = true>
__device__ __forceinline__ uint32_t dpp(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROW_MASK, BANK_MASK, BOUND);
}
// lane 8j's value in every lane of its 8-lane group
__device__ __forceinline__ uint32_t group8_first(uint32_t v) {
    const uint32_t q = dpp<0x00>(0u, v);            // quad_perm [0,0,0,0]
    return dpp<0x114, 0xf, 0xa, false>(q, q);        // row_shr:4 into lanes 4-7, 12-15 of each row
}
// OR of the 8 lanes of each group, in every lane
__device__ __forceinline__ uint32_t group8_or(uint32_t v) {
    v |= dpp<0xb1>(0u, v);   // quad_perm [1,0,3,2]
    v |= dpp<0x4e>(0u, v);   // quad_perm [2,3,0,1]
    v |= dpp<0x141>(0u, v);  // row_half_mirror
    return v;
}
// inclusive scan over the wave (all 64 lanes active)
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
    x += row_shr<1>(x);
    x += row_shr<2>(x);
    x += row_shr<4>(x);
    x += row_shr<8>(x);
    x += dpp<0x142, 0xa, 0xf, false>(0u, x);  // row_bcast:15 -> rows 1, 3
    x += dpp<0x143, 0xc, 0xf, false>(0u, x);  // row_bcast:31 -> rows 2, 3
    return x;
}

__device__ __forceinline__ uint32_t units_of(uint32_t wm) { return (wm & 15u) + ((wm >> 4) & 15u) + ((wm >> 8) & 15u); }
// Widths WIDTHS = {0, 2, 3, 4, 6, 8} by index (nibbles of 0x864320); a tile's width code is
// i_R + 6 i_G + 36 i_B (< 216, the header's top byte).
__device__ __forceinline__ uint32_t width_at(uint32_t i) { return (0x864320u >> (4u * i)) & 15u; }
// widths of a code as wm = w_R | w_G << 4 | w_B << 8
__device__ __forceinline__ uint32_t widths_of_code(uint32_t code) {
    return width_at(code % 6u) | (width_at(code / 6u % 6u) << 4) | (width_at(code / 36u) << 8);
}
// Width index of a channel: bit length of its OR of zigzag residuals rounded up to a width.
__device__ __forceinline__ uint32_t width_index(uint32_t o) {
    return o == 0 ? 0u : o < 4 ? 1u : o < 8 ? 2u : o < 16 ? 3u : o < 64 ? 4u : 5u;
}

// A row's w bytes of one channel segment (8 residuals of w bits, little-endian) at dst: the
// store shapes the alignments of ry * w allow.
__device__ __forceinline__ void store_row_bits(unsigned char* dst, uint32_t w, uint64_t acc) {
    if (w == 8) {
        *(uint64_t*)dst = acc;
    } else if (w == 4) {
        *(uint32_t*)dst = (uint32_t)acc;
    } else if (w == 2) {
        *(uint16_t*)dst = (uint16_t)acc;
    } else if (w == 6) {  // 6 ry: 2-byte aligned
        ((uint16_t*)dst)[0] = (uint16_t)acc;
        ((uint16_t*)dst)[1] = (uint16_t)(acc >> 16);
        ((uint16_t*)dst)[2] = (uint16_t)(acc >> 32);
    } else if (w == 3) {
        dst[0] = (unsigned char)acc;
        dst[1] = (unsigned char)(acc >> 8);
        dst[2] = (unsigned char)(acc >> 16);
    }
}

}  // namespace rtk
