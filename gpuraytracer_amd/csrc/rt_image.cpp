// rt_image.cpp — the reference's image epilogue (RTrace/image.swift:15-100):
// the rgba16Float render texture read back as Float16 (:35-38), then per RGB
// channel x2 exposure, Reinhard v/(v+1), pow(v, 1/2.2), clamp to [0,1] and a
// truncating UInt8(v*255) (:41-60); alpha 255 (:63).  Host-side form of the
// RT_OUT_RGBA8 epilogue the kernel fuses into its store: both call
// rt::tonemap_channel (rt_math.h), so the bytes are identical.
#include <math.h>
#include <string.h>

#include "../../include/rtpt.h"
#include "rt_math.h"

namespace {

// float -> IEEE binary16 bits, round-to-nearest-even (the texture store).
uint16_t to_half(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t ex = (x >> 23) & 0xFFu;
    uint32_t man = x & 0x7FFFFFu;
    if (ex == 0xFFu) return (uint16_t)(sign | 0x7C00u | (man ? 0x200u : 0u));
    const int e = (int)ex - 112;  // rebias 127 -> 15
    if (e >= 31) return (uint16_t)(sign | 0x7C00u);
    if (e <= 0) {  // half subnormal (or zero)
        if (e < -10) return (uint16_t)sign;
        man |= 0x800000u;
        const int shift = 14 - e;
        uint32_t h = man >> shift;
        const uint32_t rem = man & ((1u << shift) - 1u), halfway = 1u << (shift - 1);
        if (rem > halfway || (rem == halfway && (h & 1u))) ++h;
        return (uint16_t)(sign | h);
    }
    uint32_t h = ((uint32_t)e << 10) | (man >> 13);
    const uint32_t rem = man & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;  // carry may round up to inf
    return (uint16_t)(sign | h);
}

float from_half(uint16_t h) {
    const uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
    const uint32_t ex = ((uint32_t)h >> 10) & 0x1Fu;
    uint32_t man = (uint32_t)h & 0x3FFu;
    uint32_t x;
    if (ex == 0) {
        if (man == 0) {
            x = sign;
        } else {  // renormalise the subnormal
            int shift = 0;
            while (!(man & 0x400u)) { man <<= 1; ++shift; }
            x = sign | ((uint32_t)(113 - shift) << 23) | ((man & 0x3FFu) << 13);
        }
    } else if (ex == 0x1Fu) {
        x = sign | 0x7F800000u | (man << 13);
    } else {
        x = sign | ((ex + 112u) << 23) | (man << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}

}  // namespace

extern "C" void rt_tonemap_rgba8(const float* in, size_t n, uint8_t* out) {
    if (!in || !out) return;
    for (size_t i = 0; i < n; ++i) {
        for (int ch = 0; ch < 3; ++ch)
            out[4 * i + ch] = rt::tonemap_channel(from_half(to_half(in[4 * i + ch])));
        out[4 * i + 3] = 255;
    }
}
