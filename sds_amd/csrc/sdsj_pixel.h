// sdsj_pixel.h -- per-pixel helpers shared by the fused resample kernels (device only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sdsj_common.h"

namespace sdsj {

constexpr int kMaxStrip = 64;  // output rows per fused-resample workgroup (strip) at most
constexpr int kVTaps = 16;     // vertical taps staged in LDS (= the largest ring); k_rs420: kVTapsF (sdsj_common.h)

__device__ __forceinline__ int rs_clip8(int32_t v) {
  v >>= 22;
  return v < 0 ? 0 : v > 255 ? 255 : v;
}

__device__ __forceinline__ int clamp255i(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }

// jdcolor.c ycc_rgb_convert (its tables evaluated arithmetically); cb, cr already minus 128
// (24-bit multiplies: |constant| < 2^17, |cb|, |cr| <= 128 -- exact, full rate)
// ycc_px on cb, cr without the 128 subtracted (the offsets folded into the constants: the same
// integers, so the same results)
__device__ __forceinline__ void ycc_raw(int y, int cb, int cr, int& r, int& g, int& b) {
  r = clamp255i(y + ((__mul24(91881, cr) - 11728000) >> 16));
  g = clamp255i(y + ((__mul24(-46802, cr) + __mul24(-22554, cb) + 8910336) >> 16));
  b = clamp255i(y + ((__mul24(116130, cb) - 14831872) >> 16));
}

__device__ __forceinline__ void ycc_px(int y, int cb, int cr, int& r, int& g, int& b) {
  r = clamp255i(y + ((__mul24(91881, cr) + 32768) >> 16));
  g = clamp255i(y + ((__mul24(-46802, cr) + (__mul24(-22554, cb) + 32768)) >> 16));
  b = clamp255i(y + ((__mul24(116130, cb) + 32768) >> 16));
}

// pixel (0..255) x Pillow coefficient (|k| < 2^23: normalised weights of magnitude < 2 in
// 22-bit fixed point) -- exact in a 24-bit multiply (v_mad_i32_i24, full rate)
__device__ __forceinline__ int32_t tap(int32_t px, int32_t k) { return __mul24(px, k); }

// Packs three uint8 results as R | G << 8 | B << 16.  The values go through an empty asm first:
// otherwise hipcc (ROCm 7.2, gfx950) fuses "clip8(a) | clip8(b) << 8" into v_ashr_pk_u8_i32 and
// then ORs the third byte in as if that instruction zeroed bits 16-31 -- on the hardware they keep
// the register's old contents (measured: channel 2 of k_rs420 corrupted; tools/case_diff.py).
__device__ __forceinline__ uint32_t pack3(int a, int b, int c) {
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c));
  return (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)c << 16);
}

enum { kLayGeneric = 0, kLay420 = 1, kLayFull = 2 };

// Output addressing: element (channel c, pixel p) at base + p * ps + c * cs (elements).
struct OutMap {
  int64_t base, ps, cs;
  bool f32;
};

// put3 for output row `row` (uniform: the row's first pixel index) and column x: the row's channel
// bases are uniform, so each store is a scalar base plus the lane's 32-bit offset.
__device__ __forceinline__ void put3_row(void* out, const OutMap& m, const float* lut, int64_t row, int x, int v0, int v1,
                                         int v2) {
  const int64_t e = m.base + row * m.ps;
  const uint32_t o = (uint32_t)(x * m.ps);
  if (m.f32) {
    float* b = reinterpret_cast<float*>(out) + e;
    b[o] = lut[v0];
    (b + m.cs)[o] = lut[v1];
    (b + 2 * m.cs)[o] = lut[v2];
  } else {
    uint8_t* b = reinterpret_cast<uint8_t*>(out) + e;
    b[o] = (uint8_t)v0;
    (b + m.cs)[o] = (uint8_t)v1;
    (b + 2 * m.cs)[o] = (uint8_t)v2;
  }
}

__device__ __forceinline__ void put3(void* out, const OutMap& m, const float* lut, int64_t pix, int v0, int v1, int v2) {
  const int64_t e = m.base + pix * m.ps;
  if (m.f32) {
    float* o = reinterpret_cast<float*>(out) + e;
    o[0] = lut[v0];
    o[m.cs] = lut[v1];
    o[2 * m.cs] = lut[v2];
  } else {
    uint8_t* o = reinterpret_cast<uint8_t*>(out) + e;
    o[0] = (uint8_t)v0;
    o[m.cs] = (uint8_t)v1;
    o[2 * m.cs] = (uint8_t)v2;
  }
}

}  // namespace sdsj
