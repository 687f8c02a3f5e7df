// sdsj_idct.h -- the ISLOW butterfly of jpeg_idct_islow (libjpeg-turbo jidctint.c, the IDCT Pillow's
// decoder runs for sds/transforms/functional.py:100), used by k_idct.
//
// Arithmetic: jidctint.c's butterfly (CONST_BITS 13, PASS1_BITS 2, DESCALE with rounding) in the 16-bit
// lanes of libjpeg-turbo's x86-64 SIMD version, which is what Pillow runs: see islow_1d and k_idct.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sdsj_common.h"

namespace sdsj {

#define SDSJ_FIX_0_298631336 2446
#define SDSJ_FIX_0_390180644 3196
#define SDSJ_FIX_0_541196100 4433
#define SDSJ_FIX_0_765366865 6270
#define SDSJ_FIX_0_899976223 7373
#define SDSJ_FIX_1_175875602 9633
#define SDSJ_FIX_1_501321110 12299
#define SDSJ_FIX_1_847759065 15137
#define SDSJ_FIX_1_961570560 16069
#define SDSJ_FIX_2_053119869 16819
#define SDSJ_FIX_2_562915447 20995
#define SDSJ_FIX_3_072711026 25172

__device__ __forceinline__ int wrap16(int v) { return (int)(int16_t)v; }  // (one v_bfe_i32)
__device__ __forceinline__ int sat16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }

// One 1-D ISLOW butterfly with the 16-bit lane semantics of libjpeg-turbo's x86-64 SIMD IDCT
// (simd/x86_64/jidctint-avx2.asm dodct; the IDCT Pillow's wheel runs, jsimd_can_idct_islow): in0 + in4,
// in0 - in4, z3 = in7 + in3 and z4 = in5 + in1 are vpaddw (wrapped to 16 bits); the products are
// vpmaddwd of 16-bit inputs (exact) and every other sum is vpaddd, wrapping at 32 bits -- uint32 here,
// where the jidctint.c operation order below gives the same residues as the asm's regrouped constants.
// Inputs are 16-bit values; outputs the scaled sums before the final DESCALE.  On valid streams nothing
// wraps and this is jidctint.c jpeg_idct_islow exactly.
__device__ __forceinline__ void islow_1d(int x0, int x1, int x2, int x3, int x4, int x5, int x6, int x7, uint32_t o[8]) {
  const uint32_t e2 = (uint32_t)x2, e6 = (uint32_t)x6;
  const uint32_t z1e = (e2 + e6) * (uint32_t)SDSJ_FIX_0_541196100;
  const uint32_t t2e = z1e + e6 * (uint32_t)(-SDSJ_FIX_1_847759065);
  const uint32_t t3e = z1e + e2 * (uint32_t)SDSJ_FIX_0_765366865;
  const uint32_t t0e = (uint32_t)wrap16(x0 + x4) << 13;
  const uint32_t t1e = (uint32_t)wrap16(x0 - x4) << 13;
  const uint32_t t10 = t0e + t3e, t13 = t0e - t3e, t11 = t1e + t2e, t12 = t1e - t2e;
  uint32_t t0 = (uint32_t)x7, t1 = (uint32_t)x5, t2 = (uint32_t)x3, t3 = (uint32_t)x1;
  uint32_t z1 = t0 + t3, z2 = t1 + t2;
  uint32_t z3 = (uint32_t)wrap16(x7 + x3), z4 = (uint32_t)wrap16(x5 + x1);
  const uint32_t z5 = (z3 + z4) * (uint32_t)SDSJ_FIX_1_175875602;
  t0 *= (uint32_t)SDSJ_FIX_0_298631336;
  t1 *= (uint32_t)SDSJ_FIX_2_053119869;
  t2 *= (uint32_t)SDSJ_FIX_3_072711026;
  t3 *= (uint32_t)SDSJ_FIX_1_501321110;
  z1 *= (uint32_t)(-SDSJ_FIX_0_899976223);
  z2 *= (uint32_t)(-SDSJ_FIX_2_562915447);
  z3 *= (uint32_t)(-SDSJ_FIX_1_961570560);
  z4 *= (uint32_t)(-SDSJ_FIX_0_390180644);
  z3 += z5;
  z4 += z5;
  t0 += z1 + z3;
  t1 += z2 + z4;
  t2 += z2 + z3;
  t3 += z1 + z4;
  o[0] = t10 + t3;
  o[7] = t10 - t3;
  o[1] = t11 + t2;
  o[6] = t11 - t2;
  o[2] = t12 + t1;
  o[5] = t12 - t1;
  o[3] = t13 + t0;
  o[4] = t13 - t0;
}

// Pass 1 output: (sum + 2^10) >> 11 (vpaddd, vpsrad), saturated to 16 bits (vpackssdw).
__device__ __forceinline__ int descale_p1(uint32_t v) { return sat16((int)(v + (1u << 10)) >> 11); }
// Pass 2 output sample: (sum + 2^17) >> 18, saturated to 16 then 8 bits (vpackssdw, vpacksswb), + 128
// (vpaddb CENTERJSAMPLE) -- where jidctint.c indexes range_limit[x & 1023].
__device__ __forceinline__ uint32_t descale_p2(uint32_t v) {
  const int x = (int)(v + (1u << 17)) >> 18;
  return (uint32_t)((x < -128 ? -128 : (x > 127 ? 127 : x)) + 128);
}

}  // namespace sdsj
