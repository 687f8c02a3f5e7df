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

// -- packed form (k_idct): the same arithmetic on 16-bit pairs, the way the SIMD code itself runs it --
// The SIMD butterfly multiplies with vpmaddwd (two 16-bit products summed into 32 bits) on pairs of
// inputs regrouped so each pair meets one constant pair; v_dot2_i32_i16 is that instruction, with
// the 32-bit accumulate folded in.  vpaddw / vpsubw / vpmullw are v_pk_add_u16 / v_pk_sub_u16 /
// v_pk_mul_lo_u16; vpackssdw is v_cvt_pk_i16_i32.  All sums are taken modulo 2^32, so the regrouped
// constants below give islow_1d's residues exactly (checked over random and extreme inputs).
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
// lo * c0 + hi * c1 + acc (mod 2^32).  The builtin becomes the two-address v_dot2c_i32_i16 (literal
// constant, accumulator overwritten: a v_mov for every accumulator read twice); the three-address VOP3P
// form takes the constant pair from an SGPR and needs no copies.
#ifndef SDSJ_DOT2_ASM
#define SDSJ_DOT2_ASM 1
#endif
__device__ __forceinline__ uint32_t dot2(u16x2 a, short c0, short c1, uint32_t acc) {
#if SDSJ_DOT2_ASM
  uint32_t d;
  const int k = (int)(((uint32_t)(uint16_t)c1 << 16) | (uint16_t)c0);
  asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(d) : "v"(as_u32(a)), "s"(k), "v"(acc));
  return d;
#else
  return (uint32_t)__builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, a), (s16x2){c0, c1}, (int)acc, false);
#endif
}

// islow_1d on pairs p26 = (x2, x6), p71 = (x7, x1), p53 = (x5, x3), p04 = (x0, x4) (low, high half),
// with the DESCALE rounding `rnd` added to every output.
__device__ __forceinline__ void islow_1d_pk(u16x2 p26, u16x2 p71, u16x2 p53, u16x2 p04, uint32_t rnd, uint32_t o[8]) {
  const u16x2 sw = __builtin_shufflevector(p04, p04, 1, 0);
  const u16x2 s = p04 + sw, d = p04 - sw;  // low halves: x0 + x4, x0 - x4 (16-bit)
  const uint32_t t0e = ((uint32_t)(int)(int16_t)s.x << 13) + rnd;
  const uint32_t t1e = ((uint32_t)(int)(int16_t)d.x << 13) + rnd;
  // even part: tmp3 = x2 (F0.541 + F0.765) + x6 F0.541, tmp2 = x2 F0.541 + x6 (F0.541 - F1.848)
  const uint32_t t10 = dot2(p26, 10703, 4433, t0e), t13 = dot2(p26, -10703, -4433, t0e);
  const uint32_t t11 = dot2(p26, 4433, -10704, t1e), t12 = dot2(p26, -4433, 10704, t1e);
  // odd part: (z3, z4) = (x7 + x3, x1 + x5) in 16 bits; z5 folded into both rotations
  const u16x2 pz = p71 + __builtin_shufflevector(p53, p53, 1, 0);
  const uint32_t z3 = dot2(pz, -6436, 9633, 0u), z4 = dot2(pz, 9633, 6437, 0u);
  const uint32_t t0 = dot2(p71, -4927, -7373, z3), t3 = dot2(p71, -7373, 4926, z4);
  const uint32_t t1 = dot2(p53, -4176, -20995, z4), t2 = dot2(p53, -20995, 4177, z3);
  o[0] = t10 + t3;
  o[7] = t10 - t3;
  o[1] = t11 + t2;
  o[6] = t11 - t2;
  o[2] = t12 + t1;
  o[5] = t12 - t1;
  o[3] = t13 + t0;
  o[4] = t13 - t0;
}

// zigzag index of natural (row-major) position p: the inverse of natural_order
__device__ __forceinline__ int zigzag_of(int p) {
  constexpr int8_t t[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42, 3,  8,  12, 17, 25, 30,
                            41, 43, 9,  11, 18, 24, 31, 40, 44, 53, 10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38,
                            46, 51, 55, 60, 21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};
  return t[p];
}

}  // namespace sdsj
