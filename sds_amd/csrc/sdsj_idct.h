// sdsj_idct.h -- the ISLOW butterfly of jpeg_idct_islow (libjpeg-turbo jidctint.c, the IDCT Pillow's
// decoder runs for sds/transforms/functional.py:100), used by k_idct.
//
// Arithmetic: 32-bit integers exactly as jidctint.c's (CONST_BITS 13, PASS1_BITS 2, DESCALE with
// rounding, IDCT_range_limit = (x & 1023) as a signed 10-bit value + 128, clamped).
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

// One 1-D ISLOW butterfly (even/odd parts, jidctint.c); inputs x0..x7, outputs scaled sums
// before the final DESCALE: o[0..7].
__device__ __forceinline__ void islow_1d(int x0, int x1, int x2, int x3, int x4, int x5, int x6, int x7, int o[8]) {
  int z2 = x2, z3 = x6;
  int z1 = (z2 + z3) * (SDSJ_FIX_0_541196100);
  int t2 = z1 + (z3) * (-SDSJ_FIX_1_847759065);
  int t3 = z1 + (z2) * (SDSJ_FIX_0_765366865);
  int t0 = (x0 + x4) * (1 << 13);
  int t1 = (x0 - x4) * (1 << 13);
  int t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
  t0 = x7;
  t1 = x5;
  t2 = x3;
  t3 = x1;
  z1 = t0 + t3;
  z2 = t1 + t2;
  z3 = t0 + t2;
  int z4 = t1 + t3;
  int z5 = (z3 + z4) * (SDSJ_FIX_1_175875602);
  t0 = (t0) * (SDSJ_FIX_0_298631336);
  t1 = (t1) * (SDSJ_FIX_2_053119869);
  t2 = (t2) * (SDSJ_FIX_3_072711026);
  t3 = (t3) * (SDSJ_FIX_1_501321110);
  z1 = (z1) * (-SDSJ_FIX_0_899976223);
  z2 = (z2) * (-SDSJ_FIX_2_562915447);
  z3 = (z3) * (-SDSJ_FIX_1_961570560);
  z4 = (z4) * (-SDSJ_FIX_0_390180644);
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

__device__ __forceinline__ uint32_t range_limit(int x) {
  // IDCT_range_limit: (x & 1023) as a signed 10-bit value, + 128, clamped to [0, 255]
  int s = ((x & 1023) ^ 512) - 512;
  s += 128;
  return (uint32_t)(s < 0 ? 0 : s > 255 ? 255 : s);
}

}  // namespace sdsj
