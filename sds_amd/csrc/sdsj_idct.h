// sdsj_idct.h -- dequantisation + jpeg_idct_islow (libjpeg-turbo jidctint.c, the IDCT Pillow's
// decoder runs for sds/transforms/functional.py:100) and the block geometry shared by the kernels
// that produce sample planes: the entropy write pass (it inverse-transforms every block as it
// completes, sdsj_entropy.hip), k_idct (progressive images) and k_cutfill (blocks libjpeg leaves zero).
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

// Multiply for the ISLOW butterflies: F24 = 24-bit signed operands (v_mul_i32_i24, full rate),
// exact -- the same low 32 bits as the 32-bit multiply -- whenever both operands lie in (-2^23, 2^23).
template <bool F24>
__device__ __forceinline__ int imul(int a, int b) { return F24 ? __mul24(a, b) : a * b; }

// One 1-D ISLOW butterfly (even/odd parts, jidctint.c); inputs x0..x7, outputs scaled sums
// before the final DESCALE: o[0..7].  Every multiplicand is a sum of at most 4 inputs.
template <bool F24 = false>
__device__ __forceinline__ void islow_1d(int x0, int x1, int x2, int x3, int x4, int x5, int x6, int x7, int o[8]) {
  int z2 = x2, z3 = x6;
  int z1 = imul<F24>(z2 + z3, SDSJ_FIX_0_541196100);
  int t2 = z1 + imul<F24>(z3, -SDSJ_FIX_1_847759065);
  int t3 = z1 + imul<F24>(z2, SDSJ_FIX_0_765366865);
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
  int z5 = imul<F24>(z3 + z4, SDSJ_FIX_1_175875602);
  t0 = imul<F24>(t0, SDSJ_FIX_0_298631336);
  t1 = imul<F24>(t1, SDSJ_FIX_2_053119869);
  t2 = imul<F24>(t2, SDSJ_FIX_3_072711026);
  t3 = imul<F24>(t3, SDSJ_FIX_1_501321110);
  z1 = imul<F24>(z1, -SDSJ_FIX_0_899976223);
  z2 = imul<F24>(z2, -SDSJ_FIX_2_562915447);
  z3 = imul<F24>(z3, -SDSJ_FIX_1_961570560);
  z4 = imul<F24>(z4, -SDSJ_FIX_0_390180644);
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

// Pass 1 on one column: dequantised coefficients of rows 0..7 -> workspace column, DESCALE(,
// CONST_BITS - PASS1_BITS).  (jidctint.c's all-AC-zero shortcut gives the same values.)
// F24 is exact when every dequantised coefficient of the block lies in (-2^12, 2^12): pass-1
// multiplicands then stay below 2^14, sums before the DESCALE below 2^30, so pass-2 inputs below 2^19
// and their multiplicands below 2^21 (real 8-bit images stay near 2^11: kF24Bound).
template <bool F24 = false>
__device__ __forceinline__ void islow_pass1(const int x[8], int w[8]) {
  int o[8];
  islow_1d<F24>(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], o);
#pragma unroll
  for (int k = 0; k < 8; k++) w[k] = (o[k] + (1 << 10)) >> 11;
}

// Pass 2 on one workspace row -> 8 samples, little-endian in two dwords (DESCALE(, CONST_BITS +
// PASS1_BITS + 3), range limit).
template <bool F24 = false>
__device__ __forceinline__ uint2 islow_pass2(const int w[8]) {
  int o[8];
  islow_1d<F24>(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], o);
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) lo |= range_limit((o[k] + (1 << 17)) >> 18) << (8 * k);
#pragma unroll
  for (int k = 0; k < 4; k++) hi |= range_limit((o[k + 4] + (1 << 17)) >> 18) << (8 * k);
  return make_uint2(lo, hi);
}

constexpr int kF24Bound = 1 << 12;

// a / b for 0 <= a < 2^24, 1 <= b < 2^16: float estimate, then one correction each way (exact)
__device__ __forceinline__ int qdiv(int a, int b, float rb) {
  int q = (int)((float)a * rb);
  q -= q * b > a ? 1 : 0;
  q += (q + 1) * b <= a ? 1 : 0;
  return q;
}

// Block geometry of one image: decode-order block index g -> component, block column / row, the
// block's byte offset in the image's (block-linear) plane area, and whether the crop reads it.
struct BlkGeo {
  int32_t bpm, mcux;
  float rbpm, rmcux;
  int32_t binfo[kMaxBlocksPerMcu];  // component | dx << 2 | dy << 4 of MCU block b (jdcoefct order)
  int32_t hv[kMaxComp];             // blocks per MCU across | down << 4 (1, 1 for a one-component scan)
  int32_t bw[kMaxComp];
  int32_t plane[kMaxComp];                                            // plane offset in the plane area
  int32_t bx0[kMaxComp], bx1[kMaxComp], by0[kMaxComp], by1[kMaxComp];  // blocks the crop reads (inclusive)
};

// Only the blocks whose samples the colour / resample passes read: the source rectangle [src_x0,
// src_x0 + src_w) x [src_y0, src_y1) in each component's sampling, widened by one sample for the
// fancy upsampling's neighbours (the crop drops the rest of the image).
__device__ inline void blkgeo_init(const ImgDesc* d, BlkGeo& X) {
  const int ncomp = d->ncomp;
  X.bpm = d->bpm;
  X.mcux = d->mcux;
  X.rbpm = 1.0f / (float)d->bpm;
  X.rmcux = 1.0f / (float)d->mcux;
  for (int b = 0; b < d->bpm; b++) X.binfo[b] = d->blk_comp[b] | (d->blk_dx[b] << 2) | (d->blk_dy[b] << 4);
  const int x0 = d->src_x0, x1 = d->src_x0 + d->src_w, y0 = d->src_y0, y1 = d->src_y1;
  const bool any = d->geo != kGeoZeros && x1 > x0 && y1 > y0;
  for (int c = 0; c < ncomp; c++) {
    const CompDesc& cd = d->comp[c];
    const int rh = ncomp == 1 ? 1 : d->hmax / cd.h, rv = ncomp == 1 ? 1 : d->vmax / cd.v;
    int cx0 = x0 / rh - 1, cx1 = (x1 - 1) / rh + 1, cy0 = y0 / rv - 1, cy1 = (y1 - 1) / rv + 1;
    cx0 = cx0 < 0 ? 0 : cx0;
    cy0 = cy0 < 0 ? 0 : cy0;
    cx1 = cx1 > cd.bw * 8 - 1 ? cd.bw * 8 - 1 : cx1;
    cy1 = cy1 > cd.bh * 8 - 1 ? cd.bh * 8 - 1 : cy1;
    X.hv[c] = ncomp == 1 ? 0x11 : (cd.h | (cd.v << 4));
    X.bw[c] = cd.bw;
    X.plane[c] = (int32_t)cd.plane_off;
    X.bx0[c] = any ? cx0 >> 3 : 1;
    X.bx1[c] = any ? cx1 >> 3 : 0;
    X.by0[c] = any ? cy0 >> 3 : 1;
    X.by1[c] = any ? cy1 >> 3 : 0;
  }
}

// Block g: its byte offset in the plane area (off) and component (c); true when the crop reads it.
__device__ __forceinline__ bool blk_locate(const BlkGeo& X, int g, int& c, int& off) {
  const int mcu = qdiv(g, X.bpm, X.rbpm);
  const int info = X.binfo[g - mcu * X.bpm];
  c = info & 3;
  const int my = qdiv(mcu, X.mcux, X.rmcux), mx = mcu - my * X.mcux;
  const int hv = X.hv[c];
  const int bx = mx * (hv & 15) + ((info >> 2) & 3), by = my * (hv >> 4) + (info >> 4);
  off = X.plane[c] + ((by * X.bw[c] + bx) << 6);
  return bx >= X.bx0[c] && bx <= X.bx1[c] && by >= X.by0[c] && by <= X.by1[c];
}

}  // namespace sdsj
