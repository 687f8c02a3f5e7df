// sdsj_resample.hip -- fused colour conversion + two-pass resample + output layout (gfx950).
//
// One 256-thread workgroup per (image, strip of output rows, tile of output columns); thread t owns
// output column tile_x0 + t.  It streams the crop rows the strip's vertical windows cover, kStepRows
// source rows per step:
//   A. stage the plane rows of the step (jdmainct.c context rows: chroma rows i and neighbour f for
//      v-upsampled components) for the tile's source columns into LDS (global_load_lds DMA);
//   B. fancy-upsample + colour-convert them (jdsample.c h2v2/h2v1/h1v2, jdcolor.c ycc_rgb_convert)
//      into planar R, G, B rows in LDS;
//   H. horizontal pass (Pillow ImagingResampleHorizontal_8bpc: acc from 1 << 21, >> 22, clip to
//      uint8) for the thread's column of each step row -> a per-column ring of the last R rows;
//   V. every output row whose vertical window ends in this step is summed from the ring
//      (ImagingResampleVertical_8bpc) and written with hflip, CHW/HWC layout and the uint8 /
//      normalise LUT (functional.py:100-110, presets.py:154-162).
// Integer sums are exact in any order, so this equals Pillow's row-by-row two-pass result bit for
// bit.  Nothing full-resolution is written back to HBM: per image the planes are read once and the
// output written once.  Images whose tiles or windows do not fit (plan_image: fused = 0, extreme
// downscales) keep the unfused k_color -> k_hpass -> k_vpass path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sdsj_common.h"
#include "sdsj_kernels.h"
#include "sdsj_pixel.h"

namespace sdsj {


constexpr int kRsThreads = 256;
constexpr int kStepRows = 4;                 // source rows per step (fewer when the staging pool is short)
constexpr int kStageDW = 2944;               // staging pool (dwords): plane rows of one step
constexpr int kRgbW = kMaxSpan + 32;         // LDS RGB row pitch (+ over-read of unused taps)


struct LdsResample {
  uint32_t st[kStageDW];                     // plane rows of the step, row-contiguous (global_load_lds)
  uint8_t rgb[kStepRows][3][kRgbW];          // converted source rows, planar R, G, B
  uint32_t ring[kRingDW];                    // per column: horizontal results of the last R rows (R|G<<8|B<<16)
  int32_t vb[kMaxStrip][2];                  // strip rows: vertical window (first row, row count)
  int32_t vw[kMaxStrip][kVTaps];             // strip rows: vertical weights (Pillow kk, 22-bit fixed point)
};

// Component columns [jal, jal + 4 * nd) that source columns [ax0, ax1) need (fancy upsampling
// reads one neighbour each side), dword-aligned.  jal + 4 * nd <= pitch (pitch is a multiple of 8).
__device__ __forceinline__ void comp_cols(const CompDesc& c, int ax0, int ax1, int* jal, int* nd) {
  int lo = ax0, hi = ax1 - 1;
  if (c.rh == 2) {
    lo = (ax0 >> 1) - 1;
    hi = ((ax1 - 1) >> 1) + 1;
    lo = lo < 0 ? 0 : lo;
    hi = hi > c.dw - 1 ? c.dw - 1 : hi;
  }
  *jal = lo & ~3;
  *nd = (hi + 1 - *jal + 3) >> 2;
}

// Component rows [ilo, ihi] that source rows [ya, yb) need (jdmainct.c context rows, clamped).
__device__ __forceinline__ void comp_rows(const CompDesc& c, int ya, int yb, int* ilo, int* ihi) {
  if (c.rv == 2) {
    const int lo = (ya >> 1) - 1, hi = ((yb - 1) >> 1) + 1;
    *ilo = lo < 0 ? 0 : lo;
    *ihi = hi > c.dh - 1 ? c.dh - 1 : hi;
  } else {
    *ilo = ya;
    *ihi = yb - 1;
  }
}

// up_sample() of sdsj_kernels.hip over staged rows; r0 = row i, r1 = neighbour row f, both indexed
// by absolute component column.
__device__ __forceinline__ int up_lds(const uint8_t* r0, const uint8_t* r1, int rh, int rv, int dw, int x, int y) {
  if (rh == 1 && rv == 1) return r0[x];
  if (rv == 2) {
    if (rh == 2) {
      const int jx = x >> 1;
      if (dw <= 2) return r0[jx];  // h2v2_upsample (box)
      const int cs = r0[jx] * 3 + r1[jx];
      if ((x & 1) == 0) {
        const int cn = jx > 0 ? r0[jx - 1] * 3 + r1[jx - 1] : cs;
        return (cs * 3 + cn + 8) >> 4;
      }
      const int cn = jx < dw - 1 ? r0[jx + 1] * 3 + r1[jx + 1] : cs;
      return (cs * 3 + cn + 7) >> 4;
    }
    return (r0[x] * 3 + r1[x] + ((y & 1) ? 2 : 1)) >> 2;  // h1v2_fancy_upsample
  }
  const int jx = x >> 1;  // h2v1_fancy_upsample
  const int a = r0[jx];
  if (dw <= 2) return a;
  if ((x & 1) == 0) return jx == 0 ? a : (a * 3 + r0[jx - 1] + 1) >> 2;
  return jx == dw - 1 ? a : (a * 3 + r0[jx + 1] + 2) >> 2;
}

struct RsArgs {
  const ImgDesc* d;
  CompDesc cg[kMaxComp];  // component geometry in registers (descriptor loads cannot be hoisted past stores)
  ImgDesc* dmut;  // diagnostics (SDSJ_RS_TIMING)
  const uint8_t* planes;
  const int32_t *bh, *kh, *bv, *kv;
  int ow, oh, oy0, oy1, need_h, need_v, ksh, ksv, ncomp, cx0, cy0, tw, ntiles, rmask, rstride, layout;
  bool fl;
  OutMap om;
  const float* lut;
  void* out;
};

// B. upsample + colour convert step row q (image row y) over columns [ax0, ax1).
__device__ __forceinline__ void convert_row(LdsResample& L, const RsArgs& A, int q, int y, int ax0, int ax1,
                                            const int* soff, const int* ilo, const int* nd, const int* jal) {
  const ImgDesc* d = A.d;
  const uint8_t* stb = reinterpret_cast<const uint8_t*>(L.st);
  int rowi[kMaxComp], rowf[kMaxComp];
#pragma unroll
  for (int c = 0; c < kMaxComp; c++) {
    int i = y, f = y;
    if (A.cg[c].rv == 2) {
      i = y >> 1;
      f = (y & 1) ? i + 1 : i - 1;
      f = f < 0 ? 0 : (f > A.cg[c].dh - 1 ? A.cg[c].dh - 1 : f);
    }
    rowi[c] = soff[c] + (i - ilo[c]) * nd[c];
    rowf[c] = soff[c] + (f - ilo[c]) * nd[c];
  }
  const uint8_t* a0 = stb + 4 * rowi[0] - jal[0];
  const uint8_t* b0 = stb + 4 * rowf[0] - jal[0];
  const uint8_t* a1 = stb + 4 * rowi[1] - jal[1];
  const uint8_t* b1 = stb + 4 * rowf[1] - jal[1];
  const uint8_t* a2 = stb + 4 * rowi[2] - jal[2];
  const uint8_t* b2 = stb + 4 * rowf[2] - jal[2];
  uint8_t* oR = L.rgb[q][0] - ax0;
  uint8_t* oG = L.rgb[q][1] - ax0;
  uint8_t* oB = L.rgb[q][2] - ax0;
  const int t = threadIdx.x;
  if (A.layout == kLay420) {
    // h2v2_fancy_upsample on pixel pairs (2j, 2j + 1): both use column sum j, the even one blends
    // column j - 1 in, the odd one column j + 1 (edges repeat column j)
    const int dw = A.cg[1].dw;
    const int j0 = ax0 >> 1, np = ((ax1 - 1) >> 1) - j0 + 1;
    for (int p = t; p < np; p += kRsThreads) {
      const int j = j0 + p, jm = j > 0 ? j - 1 : j, jp = j < dw - 1 ? j + 1 : j;
      const int u0 = a1[j] * 3 + b1[j], um = a1[jm] * 3 + b1[jm], up = a1[jp] * 3 + b1[jp];
      const int v0 = a2[j] * 3 + b2[j], vm = a2[jm] * 3 + b2[jm], vp = a2[jp] * 3 + b2[jp];
      const int x = 2 * j;
      int r, g, bb;
      if (x >= ax0) {
        ycc_px(a0[x], ((u0 * 3 + um + 8) >> 4) - 128, ((v0 * 3 + vm + 8) >> 4) - 128, r, g, bb);
        oR[x] = (uint8_t)r;
        oG[x] = (uint8_t)g;
        oB[x] = (uint8_t)bb;
      }
      if (x + 1 < ax1) {
        ycc_px(a0[x + 1], ((u0 * 3 + up + 7) >> 4) - 128, ((v0 * 3 + vp + 7) >> 4) - 128, r, g, bb);
        oR[x + 1] = (uint8_t)r;
        oG[x + 1] = (uint8_t)g;
        oB[x + 1] = (uint8_t)bb;
      }
    }
  } else if (A.layout == kLayFull) {  // every component at full resolution (4:4:4, gray)
    for (int x = ax0 + t; x < ax1; x += kRsThreads) {
      int r = a0[x], g = r, bb = r;
      if (A.ncomp == 3) ycc_px(a0[x], a1[x] - 128, a2[x] - 128, r, g, bb);
      oR[x] = (uint8_t)r;
      oG[x] = (uint8_t)g;
      oB[x] = (uint8_t)bb;
    }
  } else {
    const CompDesc &c0 = A.cg[0], &c1 = A.cg[1], &c2 = A.cg[2];
    for (int x = ax0 + t; x < ax1; x += kRsThreads) {
      const int Y = up_lds(a0, b0, c0.rh, c0.rv, c0.dw, x, y);
      int r = Y, g = Y, bb = Y;
      if (A.ncomp == 3)
        ycc_px(Y, up_lds(a1, b1, c1.rh, c1.rv, c1.dw, x, y) - 128, up_lds(a2, b2, c2.rh, c2.rv, c2.dw, x, y) - 128, r,
               g, bb);
      oR[x] = (uint8_t)r;
      oG[x] = (uint8_t)g;
      oB[x] = (uint8_t)bb;
    }
  }
}

// One tile of one strip.  KT > 0: exactly KT horizontal taps with the column's coefficients in
// registers (zero past its window; KT = 1 with weight 1 << 22 when there is no horizontal pass);
// KT = 0: any tap count, coefficients read from the table.
template <int KT>
__device__ __forceinline__ void resample_tile(LdsResample& L, const RsArgs& A, int tile) {
  const ImgDesc* d = A.d;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int ox0 = tile * A.tw, ox1 = ox0 + A.tw < A.ow ? ox0 + A.tw : A.ow;
  const int s_lo = A.need_h ? A.bh[2 * ox0] : ox0;
  const int s_hi = A.need_h ? A.bh[2 * (ox1 - 1)] + A.bh[2 * (ox1 - 1) + 1] : ox1;
  const int ax0 = A.cx0 + s_lo, ax1 = A.cx0 + s_hi;  // image columns of the tile (<= kMaxSpan)
  const int r_lo = A.need_v ? A.bv[2 * A.oy0] : A.oy0;
  const int r_hi = A.need_v ? A.bv[2 * (A.oy1 - 1)] + A.bv[2 * (A.oy1 - 1) + 1] : A.oy1;
  int jal[kMaxComp] = {0, 0, 0}, nd[kMaxComp] = {0, 0, 0};
#pragma unroll
  for (int c = 0; c < kMaxComp; c++)
    if (c < A.ncomp) comp_cols(A.cg[c], ax0, ax1, &jal[c], &nd[c]);
  int rs = kStepRows;  // rows per step that fit the staging pool
  for (;;) {
    int need = 0;
#pragma unroll
    for (int c = 0; c < kMaxComp; c++)
      if (c < A.ncomp) need += (A.cg[c].rv == 2 ? rs / 2 + 2 : rs) * nd[c];
    if (need <= kStageDW || rs == 1) break;
    rs--;
  }
  const int xx = ox0 + t;
  const bool active = xx < ox1;
  // this column's horizontal window, relative to the tile's first source column
  int hm = 0, hc = 1;
  const int32_t* kp = A.kh;
  if (active) {
    if (A.need_h) {
      hm = A.bh[2 * xx] - s_lo;
      hc = A.bh[2 * xx + 1];
      kp = A.kh + (int64_t)xx * A.ksh;
    } else {
      hm = xx - s_lo;
    }
  }
  int32_t cf[KT > 0 ? KT : 1];
#pragma unroll
  for (int j = 0; j < (KT > 0 ? KT : 1); j++)
    cf[j] = !A.need_h ? (j == 0 ? (1 << 22) : 0) : (active && j < hc ? kp[j] : 0);
  // the strip's vertical windows and weights (identity when there is no vertical pass)
  for (int i = t; i < (A.oy1 - A.oy0) * kVTaps; i += kRsThreads) {
    const int b = i / kVTaps, k = i % kVTaps, oy = A.oy0 + b;
    if (k == 0) {
      L.vb[b][0] = A.need_v ? A.bv[2 * oy] : oy;
      L.vb[b][1] = A.need_v ? A.bv[2 * oy + 1] : 1;
    }
    L.vw[b][k] = A.need_v ? (k < A.ksv ? A.kv[(int64_t)oy * A.ksv + k] : 0) : (k == 0 ? (1 << 22) : 0);
  }
  const uint8_t* hp = &L.rgb[0][0][0] + hm;
  uint32_t* ring = L.ring + t;
  const int ox = A.fl ? A.ow - 1 - xx : xx;
  int nb = A.oy0;  // next output row to finish

  for (int ra = r_lo; ra < r_hi; ra += rs) {
    const int rb = ra + rs < r_hi ? ra + rs : r_hi;  // crop rows [ra, rb) this step
    const int ya = A.cy0 + ra, yb = A.cy0 + rb;     // image rows
    // A. stage the plane rows: one global_load_lds_dword per 64 dwords of a row, rows spread over
    // the waves (LDS destination = wave-uniform base + lane * 4)
    int soff[kMaxComp] = {0, 0, 0}, ilo[kMaxComp] = {0, 0, 0};
    {
      int o = 0, chunk = 0;
#pragma unroll
      for (int c = 0; c < kMaxComp; c++) {
        soff[c] = o;
        if (c >= A.ncomp) continue;
        const CompDesc& cd = A.cg[c];
        int ihi;
        comp_rows(cd, ya, yb, &ilo[c], &ihi);
        const int nch = (nd[c] + 63) >> 6;
        for (int i = ilo[c]; i <= ihi; i++) {
          const uint8_t* g = A.planes + cd.plane_off + (int64_t)i * cd.pitch + jal[c];
          for (int h = 0; h < nch; h++, chunk++) {
            if ((chunk & 3) != wv) continue;
            const int k = h * 64 + lane;
            if (k < nd[c])
              __builtin_amdgcn_global_load_lds(
                  (const __attribute__((address_space(1))) void*)(g + 4 * k),
                  (__attribute__((address_space(3))) void*)(L.st + o + (i - ilo[c]) * nd[c] + h * 64), 4, 0, 0);
          }
        }
        o += (ihi - ilo[c] + 1) * nd[c];
      }
    }
    __syncthreads();  // DMA landed (vmcnt(0)); previous step's H reads of rgb are done
    // B. upsample + colour convert
    for (int q = 0; q < rb - ra; q++) convert_row(L, A, q, ya + q, ax0, ax1, soff, ilo, nd, jal);
    __syncthreads();
    if (active) {
#pragma unroll
      for (int q = 0; q < kStepRows; q++) {
        if (q >= rb - ra) break;
        // H. horizontal pass of step row q -> ring slot (row & rmask)
        int32_t s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
        const uint8_t* pr = hp + q * 3 * kRgbW;
        if (KT > 0) {
#pragma unroll
          for (int j = 0; j < (KT > 0 ? KT : 1); j++) {
            s0 += tap(pr[j], cf[j]);
            s1 += tap(pr[kRgbW + j], cf[j]);
            s2 += tap(pr[2 * kRgbW + j], cf[j]);
          }
        } else {
          for (int j = 0; j < hc; j++) {
            const int32_t c = kp[j];
            s0 += tap(pr[j], c);
            s1 += tap(pr[kRgbW + j], c);
            s2 += tap(pr[2 * kRgbW + j], c);
          }
        }
        const int r = ra + q;
        ring[(r & A.rmask) * A.rstride] =
            pack3(rs_clip8(s0), rs_clip8(s1), rs_clip8(s2));
        // V. output rows whose window [vmin, vmin + vcnt) ends at row r (ring_rows >= ksv keeps
        // the whole window; own column only, so no barrier)
        for (;;) {
          if (nb >= A.oy1) break;
          const int vmin = __builtin_amdgcn_readfirstlane(L.vb[nb - A.oy0][0]);
          const int vcnt = __builtin_amdgcn_readfirstlane(L.vb[nb - A.oy0][1]);
          if (vmin + vcnt > r + 1) break;
          int32_t v0 = 1 << 21, v1 = 1 << 21, v2 = 1 << 21;
          const int32_t* wk = L.vw[nb - A.oy0];
          for (int k = 0; k < vcnt; k++) {
            const uint32_t h = ring[((vmin + k) & A.rmask) * A.rstride];
            const int32_t w = wk[k];
            v0 += tap((int32_t)(h & 0xFF), w);
            v1 += tap((int32_t)((h >> 8) & 0xFF), w);
            v2 += tap((int32_t)(h >> 16), w);
          }
          put3(A.out, A.om, A.lut, (int64_t)nb * A.ow + ox, rs_clip8(v0), rs_clip8(v1), rs_clip8(v2));
          nb++;
        }
      }
    }
  }
}

// One image's share (output rows of strip `strip`, column tiles tz0, tz0 + ntz, ...) of the generic
// fused colour + resample (route gen_route(KT); status and zero outputs: k_finish).  One
// instantiation per horizontal tap count keeps each kernel's registers to what that count needs.
template <int KT>
__device__ void resample_image(int img, int strip, int tz0, int ntz, const ImgDesc* __restrict__ descs,
                               const sdsj_op& op, int strip_h, const uint8_t* __restrict__ scratch,
                               const uint8_t* __restrict__ flip, void* __restrict__ out, const float* __restrict__ lut) {
  const ImgDesc* d = &descs[img];
  RsArgs A;
  A.ow = op.out_w;
  A.oh = op.out_h;
  const int64_t plane = (int64_t)A.oh * A.ow;
  A.om.f32 = op.out_dtype == SDSJ_DTYPE_F32;
  A.om.base = (int64_t)img * plane * 3;
  A.om.ps = op.layout == SDSJ_LAYOUT_HWC ? 3 : 1;
  A.om.cs = op.layout == SDSJ_LAYOUT_HWC ? 1 : plane;
  A.lut = lut;
  A.out = out;
  A.oy0 = strip * strip_h;
  if (A.oy0 >= A.oh) return;
  A.oy1 = A.oy0 + strip_h < A.oh ? A.oy0 + strip_h : A.oh;
  if (d->status != SDSJ_OK) return;  // failed after planning: k_finish writes the zeros
  __shared__ LdsResample L;
  A.d = d;
  A.dmut = const_cast<ImgDesc*>(d);
  A.fl = flip ? flip[img] != 0 : false;
  A.need_h = d->need_h;
  A.need_v = d->need_v;
  A.bh = reinterpret_cast<const int32_t*>(scratch + d->off_kh);  // [2 * ow] bounds, [ow * ksh] coefficients
  A.kh = A.bh + 2 * A.ow;
  A.bv = reinterpret_cast<const int32_t*>(scratch + d->off_kv);
  A.kv = A.bv + 2 * A.oh;
  A.ksh = d->ksh;
  A.ksv = d->ksv;
  A.planes = scratch + d->off_planes;
  A.ncomp = d->ncomp;
  A.cx0 = d->cx0;
  A.cy0 = d->cy0;
  A.tw = d->tile_w;
  A.ntiles = (A.ow + A.tw - 1) / A.tw;
  A.rmask = d->ring_rows - 1;
  A.rstride = kRingDW / d->ring_rows;
  for (int c = 0; c < kMaxComp; c++) A.cg[c] = d->comp[c];
  const CompDesc &c0 = A.cg[0], &c1 = A.cg[1], &c2 = A.cg[2];
  A.layout = kLayGeneric;
  if (c0.rh == 1 && c0.rv == 1) {
    if (A.ncomp == 1 || (c1.rh == 1 && c1.rv == 1 && c2.rh == 1 && c2.rv == 1)) A.layout = kLayFull;
    else if (c1.rh == 2 && c1.rv == 2 && c2.rh == 2 && c2.rv == 2 && c1.dw > 2 && c2.dw == c1.dw) A.layout = kLay420;
  }
  for (int tile = tz0; tile < A.ntiles; tile += ntz) {
    resample_tile<KT>(L, A, tile);
    __syncthreads();  // LDS reuse by the next tile
  }
}

template <int KT>
__global__ void __launch_bounds__(kRsThreads) k_resample(int n, const ImgDesc* __restrict__ descs, sdsj_op op,
                                                         int strip_h, int strips, int ntz,
                                                         const uint8_t* __restrict__ scratch,
                                                         const uint8_t* __restrict__ flip, void* __restrict__ out,
                                                         const int32_t* __restrict__ routes, int cap,
                                                         const float* __restrict__ lut) {
  constexpr int r = KT == 0 ? kRtGen0 : (KT == 1 ? kRtGen1 : kRtGen3 + (KT - 3) / 2);
  const int cnt = routes[r];
  const int32_t* lst = route_list(routes, cap, r);
  // work items (route entry, strip, tile column) over the grid, as k_rs420
  const int per = strips * ntz;
  const int64_t items = (int64_t)cnt * per;
  for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
    const int e = (int)(it / per), rem = (int)(it - (int64_t)e * per), strip = rem / ntz;
    resample_image<KT>(lst[e], strip, rem - strip * ntz, ntz, descs, op, strip_h, scratch, flip, out, lut);
  }
}

hipError_t launch_resample(int n, const ImgDesc* descs, const sdsj_op& op, const uint8_t* scratch, const uint8_t* flip,
                           void* out, int32_t* status, const int32_t* routes, int cap, const float* lut, hipStream_t s,
                           uint64_t rm, uint64_t hint) {
  // strips of output rows: tall for big batches (less window overlap), short for small ones
  const int strip_h = n >= 512 ? kMaxStrip : 16;
  const int tiles = (op.out_w + kRsThreads - 1) / kRsThreads;
  const int strips = (op.out_h + strip_h - 1) / strip_h;
  const int64_t full = (int64_t)(n < kRsfEntries ? n : kRsfEntries) * strips * tiles;
  if (route_on(rm, kRtGen0)) hipLaunchKernelGGL(k_resample<0>, dim3(route_grid(hint, kRtGen0, full)), dim3(kRsThreads), 0, s, n, descs, op, strip_h, strips, tiles, scratch, flip, out, routes, cap, lut);
  if (route_on(rm, kRtGen1)) hipLaunchKernelGGL(k_resample<1>, dim3(route_grid(hint, kRtGen1, full)), dim3(kRsThreads), 0, s, n, descs, op, strip_h, strips, tiles, scratch, flip, out, routes, cap, lut);
  if (route_on(rm, kRtGen3)) hipLaunchKernelGGL(k_resample<3>, dim3(route_grid(hint, kRtGen3, full)), dim3(kRsThreads), 0, s, n, descs, op, strip_h, strips, tiles, scratch, flip, out, routes, cap, lut);
  if (route_on(rm, kRtGen5)) hipLaunchKernelGGL(k_resample<5>, dim3(route_grid(hint, kRtGen5, full)), dim3(kRsThreads), 0, s, n, descs, op, strip_h, strips, tiles, scratch, flip, out, routes, cap, lut);
  if (route_on(rm, kRtGen7)) hipLaunchKernelGGL(k_resample<7>, dim3(route_grid(hint, kRtGen7, full)), dim3(kRsThreads), 0, s, n, descs, op, strip_h, strips, tiles, scratch, flip, out, routes, cap, lut);
  if (route_on(rm, kRtGen9)) hipLaunchKernelGGL(k_resample<9>, dim3(route_grid(hint, kRtGen9, full)), dim3(kRsThreads), 0, s, n, descs, op, strip_h, strips, tiles, scratch, flip, out, routes, cap, lut);
  if (route_on(rm, kRtGen11)) hipLaunchKernelGGL(k_resample<11>, dim3(route_grid(hint, kRtGen11, full)), dim3(kRsThreads), 0, s, n, descs, op, strip_h, strips, tiles, scratch, flip, out, routes, cap, lut);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  (void)status;  // published by k_finish after every resample variant
  return launch_resample420(n, descs, op, strip_h, scratch, flip, out, routes, cap, lut, s, rm, hint);
}

}  // namespace sdsj
