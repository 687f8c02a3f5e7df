// sdsj_resample420.hip -- the fused colour + resample kernels specialised by chroma layout:
// 4:2:0 YCbCr (h2v2 fancy chroma), 4:2:2 (h2v1 fancy chroma), 4:4:4 and grayscale, with a
// horizontal and a vertical Pillow pass of KT taps (odd, 3..11).  Same arithmetic and the same
// streaming structure as k_resample (sdsj_resample.hip, whose header describes the phases and the
// reference lines), with the per-image geometry fixed at compile time where it matters:
//   * the plane rows of the next step go straight to LDS (global_load_lds, issued once this step's
//     conversion has read the staged rows; grayscale: through registers, its H pass reads them);
//   * conversion is one flattened loop over (step row, 8-pixel group); each item reads its luma and
//     chroma as aligned dwords from the staged rows and writes each channel's 8 pixels as 2 dwords
//     (grayscale has no conversion: the horizontal taps read the staged luma rows, and one channel
//     goes through the H and V passes and is written to all three outputs -- Image.convert('RGB') of
//     an 'L' image repeats it);
//   * staging offsets of the step's rows come from a small LDS table, not from uniform registers
//     (keeps the scalar file from spilling);
//   * the horizontal taps are KT exactly, coefficients in registers, windows read as aligned dwords.
// plan_image sets ImgDesc::rs_fast = KT and rs_lay for the images these kernels take; k_resample
// skips them.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sdsj_common.h"
#include "sdsj_kernels.h"
#include "sdsj_pixel.h"

namespace sdsj {

constexpr int kFThreads = 256;
#ifndef SDSJ_FROWS
#define SDSJ_FROWS 4
#endif
constexpr int kFRows = SDSJ_FROWS;       // source rows per step
// Per layout and tap count: source columns per staged row (rs_span), staged luma and chroma row widths
// (dwords), staged rows (luma + both chroma planes), RGB rows and their pitch (bytes).
template <int LAY, int KT>
struct FGeo {
  static constexpr int kSpan = rs_span(KT);
  static constexpr int kYDW = kSpan / 4 + 2;  // staged luma (full-width) row
  static constexpr int kCDW = LAY == kRs444 ? kYDW : (LAY == kRsGray ? 0 : kSpan / 8 + 3);
  // staged rows per chroma plane: 4:2:0 reads rows y >> 1 and their vertical neighbours, at most
  // kFRows / 2 + 2 of them for kFRows luma rows; the other layouts the luma rows' own
  static constexpr int kCRows = LAY == kRsGray ? 0 : (LAY == kRs420 ? kFRows / 2 + 2 : kFRows);
  static constexpr int kStageDW = kFRows * kYDW + 2 * kCRows * kCDW;
  static constexpr int kRgbRows = LAY == kRsGray ? 0 : kFRows;
  static constexpr int kRgbW = kSpan + 32;  // (even)
  static constexpr int kRows = kFRows + 2 * kCRows;  // staged rows per step at most
};

template <int LAY, int KT>
struct LdsF {
  using G = FGeo<LAY, KT>;
  alignas(16) uint32_t st[G::kStageDW];                                  // step's plane rows: 4 luma, then Cb, Cr
  alignas(16) uint8_t rgb[G::kRgbRows > 0 ? G::kRgbRows : 1][3][G::kRgbW];  // converted rows, planar
  uint32_t ring[rs_ring_dw(KT)];                             // per column: H results of the last R rows
  int32_t vb[kMaxStrip][2];                                  // strip rows: vertical window (first, count)
  int32_t vw[kMaxStrip][rs_vtaps(KT)];                       // strip rows: vertical weights
  int32_t rinfo[kFRows][8];                                  // step row q: byte offsets of its staged rows
};

// Pillow horizontal pass of one channel at one output column: KT taps from the byte window that
// starts hsh bytes into dword w[0] (accumulator from 1 << 21, clip8 after >> 22).
template <int KT>
__device__ __forceinline__ int htaps(const uint32_t* w, int hsh, const int32_t* cf) {
  constexpr int ND = (KT + 3 + 3) / 4 + 1;  // dwords covering hsh + KT bytes, + 1 for the realign
  uint32_t d[ND];
#pragma unroll
  for (int i = 0; i < ND; i++) d[i] = w[i];
  int32_t acc = 1 << 21;
#pragma unroll
  for (int g = 0; g * 4 < KT; g++) {
    const uint32_t v = __builtin_amdgcn_alignbyte(d[g + 1], d[g], hsh);  // bytes hsh + 4g ..
#pragma unroll
    for (int k = 0; k < 4 && g * 4 + k < KT; k++) acc += tap((int32_t)((v >> (8 * k)) & 0xFF), cf[g * 4 + k]);
  }
  return rs_clip8(acc);
}

// Pillow vertical pass of one output pixel from the ring (KT <= 7: 8 rows of 256 columns), window
// starting at ring row P: every tap's row is a compile-time offset from the lane's column, so the
// reads need no address arithmetic (rsf_image picks P = vmin & 7 with a uniform switch).
template <int KT, int P, bool GRAY>
__device__ __forceinline__ void vtaps8(const uint32_t* ring, int lane_col, const int32_t* wk, int32_t& v0, int32_t& v1,
                                       int32_t& v2) {
  // (the empty asm keeps the column index a value of this block, so each tap's row becomes the
  // read's immediate offset instead of one of 8 addresses held in registers through the loop)
  asm volatile("" : "+v"(lane_col));
#pragma unroll
  for (int k = 0; k < KT; k++) {
    const uint32_t h = ring[lane_col + ((P + k) & 7) * 256];
    const int32_t w = wk[k];
    if (GRAY) {
      v0 += tap((int32_t)h, w);
    } else {
      v0 += tap((int32_t)(h & 0xFF), w);
      v1 += tap((int32_t)((h >> 8) & 0xFF), w);
      v2 += tap((int32_t)(h >> 16), w);
    }
  }
}

template <int KT, bool GRAY>
__device__ __forceinline__ void vtaps8_at(int p, const uint32_t* ring, int lane_col, const int32_t* wk, int32_t& v0,
                                          int32_t& v1, int32_t& v2) {
  switch (__builtin_amdgcn_readfirstlane(p)) {  // (uniform: scalar compares, no exec masking)
    case 0: vtaps8<KT, 0, GRAY>(ring, lane_col, wk, v0, v1, v2); break;
    case 1: vtaps8<KT, 1, GRAY>(ring, lane_col, wk, v0, v1, v2); break;
    case 2: vtaps8<KT, 2, GRAY>(ring, lane_col, wk, v0, v1, v2); break;
    case 3: vtaps8<KT, 3, GRAY>(ring, lane_col, wk, v0, v1, v2); break;
    case 4: vtaps8<KT, 4, GRAY>(ring, lane_col, wk, v0, v1, v2); break;
    case 5: vtaps8<KT, 5, GRAY>(ring, lane_col, wk, v0, v1, v2); break;
    case 6: vtaps8<KT, 6, GRAY>(ring, lane_col, wk, v0, v1, v2); break;
    default: vtaps8<KT, 7, GRAY>(ring, lane_col, wk, v0, v1, v2); break;
  }
}

template <int KT, int LAY>
__device__ void rsf_image(int img, int strip, int tz0, int ntz, const ImgDesc* __restrict__ descs, const sdsj_op& op,
                          int strip_h, const uint8_t* __restrict__ scratch, const uint8_t* __restrict__ flip,
                          void* __restrict__ out, const float* __restrict__ lut);

// Route (LAY, KT): a small grid strides over the route's list (an empty route costs one short launch).
// Occupancy: the KT <= 7 kernels' LDS (the smaller ring and weight table, 768-column rows: 26.1 KB)
// fits 6 workgroups per CU, and 6 waves per SIMD fit their registers without spills (<= 85 VGPRs with
// the staged-row loops' addressing scalar): k_rs420<5> 29.6 -> 28.0 ms per 65,536 images
// (profiles/r05_ab.txt; 5 waves at 30.6 KB: 9.95 -> 9.23 ms per 16,384 in round 3,
// profiles/r03b_rs420_occupancy_ab.txt).  4:4:4 at KT <= 7 (full-width chroma rows: 30 KB) takes 5;
// the 9- and 11-tap kernels keep 4.
#ifndef SDSJ_RS_WAVES
#define SDSJ_RS_WAVES 6
#endif
#define SDSJ_RS_OCC __attribute__((amdgpu_waves_per_eu(KT <= 7 ? (LAY != kRs444 ? SDSJ_RS_WAVES : 5) : 4)))
template <int KT, int LAY>
__global__ void __launch_bounds__(kFThreads) SDSJ_RS_OCC k_rs420(int n, const ImgDesc* __restrict__ descs, sdsj_op op,
                                                      int strip_h, int strips, int ntz, const uint8_t* __restrict__ scratch,
                                                      const uint8_t* __restrict__ flip, void* __restrict__ out,
                                                      const int32_t* __restrict__ routes, int cap,
                                                      const float* __restrict__ lut) {
  const int r = rs_route(LAY, KT);
  const int cnt = routes[r];
  const int32_t* lst = route_list(routes, cap, r);
  // work items (route entry, strip, tile column), an image's strips consecutive; the grid (one item per
  // workgroup up to kRsfEntries entries, a cold route's small grid: route_grid) strides over them
  const int per = strips * ntz;
  const int64_t items = (int64_t)cnt * per;
  for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
    const int e = (int)(it / per), rem = (int)(it - (int64_t)e * per), strip = rem / ntz;
    rsf_image<KT, LAY>(lst[e], strip, rem - strip * ntz, ntz, descs, op, strip_h, scratch, flip, out, lut);
  }
}

// One image's share (output strip `strip`, column tiles tz0, tz0 + ntz, ...) of the fused resample.
template <int KT, int LAY>
__device__ void rsf_image(int img, int strip, int tz0, int ntz, const ImgDesc* __restrict__ descs, const sdsj_op& op,
                          int strip_h, const uint8_t* __restrict__ scratch, const uint8_t* __restrict__ flip,
                          void* __restrict__ out, const float* __restrict__ lut) {
  using G = FGeo<LAY, KT>;
  const ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK || d->rs_fast != KT || d->rs_lay != LAY) return;
  const int oh = op.out_h, ow = op.out_w;
  const int oy0 = strip * strip_h;
  if (oy0 >= oh) return;
  const int oy1 = oy0 + strip_h < oh ? oy0 + strip_h : oh;
  __shared__ LdsF<LAY, KT> L;
  constexpr int kVT = rs_vtaps(KT);
  // (the wave index through readfirstlane: the staged-row loops' row tests and plane addresses are
  // then scalar work, off the VALU this kernel is bound by)
  const int t = threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const int64_t plane = (int64_t)oh * ow;
  OutMap om;
  om.f32 = op.out_dtype == SDSJ_DTYPE_F32;
  om.base = (int64_t)img * plane * 3;
  om.ps = op.layout == SDSJ_LAYOUT_HWC ? 3 : 1;
  om.cs = op.layout == SDSJ_LAYOUT_HWC ? 1 : plane;
  const bool fl = flip ? flip[img] != 0 : false;
  const int32_t* bh = reinterpret_cast<const int32_t*>(scratch + d->off_kh);
  const int32_t* kh = bh + 2 * ow;
  const int32_t* bv = reinterpret_cast<const int32_t*>(scratch + d->off_kv);
  const int32_t* kv = bv + 2 * oh;
  const int ksv = d->ksv, cx0 = d->cx0, cy0 = d->cy0, tw = d->tile_w;
  // KT <= 7: the ring is always 8 rows of 256 columns (plan_image: ksv <= 8, tile_w <= 256), so its
  // row offsets are compile-time constants
  constexpr bool kRing8 = KT <= 7;
  static_assert(!kRing8 || (rs_ring_rows(KT) == 8 && rs_ring_dw(KT) == 8 * 256), "ring geometry");
  const int rmask = kRing8 ? 7 : d->ring_rows - 1, rstride = kRing8 ? 256 : rs_ring_dw(KT) / d->ring_rows;
  const int dwc = LAY == kRsGray ? 0 : d->comp[1].dw, dhc = LAY == kRsGray ? 0 : d->comp[1].dh;
  const uint8_t* pY = scratch + d->off_planes + d->comp[0].plane_off;
  const uint8_t* pCb = LAY == kRsGray ? pY : scratch + d->off_planes + d->comp[1].plane_off;
  const uint8_t* pCr = LAY == kRsGray ? pY : scratch + d->off_planes + d->comp[2].plane_off;
  const int pitchY = d->comp[0].pitch, pitchC = LAY == kRsGray ? 0 : d->comp[1].pitch;
  const int ntiles = (ow + tw - 1) / tw;
  const int r_lo = bv[2 * oy0], r_hi = bv[2 * (oy1 - 1)] + bv[2 * (oy1 - 1) + 1];
  // the strip's vertical windows and weights
  for (int i = t; i < (oy1 - oy0) * kVT; i += kFThreads) {
    const int b = i / kVT, k = i % kVT, oy = oy0 + b;
    if (k == 0) {
      L.vb[b][0] = bv[2 * oy];
      L.vb[b][1] = bv[2 * oy + 1];
    }
    L.vw[b][k] = k < ksv ? kv[(int64_t)oy * ksv + k] : 0;
  }

  for (int tile = tz0; tile < ntiles; tile += ntz) {
    const int ox0 = tile * tw, ox1 = ox0 + tw < ow ? ox0 + tw : ow;
    const int s_lo = bh[2 * ox0], s_hi = bh[2 * (ox1 - 1)] + bh[2 * (ox1 - 1) + 1];
    const int ax0 = cx0 + s_lo, ax1 = cx0 + s_hi;  // image columns of the tile
    // 8-pixel groups: luma columns [xb, xb + 8 ng) with xb 8-aligned (dword writes); half-width
    // chroma columns [jb - 4, jb + 4 ng + 4) (the fancy upsampling reads one neighbour each side),
    // full-width chroma (4:4:4) columns [xb, xb + 8 ng).  Bytes past a row end (or before the first
    // one) come from neighbouring scratch and only feed pixels outside the tile.
    const int jb = (ax0 >> 1) & ~3;
    const int xb = 2 * jb;
    const int ng = (ax1 - 1 - xb) / 8 + 1;
    const int jalY = xb, ndY = 2 * ng;
    const int jalC = LAY == kRs444 ? xb : jb - 4, ndC = LAY == kRs444 ? 2 * ng : ng + 2;
    const int xx = ox0 + t;
    const bool active = xx < ox1;
    int hm = 0, hc = 0;
    if (active) {
      hm = bh[2 * xx] - s_lo + (ax0 - xb);
      hc = bh[2 * xx + 1];
    }
    int32_t cf[KT];
#pragma unroll
    for (int j = 0; j < KT; j++) cf[j] = active && j < hc ? kh[(int64_t)xx * KT + j] : 0;
    // H windows: the converted RGB rows, or (grayscale) the staged luma rows themselves
    const uint32_t* hw = LAY == kRsGray ? L.st + (hm >> 2) : reinterpret_cast<const uint32_t*>(&L.rgb[0][0][0]) + (hm >> 2);
    const int hsh = hm & 3;
    uint32_t* ring = L.ring + t;
    const int ox = fl ? ow - 1 - xx : xx;
    int nb = oy0;

    // Plane rows of a step (4 source rows): luma rows ya..; chroma rows ilo..ilo + nrc - 1 -- for
    // 4:2:0 the rows the h2v2 fancy upsampling reads (row i = y >> 1 and its neighbour f = i -/+ 1
    // for even/odd y, clamped: at most 4 per plane), otherwise the luma rows' own.
    struct Step {
      int ra, nr, ya, ilo, nrc;
    };
    auto plan_step = [&](int ra) {
      Step p;
      p.ra = ra;
      p.nr = r_hi - ra < kFRows ? r_hi - ra : kFRows;
      p.ya = cy0 + ra;
      if (LAY == kRs420) {
        int ilo = ((p.ya + 1) >> 1) - 1, ihi = (p.ya + p.nr) >> 1;
        ilo = ilo < 0 ? 0 : ilo;
        ihi = ihi > dhc - 1 ? dhc - 1 : ihi;
        p.ilo = ilo;
        p.nrc = ihi - ilo + 1;
      } else {
        p.ilo = p.ya;
        p.nrc = LAY == kRsGray ? 0 : p.nr;
      }
      return p;
    };
    // Grayscale: the next step's rows travel through registers (global loads issued before this
    // step's H pass, written to LDS after it), so their latency hides behind a whole step.  Wave wv
    // holds staged rows wv, wv + 4, wv + 8 (<= 12 rows), 64 dwords per load.  Colour layouts
    // (kGlds): the same rows and lanes, loaded straight into LDS by issue_lds below.
    constexpr int kPR = (G::kRows + 3) / 4, kPC = (G::kSpan / 4 + 2 + 63) / 64;
    constexpr bool kGlds = LAY != kRsGray;
    uint32_t pre[kPR][kPC];
    auto row_src = [&](const Step& p, int row, const uint8_t*& g, int& nd, int& o) {
      if (row < p.nr) {
        g = pY + (int64_t)(p.ya + row) * pitchY + jalY;
        nd = ndY;
        o = row * G::kYDW;
      } else if (row < p.nr + p.nrc) {
        g = pCb + (int64_t)(p.ilo + row - p.nr) * pitchC + jalC;
        nd = ndC;
        o = kFRows * G::kYDW + (row - p.nr) * G::kCDW;
      } else {
        g = pCr + (int64_t)(p.ilo + row - p.nr - p.nrc) * pitchC + jalC;
        nd = ndC;
        o = kFRows * G::kYDW + G::kCRows * G::kCDW + (row - p.nr - p.nrc) * G::kCDW;
      }
    };
    auto issue = [&](const Step& p) {
#pragma unroll
      for (int i = 0; i < kPR; i++) {
        const int row = wv + 4 * i;
        if (row < p.nr + 2 * p.nrc) {
          const uint8_t* g;
          int nd, o;
          row_src(p, row, g, nd, o);
          const uint32_t* g4 = reinterpret_cast<const uint32_t*>(g);
#pragma unroll
          for (int h = 0; h < kPC; h++)
            if (64 * h + lane < nd) pre[i][h] = __builtin_nontemporal_load(g4 + 64 * h + lane);
        }
      }
    };
    // Colour layouts: the next step's rows go straight to LDS (global_load_lds, no
    // register staging), issued after this step's conversion has read the staged rows; the step-end
    // barrier retires them.
    auto issue_lds = [&](const Step& p) {
#pragma unroll
      for (int i = 0; i < kPR; i++) {
        const int row = wv + 4 * i;
        if (row < p.nr + 2 * p.nrc) {
          const uint8_t* g;
          int nd, o;
          row_src(p, row, g, nd, o);
          const uint32_t* g4 = reinterpret_cast<const uint32_t*>(g);
#pragma unroll
          for (int h = 0; h < kPC; h++)
            if (64 * h + lane < nd)
              __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g4 + 64 * h + lane),
                                               (__attribute__((address_space(3))) void*)(&L.st[o + 64 * h]), 4, 0, 0);
        }
      }
    };
    auto commit = [&](const Step& p) {
#pragma unroll
      for (int i = 0; i < (kGlds ? 0 : kPR); i++) {
        const int row = wv + 4 * i;
        if (row < p.nr + 2 * p.nrc) {
          const uint8_t* g;
          int nd, o;
          row_src(p, row, g, nd, o);
#pragma unroll
          for (int h = 0; h < kPC; h++)
            if (64 * h + lane < nd) L.st[o + 64 * h + lane] = pre[i][h];
        }
      }
      if (LAY != kRsGray && t < p.nr) {
        const int y = p.ya + t;
        int i = y - p.ilo, f = i;  // staged chroma row of this luma row, and its vertical neighbour
        if (LAY == kRs420) {
          const int ci = y >> 1;
          int cfr = (y & 1) ? ci + 1 : ci - 1;
          cfr = cfr < 0 ? 0 : (cfr > dhc - 1 ? dhc - 1 : cfr);
          i = ci - p.ilo;
          f = cfr - p.ilo;
        }
        L.rinfo[t][0] = 4 * (t * G::kYDW) - jalY;
        L.rinfo[t][1] = 4 * (kFRows * G::kYDW + i * G::kCDW) - jalC;
        L.rinfo[t][2] = 4 * (kFRows * G::kYDW + f * G::kCDW) - jalC;
        L.rinfo[t][3] = 4 * (kFRows * G::kYDW + G::kCRows * G::kCDW + i * G::kCDW) - jalC;
        L.rinfo[t][4] = 4 * (kFRows * G::kYDW + G::kCRows * G::kCDW + f * G::kCDW) - jalC;
      }
    };
    Step cur = plan_step(r_lo);
    if (kGlds) issue_lds(cur);
    else issue(cur);
    commit(cur);
    __syncthreads();
    // the next output row's window (uniform, carried in scalars): first row, and one past its last
    auto window = [&](int row, int& vmin, int& vend) {
      vmin = __builtin_amdgcn_readfirstlane(L.vb[row - oy0][0]);
      vend = vmin + __builtin_amdgcn_readfirstlane(L.vb[row - oy0][1]);
    };
    int nvmin, nvend;
    window(oy0, nvmin, nvend);
    for (int ra = r_lo; ra < r_hi; ra += kFRows) {
      const int nr = cur.nr;
      const bool more = ra + kFRows < r_hi;
      const Step nxt = more ? plan_step(ra + kFRows) : cur;
      if (more && !kGlds) issue(nxt);
      if (LAY != kRsGray) {
        // B. fancy upsampling + ycc->rgb on 8 pixels per item
        // items of one step row per wave (64 item slots per row, 128 when the tile needs more than 64
        // groups): a wave's chroma and luma reads then never straddle two rows, whose words met
        // bank conflicts, and its row is uniform
        static_assert(G::kSpan / 8 + 2 <= 128, "a row's items fit two waves");
        const int rsh = ng > 64 ? 7 : 6;
        for (int it = t; it < (nr << rsh); it += kFThreads) {
          const int q = __builtin_amdgcn_readfirstlane(it >> rsh);  // step row of the item
          const int gi = it - (q << rsh);
          if (gi >= ng) continue;
          const int x = xb + 8 * gi, jg = x >> 1;
          const int oY = L.rinfo[q][0], oBi = L.rinfo[q][1], oRi = L.rinfo[q][3];
          const uint32_t* sw = L.st;
          const uint8_t* sb = reinterpret_cast<const uint8_t*>(L.st);  // (byte offsets: rinfo's are bytes)
          // the item's 8 luma bytes as one 8-byte read (oY + x is 8-aligned: G::kYDW is even, xb and x are
          // multiples of 8): consecutive items 8 bytes apart fill all 64 banks, where two dword reads at
          // a 2-dword lane stride met 2-way bank conflicts
          static_assert(G::kYDW % 2 == 0, "8-byte aligned luma rows");
          const uint2 yy = *reinterpret_cast<const uint2*>(sb + oY + x);
          const uint32_t y0 = yy.x, y1 = yy.y;
          uint32_t wr[2] = {0, 0}, wg[2] = {0, 0}, wb[2] = {0, 0};
          if (LAY == kRs444) {
            const uint32_t cbw[2] = {sw[(oBi + x) >> 2], sw[(oBi + x + 4) >> 2]};
            const uint32_t crw[2] = {sw[(oRi + x) >> 2], sw[(oRi + x + 4) >> 2]};
#pragma unroll
            for (int k = 0; k < 8; k++) {
              const int sh = 8 * (k & 3);
              const uint32_t yw = k < 4 ? y0 : y1;
              int r, g, b;
              ycc_px((int)((yw >> sh) & 0xFF), (int)((cbw[k >> 2] >> sh) & 0xFF) - 128,
                     (int)((crw[k >> 2] >> sh) & 0xFF) - 128, r, g, b);
              wr[k >> 2] |= (uint32_t)r << sh;
              wg[k >> 2] |= (uint32_t)g << sh;
              wb[k >> 2] |= (uint32_t)b << sh;
            }
          } else if (LAY == kRs420) {
            // h2v2 fancy upsampling (jdsample.c): the chroma column sums 3 * row_i + row_f of columns
            // jg - 1 .. jg + 4, then per output pixel (3 * own + neighbour + 8 or 7) >> 4.  Interior
            // items take two columns per 32-bit op (16-bit halves: sums <= 4,088, no carries); items
            // at the plane's edges (repeated columns) the per-column path.
            const int oBf = L.rinfo[q][2], oRf = L.rinfo[q][4];
            int ube[4], ubo[4], ure[4], uro[4];  // upsampled Cb / Cr of the even / odd pixel of column jg + k
            auto up = [&](int oi, int of, int* ue, int* uo) {
              // (oi + jg and of + jg are multiples of 4: rinfo's offsets and jalC, jb and jg are; one address
              // per row, the neighbour dwords at immediate offsets)
              const uint32_t* wi = reinterpret_cast<const uint32_t*>(sb + oi + jg);
              const uint32_t* wf = reinterpret_cast<const uint32_t*>(sb + of + jg);
              const uint32_t i0 = wi[-1], i1 = wi[0], i2 = wi[1];
              const uint32_t f0 = wf[-1], f1 = wf[0], f2 = wf[1];
              if (jg > 0 && jg + 4 <= dwc - 1) {
                constexpr uint32_t M = 0x00FF00FFu;
                const uint32_t E = (i1 & M) * 3 + (f1 & M), O = ((i1 >> 8) & M) * 3 + ((f1 >> 8) & M);  // [jg, jg+2], [jg+1, jg+3]
                const uint32_t l = (i0 >> 24) * 3 + (f0 >> 24), rr = (i2 & 0xFF) * 3 + (f2 & 0xFF);    // jg - 1, jg + 4
                const uint32_t A = E * 3 + (l | (O << 16)) + 0x00080008u;
                const uint32_t B = E * 3 + O + 0x00070007u;
                const uint32_t C = O * 3 + E + 0x00080008u;
                const uint32_t D = O * 3 + ((E >> 16) | (rr << 16)) + 0x00070007u;
                ue[0] = (int)((A >> 4) & 0xFFF);
                ue[1] = (int)((C >> 4) & 0xFFF);
                ue[2] = (int)(A >> 20);
                ue[3] = (int)(C >> 20);
                uo[0] = (int)((B >> 4) & 0xFFF);
                uo[1] = (int)((D >> 4) & 0xFFF);
                uo[2] = (int)(B >> 20);
                uo[3] = (int)(D >> 20);
              } else {
                int c[6];
                c[0] = (int)(i0 >> 24) * 3 + (int)(f0 >> 24);
#pragma unroll
                for (int k = 0; k < 4; k++) c[1 + k] = (int)((i1 >> (8 * k)) & 0xFF) * 3 + (int)((f1 >> (8 * k)) & 0xFF);
                c[5] = (int)(i2 & 0xFF) * 3 + (int)(f2 & 0xFF);
                if (jg == 0) c[0] = c[1];
#pragma unroll
                for (int k = 0; k < 4; k++)  // right edge: column j + 1 past dwc - 1 repeats column j
                  if (jg + k + 1 > dwc - 1) c[2 + k] = c[1 + k];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                  ue[k] = (c[1 + k] * 3 + c[k] + 8) >> 4;
                  uo[k] = (c[1 + k] * 3 + c[2 + k] + 7) >> 4;
                }
              }
            };
            up(oBi, oBf, ube, ubo);
            up(oRi, oRf, ure, uro);
#pragma unroll
            for (int k = 0; k < 4; k++) {
              const uint32_t yw = k < 2 ? y0 : y1;
              const int ye = (int)((yw >> (16 * (k & 1))) & 0xFF), yo = (int)((yw >> (16 * (k & 1) + 8)) & 0xFF);
              int r0, g0, b0, r1, g1, b1;
              ycc_raw(ye, ube[k], ure[k], r0, g0, b0);
              ycc_raw(yo, ubo[k], uro[k], r1, g1, b1);
              const int sh = 16 * (k & 1);
              wr[k >> 1] |= (uint32_t)(r0 | (r1 << 8)) << sh;
              wg[k >> 1] |= (uint32_t)(g0 | (g1 << 8)) << sh;
              wb[k >> 1] |= (uint32_t)(b0 | (b1 << 8)) << sh;
            }
          } else {
            // 4:2:2 (jdsample.c h2v1_fancy_upsample): the chroma row's columns jg - 1 .. jg + 4, per
            // output pixel (3 * own + neighbour + 1 or 2) >> 2; interior items two columns per op
            int ube[4], ubo[4], ure[4], uro[4];
            auto up = [&](int oi, int* ue, int* uo) {
              const uint32_t* wi = reinterpret_cast<const uint32_t*>(sb + oi + jg);  // (a multiple of 4, as for 4:2:0)
              const uint32_t i0 = wi[-1], i1 = wi[0], i2 = wi[1];
              if (jg > 0 && jg + 4 <= dwc - 1) {
                constexpr uint32_t M = 0x00FF00FFu;
                const uint32_t E = i1 & M, O = (i1 >> 8) & M;  // columns [jg, jg+2], [jg+1, jg+3]
                const uint32_t l = i0 >> 24, rr = i2 & 0xFF;    // jg - 1, jg + 4
                const uint32_t A = E * 3 + (l | (O << 16)) + 0x00010001u;
                const uint32_t B = E * 3 + O + 0x00020002u;
                const uint32_t C = O * 3 + E + 0x00010001u;
                const uint32_t D = O * 3 + ((E >> 16) | (rr << 16)) + 0x00020002u;
                ue[0] = (int)((A >> 2) & 0x3FFF);
                ue[1] = (int)((C >> 2) & 0x3FFF);
                ue[2] = (int)(A >> 18);
                ue[3] = (int)(C >> 18);
                uo[0] = (int)((B >> 2) & 0x3FFF);
                uo[1] = (int)((D >> 2) & 0x3FFF);
                uo[2] = (int)(B >> 18);
                uo[3] = (int)(D >> 18);
              } else {
                int c[6];
                c[0] = (int)(i0 >> 24);
#pragma unroll
                for (int k = 0; k < 4; k++) c[1 + k] = (int)((i1 >> (8 * k)) & 0xFF);
                c[5] = (int)(i2 & 0xFF);
                if (jg == 0) c[0] = c[1];
#pragma unroll
                for (int k = 0; k < 4; k++)  // right edge: column j + 1 past dwc - 1 repeats column j
                  if (jg + k + 1 > dwc - 1) c[2 + k] = c[1 + k];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                  ue[k] = (c[1 + k] * 3 + c[k] + 1) >> 2;
                  uo[k] = (c[1 + k] * 3 + c[2 + k] + 2) >> 2;
                }
              }
            };
            up(oBi, ube, ubo);
            up(oRi, ure, uro);
#pragma unroll
            for (int k = 0; k < 4; k++) {
              const uint32_t yw = k < 2 ? y0 : y1;
              const int ye = (int)((yw >> (16 * (k & 1))) & 0xFF), yo = (int)((yw >> (16 * (k & 1) + 8)) & 0xFF);
              int r0, g0, b0, r1, g1, b1;
              ycc_raw(ye, ube[k], ure[k], r0, g0, b0);
              ycc_raw(yo, ubo[k], uro[k], r1, g1, b1);
              const int sh = 16 * (k & 1);
              wr[k >> 1] |= (uint32_t)(r0 | (r1 << 8)) << sh;
              wg[k >> 1] |= (uint32_t)(g0 | (g1 << 8)) << sh;
              wb[k >> 1] |= (uint32_t)(b0 | (b1 << 8)) << sh;
            }
          }
          // one 8-byte store per channel (x - xb and G::kRgbW are multiples of 8)
          static_assert(G::kRgbW % 8 == 0, "8-byte aligned RGB rows");
          uint2* o = reinterpret_cast<uint2*>(&L.rgb[q][0][x - xb]);
          o[0] = make_uint2(wr[0], wr[1]);
          o[G::kRgbW / 8] = make_uint2(wg[0], wg[1]);
          o[G::kRgbW / 4] = make_uint2(wb[0], wb[1]);
        }
        __syncthreads();
        if (kGlds && more) issue_lds(nxt);
      }
      if (active) {
#pragma unroll
        for (int q = 0; q < kFRows; q++) {
          if (q >= nr) break;
          // H. KT taps of step row q -> ring slot.  Each channel's window comes in as aligned dwords
          // (unaligned sub-dword LDS reads are slow) and is realigned with v_alignbyte.
          const int r = ra + q;
          if (LAY == kRsGray) {
            ring[(r & rmask) * rstride] = (uint32_t)htaps<KT>(hw + q * G::kYDW, hsh, cf);
          } else {
            const int s0 = htaps<KT>(hw + q * 3 * (G::kRgbW / 4), hsh, cf);
            const int s1 = htaps<KT>(hw + (q * 3 + 1) * (G::kRgbW / 4), hsh, cf);
            const int s2 = htaps<KT>(hw + (q * 3 + 2) * (G::kRgbW / 4), hsh, cf);
            ring[(r & rmask) * rstride] = pack3(s0, s1, s2);
          }
          // V. output rows whose window ends at row r
          while (nvend <= r + 1) {
            const int vmin = nvmin, vcnt = nvend - nvmin;
            // (the output row through readfirstlane: its weights and store bases stay scalar, not 64-bit
            // pointers the vector unit re-derives for every row)
            const int nbu = __builtin_amdgcn_readfirstlane(nb);
            const int32_t* wk = L.vw[nbu - oy0];
            int32_t v0 = 1 << 21, v1 = 1 << 21, v2 = 1 << 21;
            if constexpr (kRing8) {
              // all taps unrolled (KT of them, or 8 when ksv > KT): their ring and weight reads issue
              // together (the weights past the window are zero, k_coeffs / the strip table; ring rows
              // past it are finite values)
              if (ksv <= KT) vtaps8_at<KT, LAY == kRsGray>(vmin & 7, L.ring, t, wk, v0, v1, v2);
              else vtaps8_at<8, LAY == kRsGray>(vmin & 7, L.ring, t, wk, v0, v1, v2);
            } else {
              auto vtap = [&](int k) {
                const uint32_t h = ring[((vmin + k) & rmask) * rstride];
                const int32_t w = wk[k];
                if (LAY == kRsGray) {
                  v0 += tap((int32_t)h, w);
                } else {
                  v0 += tap((int32_t)(h & 0xFF), w);
                  v1 += tap((int32_t)((h >> 8) & 0xFF), w);
                  v2 += tap((int32_t)(h >> 16), w);
                }
              };
              if (ksv <= KT) {
#pragma unroll
                for (int k = 0; k < KT; k++) vtap(k);
              } else {
                for (int k = 0; k < vcnt; k++) vtap(k);
              }
            }
            if (LAY == kRsGray) {
              const int c = rs_clip8(v0);
              put3_row(out, om, lut, (int64_t)nbu * ow, ox, c, c, c);
            } else {
              put3_row(out, om, lut, (int64_t)nbu * ow, ox, rs_clip8(v0), rs_clip8(v1), rs_clip8(v2));
            }
            nb++;
            if (nb < oy1) window(nb, nvmin, nvend);
            else nvend = 1 << 30;
          }
        }
      }
      if (LAY == kRsGray) __syncthreads();  // the H pass read the staged rows themselves
      if (more) {
        commit(nxt);
        cur = nxt;
      }
      __syncthreads();  // next step's rows staged; this step's H reads are done
    }
    __syncthreads();  // LDS reuse by the next tile
  }
}

template <int LAY>
static void launch_lay(int64_t full, uint64_t hint, int n, const ImgDesc* descs, const sdsj_op& op, int strip_h, int strips,
                       int ntz,
                       const uint8_t* scratch, const uint8_t* flip, void* out, const int32_t* routes, int cap,
                       const float* lut, hipStream_t s, uint64_t rm) {
  if (route_on(rm, rs_route(LAY, 3)))
    hipLaunchKernelGGL((k_rs420<3, LAY>), dim3(route_grid(hint, rs_route(LAY, 3), full)), dim3(kFThreads), 0, s, n, descs, op, strip_h, strips, ntz, scratch, flip, out, routes, cap, lut);
  if (route_on(rm, rs_route(LAY, 5)))
    hipLaunchKernelGGL((k_rs420<5, LAY>), dim3(route_grid(hint, rs_route(LAY, 5), full)), dim3(kFThreads), 0, s, n, descs, op, strip_h, strips, ntz, scratch, flip, out, routes, cap, lut);
  if (route_on(rm, rs_route(LAY, 7)))
    hipLaunchKernelGGL((k_rs420<7, LAY>), dim3(route_grid(hint, rs_route(LAY, 7), full)), dim3(kFThreads), 0, s, n, descs, op, strip_h, strips, ntz, scratch, flip, out, routes, cap, lut);
  if (route_on(rm, rs_route(LAY, 9)))
    hipLaunchKernelGGL((k_rs420<9, LAY>), dim3(route_grid(hint, rs_route(LAY, 9), full)), dim3(kFThreads), 0, s, n, descs, op, strip_h, strips, ntz, scratch, flip, out, routes, cap, lut);
  if (route_on(rm, rs_route(LAY, 11)))
    hipLaunchKernelGGL((k_rs420<11, LAY>), dim3(route_grid(hint, rs_route(LAY, 11), full)), dim3(kFThreads), 0, s, n, descs, op, strip_h, strips, ntz, scratch, flip, out, routes, cap, lut);
}

hipError_t launch_resample420(int n, const ImgDesc* descs, const sdsj_op& op, int strip_h, const uint8_t* scratch,
                              const uint8_t* flip, void* out, const int32_t* routes, int cap, const float* lut,
                              hipStream_t s, uint64_t rm, uint64_t hint) {
  const int tiles = (op.out_w + kFThreads - 1) / kFThreads;
  const int strips = (op.out_h + strip_h - 1) / strip_h;
  const int64_t full = (int64_t)(n < kRsfEntries ? n : kRsfEntries) * strips * tiles;
  launch_lay<kRs420>(full, hint, n, descs, op, strip_h, strips, tiles, scratch, flip, out, routes, cap, lut, s, rm);
  launch_lay<kRs422>(full, hint, n, descs, op, strip_h, strips, tiles, scratch, flip, out, routes, cap, lut, s, rm);
  launch_lay<kRs444>(full, hint, n, descs, op, strip_h, strips, tiles, scratch, flip, out, routes, cap, lut, s, rm);
  launch_lay<kRsGray>(full, hint, n, descs, op, strip_h, strips, tiles, scratch, flip, out, routes, cap, lut, s, rm);
  return hipGetLastError();
}

}  // namespace sdsj
