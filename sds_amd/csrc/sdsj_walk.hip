// sdsj_walk.hip -- k_walk: dequantisation + jpeg_idct_islow straight from the entropy decoder's
// symbol records (baseline images; progressive images keep the dense k_idct).
//
// The entropy stage (sdsj_entropy.hip) leaves, per subsequence, the fix pass's records of its first
// true blocks and the speculative pass's records of the rest (SubState fix_n / nblk_f / spec_m);
// both are decode-ordered streams of int32 SymRec (k = zigzag index, k = 0 opens a block, the DC
// record carries the running DC sum since the stream's entry).  One wave walks one subsequence:
//   1. 128 records per step (two coalesced dword loads per lane), block starts found by ballot;
//   2. up to 8 complete blocks per step: lane q looks up block q's position (decode-order index
//      g -> MCU, component, block row/column), whether the crop reads it (the needed rectangle of
//      each component, one sample of fancy-upsampling context around the source window) and whether
//      libjpeg leaves it zero (jdhuff.c insufficient_data: SegView vend / kSegEmpty after kSegIns);
//   3. every record lane scatters its dequantised coefficient into its block's LDS buffer (natural
//      order; the DC value is the stream's DC base + the record's running sum, as int16 like
//      libjpeg's JCOEF store); indices past 63 (corrupt runs) land on 63, as jpeg_natural_order's
//      guard entries make them;
//   4. 8 lanes per block run the two ISLOW passes (columns, then rows) and store 8 bytes per row
//      into the component plane.
// Blocks past the data (g >= vend of their interval) were never decoded: the workgroup 0 of each
// image writes them as IDCT(0) = 128.  Per image the records are read once and the planes written
// once; nothing dense passes between the entropy decoder and this kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sdsj_common.h"
#include "sdsj_idct.h"
#include "sdsj_kernels.h"

#pragma clang fp contract(off)

namespace sdsj {

constexpr int kWalkThreads = 256;
constexpr int kWalkWaves = kWalkThreads / 64;
constexpr int kWalkGrid = 8;  // workgroups per image (each wave strides over the subsequences)
constexpr int kWalkWs = 72;   // ints per LDS block buffer (conflict-free column reads)
constexpr uint32_t kNoRec = 0x7Fu << 16;  // past the stream: k = 127, never a block start

struct LdsWalk {
  int32_t qt[kMaxComp][64];  // quantisation table of each component, natural order
  uint8_t nat[80];           // jpeg_natural_order + 16 guard entries
  int32_t bcomp[kMaxBlocksPerMcu], bdx[kMaxBlocksPerMcu], bdy[kMaxBlocksPerMcu];
  int32_t ch[kMaxComp], cv[kMaxComp], pitch[kMaxComp];
  int32_t bxlo[kMaxComp], bxhi[kMaxComp], bylo[kMaxComp], byhi[kMaxComp];  // blocks the crop reads
  int64_t plane[kMaxComp];
  alignas(16) int32_t W[kWalkWaves][8][kWalkWs];  // per wave: 8 block buffers (dequantised, natural order)
  int32_t binfo[kWalkWaves][8][4];  // per wave, block q: flags | component, block column, block row, DC base
};
constexpr int kBiValid = 1 << 4, kBiZero = 1 << 5;

// a / b for 0 <= a < 2^24, 1 <= b <= 2^16: float estimate, then one correction each way (exact)
__device__ __forceinline__ int wdiv(int a, int b) {
  int q = (int)((float)a / (float)b);
  q -= q * b > a ? 1 : 0;
  q += (q + 1) * b <= a ? 1 : 0;
  return q;
}

// Walks one record stream of a subsequence: skips its first `skip` blocks, then transforms `nuse`
// blocks whose decode-order indices are g0 + kstart, ...  base: the DC predictors at the stream's
// entry.  Wave-uniform control flow; lanes own records, then blocks.
__device__ void walk_stream(LdsWalk& L, const ImgDesc* d, const int32_t* vend, const int32_t* sflag, uint8_t* planes,
                            const uint32_t* recs, int nrec, int skip, int nuse, int64_t gfirst, int64_t gend, int bps,
                            int b0, int b1, int b2) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int bpm = d->bpm, mcux = d->mcux, nseg = d->nseg;
  int pos = 0;
  int64_t g = gfirst;  // decode-order index of the next block to transform
  int (*W)[kWalkWs] = L.W[wv];
  int (*BI)[4] = L.binfo[wv];
  while ((nuse > 0 || skip > 0) && pos < nrec) {
    const uint32_t r0 = pos + lane < nrec ? recs[pos + lane] : kNoRec;
    const uint32_t r1 = pos + 64 + lane < nrec ? recs[pos + 64 + lane] : kNoRec;
    const int k0 = (int)(r0 >> 16) & 0x7F, k1 = (int)(r1 >> 16) & 0x7F;
    const uint64_t s0 = __builtin_amdgcn_ballot_w64(k0 == 0), s1 = __builtin_amdgcn_ballot_w64(k1 == 0);
    const int n0 = __popcll(s0), nst = n0 + __popcll(s1);
    // blocks complete in this window: all but the last start, and that one too if the stream ends
    // inside (a block has at most 64 records, so the block at pos always ends inside)
    const int ncomp = nst - 1 + (pos + 128 >= nrec ? 1 : 0);
    if (nst == 0 || ncomp <= 0) break;  // (malformed stream: cannot happen for records the decoder wrote)
    // exclusive block-start counts of this lane's two records
    const int e0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(s0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)s0, 0));
    const int e1 = n0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(s1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)s1, 0));
    // record index of the m-th block start of the window (m < nst), or the stream end
    auto start_of = [&](int m) {
      if (m >= nst) return nrec;
      const uint64_t a = __builtin_amdgcn_ballot_w64(k0 == 0 && e0 == m);
      if (a) return pos + (int)__builtin_ctzll(a);
      const uint64_t b = __builtin_amdgcn_ballot_w64(k1 == 0 && e1 == m);
      return pos + 64 + (int)__builtin_ctzll(b);
    };
    if (skip > 0) {
      const int m = skip < ncomp ? skip : ncomp;
      pos = start_of(m);
      skip -= m;
      continue;
    }
    const int nb = ncomp < 8 ? (ncomp < nuse ? ncomp : nuse) : (nuse < 8 ? nuse : 8);
    // 2. block q (lane q): position, crop, zero rule
    if (lane < nb) {
      const int64_t gq = g + lane;
      int flags = 0, bx = 0, by = 0, base = 0;
      if (gq < gend) {
        const int gi = (int)gq;
        const int mcu = wdiv(gi, bpm), b = gi - mcu * bpm;
        const int c = L.bcomp[b];
        const int my = wdiv(mcu, mcux), mx = mcu - my * mcux;
        bx = mx * L.ch[c] + L.bdx[b];
        by = my * L.cv[c] + L.bdy[b];
        const bool need = bx >= L.bxlo[c] && bx <= L.bxhi[c] && by >= L.bylo[c] && by <= L.byhi[c];
        int k = 0;
        if (nseg > 1) k = wdiv(gi, bps);
        const bool zero = gi >= vend[k] || (k > 0 && (sflag[k] & kSegEmpty) && (sflag[k - 1] & kSegIns));
        flags = c | (need ? kBiValid : 0) | (zero ? kBiZero : 0);
        base = c == 0 ? b0 : (c == 1 ? b1 : b2);
      }
      BI[lane][0] = flags;
      BI[lane][1] = bx;
      BI[lane][2] = by;
      BI[lane][3] = base;
    }
    for (int i = lane; i < nb * 16; i += 64)  // zero the nb block buffers (16 x 4 ints each)
      *reinterpret_cast<int4*>(&W[i >> 4][(i & 15) * 4]) = make_int4(0, 0, 0, 0);
    wave_lds_sync();
    // 3. scatter the records of blocks [0, nb) into their buffers.  Positions within a block are
    // distinct: zigzag indices increase, and an index past 63 (corrupt run, clamped to 63 by the guard
    // entries) ends its block (decode_mcu's k loop), so nothing else of the block lands on 63 after it.
    const int bid0 = e0 + (k0 == 0 ? 1 : 0) - 1, bid1 = e1 + (k1 == 0 ? 1 : 0) - 1;
    auto scatter = [&](uint32_t r, int k, int bid) {
      const int f = BI[bid][0];
      if ((f & (kBiValid | kBiZero)) != kBiValid) return;
      const int c = f & 3, nk = L.nat[k];
      int v = (int)(int16_t)(r & 0xFFFF);
      if (k == 0) v = (int)(int16_t)(v + BI[bid][3]);
      W[bid][nk] = v * L.qt[c][nk];
    };
    if (bid0 < nb && k0 != 127) scatter(r0, k0, bid0);
    if (bid1 < nb && k1 != 127) scatter(r1, k1, bid1);
    wave_lds_sync();
    // 4. ISLOW: 8 lanes per block (lane r: column r, then row r)
    const int q = lane >> 3, r = lane & 7;
    const int f = q < nb ? BI[q][0] : 0;
    const bool act = (f & kBiValid) != 0;
    int col[8];
    if (act) {
      int x[8];
      for (int k = 0; k < 8; k++) x[k] = W[q][k * 8 + r];
      if ((x[1] | x[2] | x[3] | x[4] | x[5] | x[6] | x[7]) == 0) {
        for (int k = 0; k < 8; k++) col[k] = x[0] * 4;  // << PASS1_BITS
      } else {
        int o[8];
        islow_1d(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], o);
        for (int k = 0; k < 8; k++) col[k] = (o[k] + (1 << 10)) >> 11;  // DESCALE(, CONST_BITS-PASS1_BITS)
      }
    }
    wave_lds_sync();
    if (act)
      for (int k = 0; k < 8; k++) W[q][k * 8 + r] = col[k];
    wave_lds_sync();
    if (act) {
      const int* w = W[q] + r * 8;
      int o[8];
      islow_1d(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], o);
      uint32_t lo = 0, hi = 0;
      for (int k = 0; k < 4; k++) lo |= range_limit((o[k] + (1 << 17)) >> 18) << (8 * k);
      for (int k = 0; k < 4; k++) hi |= range_limit((o[k + 4] + (1 << 17)) >> 18) << (8 * k);
      const int c = f & 3;
      *reinterpret_cast<uint2*>(planes + L.plane[c] + (int64_t)(BI[q][2] * 8 + r) * L.pitch[c] + BI[q][1] * 8) =
          make_uint2(lo, hi);
    }
    wave_lds_sync();
    pos = start_of(nb);
    nuse -= nb;
    g += nb;
  }
}

__global__ void __launch_bounds__(kWalkThreads) k_walk(int n, const ImgDesc* __restrict__ descs,
                                                       const ImgTables* __restrict__ tables,
                                                       uint8_t* __restrict__ scratch) {
  const int img = blockIdx.y;
  if (img >= n) return;
  const ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK || d->geo == kGeoZeros || d->progressive) return;
  __shared__ LdsWalk L;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int ncomp = d->ncomp;
  for (int i = t; i < ncomp * 64; i += kWalkThreads) L.qt[i / 64][i % 64] = tables[img].qt[d->comp[i / 64].tq][i % 64];
  for (int i = t; i < 80; i += kWalkThreads) L.nat[i] = (uint8_t)natural_order(i);
  if (t < d->bpm) {
    L.bcomp[t] = d->blk_comp[t];
    L.bdx[t] = d->blk_dx[t];
    L.bdy[t] = d->blk_dy[t];
  }
  if (t < ncomp) {
    // the blocks whose samples the colour / resample passes read: the source rectangle
    // [src_x0, src_x0 + src_w) x [src_y0, src_y1) in this component's sampling, widened by one sample
    // for the fancy upsampling's neighbours
    const CompDesc& cd = d->comp[t];
    const int x0 = d->src_x0, x1 = d->src_x0 + d->src_w, y0 = d->src_y0, y1 = d->src_y1;
    const int rh = ncomp == 1 ? 1 : d->hmax / cd.h, rv = ncomp == 1 ? 1 : d->vmax / cd.v;
    int cx0 = x0 / rh - 1, cx1 = (x1 - 1) / rh + 1, cy0 = y0 / rv - 1, cy1 = (y1 - 1) / rv + 1;
    cx0 = cx0 < 0 ? 0 : cx0;
    cy0 = cy0 < 0 ? 0 : cy0;
    cx1 = cx1 > cd.bw * 8 - 1 ? cd.bw * 8 - 1 : cx1;
    cy1 = cy1 > cd.bh * 8 - 1 ? cd.bh * 8 - 1 : cy1;
    const bool any = x1 > x0 && y1 > y0;
    L.bxlo[t] = cx0 >> 3;
    L.bxhi[t] = any ? cx1 >> 3 : -1;
    L.bylo[t] = cy0 >> 3;
    L.byhi[t] = any ? cy1 >> 3 : -1;
    L.ch[t] = ncomp == 1 ? 1 : cd.h;
    L.cv[t] = ncomp == 1 ? 1 : cd.v;
    L.pitch[t] = cd.pitch;
    L.plane[t] = cd.plane_off;
  }
  __syncthreads();
  uint8_t* planes = scratch + d->off_planes;
  const SegView sv = seg_view(scratch + d->off_seg, d->nseg);
  const SubState* sub = reinterpret_cast<const SubState*>(scratch + d->off_sub);
  const uint32_t* srec = reinterpret_cast<const uint32_t*>(scratch + d->off_srec);
  const uint32_t* frec = reinterpret_cast<const uint32_t*>(scratch + d->off_frec);
  const int nsub = d->nsub, rec_cap = d->rec_cap, bpm = d->bpm;
  const int bps = d->restart_interval ? d->restart_interval * bpm : (int)d->total_blocks;
  const int64_t total = d->total_blocks;
  for (int j = blockIdx.x * kWalkWaves + wv; j < nsub; j += gridDim.x * kWalkWaves) {
    const SubState& S = sub[j];
    const int fix_n = __builtin_amdgcn_readfirstlane(S.fix_n);
    const int seg = __builtin_amdgcn_readfirstlane(S.seg);
    const int nblk_ex = __builtin_amdgcn_readfirstlane(S.nblk_ex);
    const int64_t g0 = (int64_t)seg * bps + nblk_ex;
    const int64_t gend = (int64_t)(seg + 1) * bps < total ? (int64_t)(seg + 1) * bps : total;
    const int dc0 = __builtin_amdgcn_readfirstlane(S.dc_ex[0]), dc1 = __builtin_amdgcn_readfirstlane(S.dc_ex[1]),
              dc2 = __builtin_amdgcn_readfirstlane(S.dc_ex[2]);
    const int F = fix_n != 0 ? __builtin_amdgcn_readfirstlane(S.nblk_f) : 0;
    if (F > 0)
      walk_stream(L, d, sv.vend, sv.flag, planes, frec + fix_stream(j, seg, rec_cap, bpm),
                  __builtin_amdgcn_readfirstlane(S.nrec_f),
                  0, F, g0, gend, bps, dc0, dc1, dc2);
    if (fix_n >= 0) {
      const int nuse = __builtin_amdgcn_readfirstlane(S.cur_nblk) - F;
      if (nuse > 0)
        walk_stream(L, d, sv.vend, sv.flag, planes, srec + (int64_t)j * rec_cap,
                    __builtin_amdgcn_readfirstlane(S.nrec_s),
                    __builtin_amdgcn_readfirstlane(S.spec_m), nuse, g0 + F, gend, bps,
                    dc0 + __builtin_amdgcn_readfirstlane(S.dc_adj[0]), dc1 + __builtin_amdgcn_readfirstlane(S.dc_adj[1]),
                    dc2 + __builtin_amdgcn_readfirstlane(S.dc_adj[2]));
    }
  }
  // blocks past the data of their interval (damaged streams): never decoded, IDCT(0) = 128
  if (blockIdx.x == 0) {
    const int q = lane >> 3, r = lane & 7;
    for (int s = 0; s < d->nseg; s++) {
      const int64_t lo = sv.vend[s];
      const int64_t hi = (int64_t)(s + 1) * bps < total ? (int64_t)(s + 1) * bps : total;
      for (int64_t gb = lo + wv * 8; gb < hi; gb += kWalkWaves * 8) {
        const int64_t gq = gb + q;
        if (gq >= hi) continue;
        const int gi = (int)gq;
        const int mcu = wdiv(gi, bpm), b = gi - mcu * bpm;
        const int c = L.bcomp[b];
        const int my = wdiv(mcu, d->mcux), mx = mcu - my * d->mcux;
        const int bx = mx * L.ch[c] + L.bdx[b], by = my * L.cv[c] + L.bdy[b];
        if (bx >= L.bxlo[c] && bx <= L.bxhi[c] && by >= L.bylo[c] && by <= L.byhi[c])
          *reinterpret_cast<uint2*>(planes + L.plane[c] + (int64_t)(by * 8 + r) * L.pitch[c] + bx * 8) =
              make_uint2(0x80808080u, 0x80808080u);
      }
    }
  }
}

hipError_t launch_walk(int n, const ImgDesc* descs, const ImgTables* tables, uint8_t* scratch, hipStream_t s) {
  hipLaunchKernelGGL(k_walk, dim3(kWalkGrid, n), dim3(kWalkThreads), 0, s, n, descs, tables, scratch);
  return hipGetLastError();
}

}  // namespace sdsj
