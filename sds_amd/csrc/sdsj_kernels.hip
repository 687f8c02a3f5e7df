// sdsj_kernels.hip -- gfx950 (MI355X) kernels of the batched JPEG decode + crop/resize path.
//
// Stage map (reference behaviour each kernel reproduces, see DESIGN.md for the layout/rooflines):
//   k_parse    markers, tables, geometry          jdmarker.c / jdhuff.c tables / functional.py:118-140
//   k_plan     per-batch scratch offsets          (no reference counterpart)
//   k_unstuff  byte unstuffing + RSTn split        jdhuff.c jpeg_fill_bit_buffer / process_restart
//   k_entsync  speculative decode + self-sync     jdhuff.c decode_mcu (parallel restatement), in
//   k_entwrite verified decode -> coefficients    sdsj_entropy.hip
//   k_idct     dequant + ISLOW IDCT                jidctint.c jpeg_idct_islow
//   k_color    fancy upsampling + YCbCr->RGB      jdsample.c / jdmainct.c / jdcolor.c
//   k_coeffs   resampling tables (doubles)        Pillow Resample.c precompute_coeffs
//   k_hpass    horizontal pass, uint8 out         Pillow ImagingResampleHorizontal_8bpc
//   k_vpass    vertical pass + hflip + layout/LUT Pillow ImagingResampleVertical_8bpc,
//                                                 functional.py:102-110, presets.py:154-162
//   (k_color / k_hpass / k_vpass only run for images with fused = 0; the others, and every
//    failed sample, go through k_resample in sdsj_resample.hip)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sdsj_common.h"
#include "sdsj_kernels.h"
#include "sdsj_idct.h"

#pragma clang fp contract(off)

namespace sdsj {

// ------------------------------------------------------------------------------------------
// k_parse: one wave per image.  The first kHdrStage bytes are staged into LDS (coalesced); lane 0
// walks the markers; all lanes build the derived Huffman tables.
// ------------------------------------------------------------------------------------------
constexpr int kHdrStage = 4096;

struct DevReader {
  const uint8_t* lds;
  int64_t nlds;
  const uint8_t* g;
  __device__ int operator()(int64_t i) const { return i < nlds ? lds[i] : g[i]; }
};

// Pillow precompute_coeffs bounds for output index xx (doubles, same operation order).
__device__ __host__ inline void resample_bounds(int in_size, int out_size, double support_base, int xx,
                                                int* xmin_out, int* xmax_out) {
  double scale = (double)in_size / out_size;
  double filterscale = scale < 1.0 ? 1.0 : scale;
  double support = support_base * filterscale;
  double center = 0.0 + (xx + 0.5) * scale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  *xmin_out = xmin;
  *xmax_out = xmax - xmin;
}

// frames = true: raw RGB frames (sdsj_resize_frames_device): the unfused passes read the frame rows
// in place (off_rgb / rgb_pitch are set by the caller), no entropy / plane / RGB-row scratch.
__device__ __host__ inline int warm_for(int sub_bits, int floor_bits) {
  const int w = sub_bits / kWarmDiv > floor_bits ? sub_bits / kWarmDiv : floor_bits;
  return sub_bits * 3 / 2 < w ? sub_bits * 3 / 2 : w;
}

// Distinct Huffman table slots the scan uses (DC keys td, AC keys 4 | ta), counted as load_tables
// counts them: more than 4 selects the 10-bit entropy route (kRtEnt10, image_routes).
__device__ __host__ inline int huff_slots(const ImgDesc& d) {
  int keys[2 * kMaxComp], ns = 0;
  for (int c = 0; c < d.ncomp; c++)
    for (int k = 0; k < 2; k++) {
      const int key = k ? (4 | d.comp[c].ta) : d.comp[c].td;
      bool seen = false;
      for (int q = 0; q < ns; q++) seen |= keys[q] == key;
      if (!seen) keys[ns++] = key;
    }
  return ns;
}

__device__ __host__ inline int64_t plan_image(ImgDesc* d, const sdsj_op& op, bool frames = false, bool small = false) {
  // Geometry: functional.py:78-80 shortcut, :118-147 crop, Pillow ImagingResampleInner.
  const int W = d->width, H = d->height;
  if (W == op.out_w && H == op.out_h) {
    d->geo = kGeoIdentity;
    d->cx0 = d->cy0 = 0;
    d->cw = W;
    d->ch = H;
  } else {
    d->geo = kGeoResize;
    if (op.crop_before_resize) {
      crop_box(W, H, op.out_h, op.out_w, &d->cx0, &d->cy0, &d->cw, &d->ch);
    } else {
      d->cx0 = d->cy0 = 0;
      d->cw = W;
      d->ch = H;
    }
    if (d->cw <= 0 || d->ch <= 0) d->geo = kGeoZeros;
  }
  d->need_h = d->geo == kGeoResize && d->cw != op.out_w;
  d->need_v = d->geo == kGeoResize && d->ch != op.out_h;
  // NEAREST (Pillow ImagingScaleAffine) runs as a one-tap resample through the unfused passes: tap
  // weight 1 << 22 at the source index nearest_src picks, none where it is outside (fill value 0)
  const bool nearest = op.filter == SDSJ_FILTER_NEAREST;
  double sup = filter_support(op.filter);
  d->ksh = d->need_h ? (nearest ? 1 : resample_ksize(d->cw, op.out_w, sup)) : 0;
  d->ksv = d->need_v ? (nearest ? 1 : resample_ksize(d->ch, op.out_h, sup)) : 0;
  if (d->geo == kGeoZeros) {
    d->yf = d->yl = 0;
  } else if (d->need_v && nearest) {
    const int a = nearest_src(d->ch, op.out_h, 0), b = nearest_src(d->ch, op.out_h, op.out_h - 1);
    d->yf = a < 0 || b < 0 ? 0 : a;
    d->yl = a < 0 || b < 0 ? d->ch : b + 1;
  } else if (d->need_v) {
    int a0, a1, b0, b1;
    resample_bounds(d->ch, op.out_h, sup, 0, &a0, &a1);
    resample_bounds(d->ch, op.out_h, sup, op.out_h - 1, &b0, &b1);
    d->yf = a0;
    d->yl = b0 + b1;
  } else {
    d->yf = 0;
    d->yl = d->ch;
  }
  d->src_y0 = d->cy0 + d->yf;
  d->src_y1 = d->cy0 + d->yl;
  d->src_x0 = d->cx0;
  d->src_w = d->geo == kGeoZeros ? 0 : d->cw;
  // fused resample tiles: halve the tile width until a tile's source columns fit kMaxSpan
  // (bound: (tw - 1) * scale + 2 * support + 2 columns, Pillow precompute_coeffs windows)
  d->fused = 0;
  d->tile_w = 0;
  double span = 0.0;  // the tile's source-column bound
  d->ring_rows = 1;
  while (d->ring_rows < d->ksv) d->ring_rows *= 2;  // vertical window rows kept per column
  if (d->geo != kGeoZeros && d->ring_rows <= kRingMaxRows && !nearest) {
    const double scale = d->need_h ? (double)d->cw / op.out_w : 1.0;
    const double supp = d->need_h ? sup * (scale < 1.0 ? 1.0 : scale) : 0.0;
    int tw = op.out_w < 256 ? op.out_w : 256;
    if (tw > kRingDW / d->ring_rows) tw = kRingDW / d->ring_rows;
    const int lim = d->ksh <= 7 ? rs_span(d->ksh) : kMaxSpan;  // (the KT <= 7 fused kernels' rows)
    for (;;) {
      span = (double)tw * scale + 2.0 * supp + 4.0;
      if (span <= (double)lim) {
        d->fused = 1;
        d->tile_w = tw;
        break;
      }
      if (tw == 1) break;
      tw = (tw + 1) / 2;
    }
  }
  if (frames) d->fused = 0;
  // specialised fused kernels (sdsj_resample420.hip): 4:2:0 (h2v2 fancy chroma), 4:2:2 (h2v1 fancy
  // chroma), 4:4:4 and grayscale, horizontal and vertical passes, odd tap counts 3..11; everything
  // else takes the generic k_resample
  d->rs_fast = 0;
  d->rs_lay = kRs420;
  if (d->fused && d->need_h && d->need_v && d->ksh >= 3 && d->ksh <= 11 && (d->ksh & 1) &&
      d->ring_rows <= rs_ring_rows(d->ksh) && d->ksv <= rs_vtaps(d->ksh) && d->tile_w * d->ring_rows <= rs_ring_dw(d->ksh) &&
      span <= (double)rs_span(d->ksh) && d->comp[0].rh == 1 && d->comp[0].rv == 1) {
    const CompDesc &c1 = d->comp[1], &c2 = d->comp[2];
    const bool same = d->ncomp == 3 && c2.rh == c1.rh && c2.rv == c1.rv && c2.dw == c1.dw && c2.dh == c1.dh;
    int lay = -1;
    if (d->ncomp == 1) lay = kRsGray;
    else if (same && c1.rh == 1 && c1.rv == 1) lay = kRs444;
    else if (same && c1.rh == 2 && c1.rv == 1 && c1.dw > 2) lay = kRs422;
    else if (same && c1.rh == 2 && c1.rv == 2 && c1.dw > 2) lay = kRs420;
    if (lay >= 0) {
      d->rs_fast = d->ksh;
      d->rs_lay = lay;
    }
  }
  d->lat = small && !frames;
  // multi-hypothesis speculative pass for latency-mode baseline images without restart intervals;
  // only the 11-bit entropy routes launch it (k_entspec_mh), so images of more than 4 table slots
  // (kRtEnt10) keep the ordinary speculative pass
  d->mh = (int8_t)(SDSJ_MH && d->lat && !d->progressive && d->restart_interval == 0 && d->bpm <= kMhMaxPhases &&
                   huff_slots(*d) <= 4);
  {
    const int64_t bits = d->entropy_len * 8;
    const int64_t per_group = (int64_t)kDecodeThreads * (d->lat ? kLatSubBits : kGroupBits);
    int64_t g = (bits + per_group - 1) / per_group;
    g = g < 1 ? 1 : (g > kMaxEntGroups ? kMaxEntGroups : g);
    d->ent_groups = frames ? 1 : (int32_t)g;
    const int64_t lanes = (int64_t)kDecodeThreads * d->ent_groups;
    d->sub_bits = (int32_t)align_up((bits + lanes - 1) / lanes, 32);
  }
  const int min_sub = d->lat ? kLatSubBits : kMinSubBits;
  if (d->sub_bits < min_sub) d->sub_bits = min_sub;
  // warm-up: kWarmBits (k_parse may raise the floor for small lanes), or sub_bits / kWarmDiv for long
  // subsequences (large images: a few percent more speculative work removes nearly every sync task,
  // each of which is a serial re-decode); latency mode: kLatWarm
  d->warm_bits = d->lat ? kLatWarm : warm_for(d->sub_bits, kWarmBits);
  d->nsub_cap = (int32_t)((d->entropy_len * 8 + d->sub_bits - 1) / d->sub_bits) + d->nseg + 1;
  const bool prog = d->progressive && !frames;  // k_prog decodes it: no unstuffed stream, no subsequences
  if (prog) {
    d->ent_groups = 1;
    d->nsub_cap = 1;
  }
  // scratch layout (relative offsets; k_plan adds the image base)
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    int64_t r = o;
    o += align_up(bytes, 256);
    return r;
  };
  d->off_ustream = take(prog ? 32 : d->entropy_len + kUPad + 32);  // + the 16-byte granule of the final pad store
  d->ustream_cap = prog ? 0 : d->entropy_len + kUPad;
  d->off_seg = take(seg_bytes(d->nseg));
  d->ntiles = prog ? 0 : (int32_t)((d->entropy_len + kUsTileBytes - 1) / kUsTileBytes);
  d->off_tiles = take((int64_t)d->ntiles * sizeof(UsTile));
  d->off_sub = take((int64_t)d->nsub_cap * sizeof(SubState));
  d->off_rec = take((int64_t)d->nsub_cap * kRec * sizeof(SyncRec));
  d->off_ptab = take(prog ? (int64_t)sizeof(ProgTables) : 0);
  d->off_coef = take(d->total_blocks * 128);
  int64_t planes = 0;
  for (int c = 0; c < d->ncomp; c++) planes += align_up((int64_t)d->comp[c].pitch * d->comp[c].bh * 8, 256);
  d->off_planes = take(planes);
  d->off_rgb = take(d->fused || frames ? 0 : (int64_t)d->src_w * (d->src_y1 - d->src_y0) * 3);
  d->rgb_pitch = d->src_w;  // k_color packs the crop rows
  d->off_tmp = take(!d->fused && d->need_h ? (int64_t)(d->yl - d->yf) * op.out_w * 3 : 0);
  d->off_kh = take(d->need_h ? ((int64_t)2 * op.out_w + (int64_t)op.out_w * d->ksh) * 4 : 0);
  d->off_kv = take(d->need_v ? ((int64_t)2 * op.out_h + (int64_t)op.out_h * d->ksv) * 4 : 0);
  d->need = o;
  return o;
}

// Device sink of the shared parser: lane 0 records the DHT/DQT copies (the last definition of a
// table wins, as with sequential copying); every lane then performs them.
struct ParseJob {
  int32_t kind;  // 0 DHT values, 1 DQT entries (pq = 0), 2 DQT entries (pq = 1)
  int32_t cnt;
  int64_t src;
  void* dst;
};
constexpr int kMaxJobs = 16;

struct DevSink {
  ParseJob* jobs;
  int* njobs;
  const DevReader& rd;
  __device__ void add(int kind, void* dst, int64_t src, int cnt) const {
    for (int q = 0; q < *njobs; q++)
      if (jobs[q].dst == dst) {
        jobs[q] = ParseJob{kind, cnt, src, dst};
        return;
      }
    if (*njobs < kMaxJobs) {
      jobs[(*njobs)++] = ParseJob{kind, cnt, src, dst};
      return;
    }
    // (more distinct tables than kMaxJobs cannot happen: 8 Huffman + 4 quantisation tables)
  }
  __device__ void dht(HuffSpec* h, int64_t src, int cnt) const { add(0, h->vals, src, cnt); }
  __device__ void dqt(uint16_t* qt, int pq, int64_t src) const { add(pq ? 2 : 1, qt, src, 64); }
};

__global__ void __launch_bounds__(64) k_parse(int n, const uint8_t* __restrict__ blob, int64_t blob_bytes,
                                              const int64_t* __restrict__ offsets, const int32_t* __restrict__ lengths,
                                              sdsj_op op, int warm_bits, int small, ImgDesc* __restrict__ descs,
                                              ImgTables* __restrict__ tables) {
  const int img = blockIdx.x;
  if (img >= n) return;
  const int lane = threadIdx.x;
  {  // the sample's range must lie inside the blob (nothing below reads outside it); otherwise EINVAL
    const int64_t o = offsets[img], l = lengths[img];
    if (o < 0 || l < 0 || o > blob_bytes || l > blob_bytes - o) {
      if (lane == 0) descs[img].status = SDSJ_EINVAL;
      return;
    }
  }
  __shared__ alignas(16) uint8_t hdr[kHdrStage];
  __shared__ ImgDesc sd;
  __shared__ ImgTables st;
  __shared__ ParseJob jobs[kMaxJobs];
  __shared__ int njobs, s_status;

  const uint8_t* g = blob + offsets[img];
  const int64_t len = lengths[img];
  const int64_t nstage = len < kHdrStage ? len : kHdrStage;
  for (int64_t i = lane; i < nstage; i += 64) hdr[i] = g[i];
  if (lane == 0) njobs = 0;
  __syncthreads();
  DevReader rd{hdr, nstage, g};
  if (lane == 0) {
    DevSink sink{jobs, &njobs, rd};
    int status = parse_headers(rd, len, &sd, &st, sink);
    if (status == SDSJ_OK) status = setup_geometry(&sd, &st);
    if (status == SDSJ_OK) plan_image(&sd, op, false, small != 0);
    if (warm_bits >= 0) sd.warm_bits = warm_bits;  // override (experiments)
    else if (n < kWarmSmallLane && !sd.lat) sd.warm_bits = warm_for(sd.sub_bits, kWarmBitsSmall);  // small lane
    sd.status = status;
    for (int k = 0; k < 4; k++) sd.t_rs[k] = 0;
    s_status = status;
  }
  __syncthreads();
  // the recorded table copies, all lanes (values beyond a DHT's count are zero, jdmarker.c get_dht)
  const int nj = njobs;
  for (int q = 0; q < nj; q++) {
    const ParseJob jb = jobs[q];
    if (jb.kind == 0) {
      uint8_t* v = static_cast<uint8_t*>(jb.dst);
      for (int i = lane; i < 256; i += 64) v[i] = i < jb.cnt ? (uint8_t)rd(jb.src + i) : 0;
    } else {
      uint16_t* qt = static_cast<uint16_t*>(jb.dst);
      const int i = lane;
      qt[natural_order(i)] = (uint16_t)(jb.kind == 2 ? ((rd(jb.src + 2 * i) << 8) | rd(jb.src + 2 * i + 1)) : rd(jb.src + i));
    }
  }
  __syncthreads();
  // validation of the tables the scan uses (jdhuff.c jpeg_make_d_derived_tbl), one lane per table
  if (s_status == SDSJ_OK && !sd.progressive && lane < 2 * sd.ncomp) {
    const int c = lane >> 1;
    const bool dc = (lane & 1) == 0;
    const HuffSpec& h = dc ? st.dc_spec[sd.comp[c].td] : st.ac_spec[sd.comp[c].ta];
    if (!huff_table_ok(h, dc)) sd.status = SDSJ_CORRUPT;
  }
  __syncthreads();
  // write back
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&st);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&tables[img]);
    for (int i = lane; i < (int)(sizeof(ImgTables) / 4); i += 64) dst[i] = src[i];
    const uint32_t* s2 = reinterpret_cast<const uint32_t*>(&sd);
    uint32_t* d2 = reinterpret_cast<uint32_t*>(&descs[img]);
    for (int i = lane; i < (int)(sizeof(ImgDesc) / 4); i += 64) d2[i] = s2[i];
  }
}

// ------------------------------------------------------------------------------------------
// k_plan: one workgroup; exclusive scan of per-image scratch needs -> absolute offsets.
// ------------------------------------------------------------------------------------------
// The routes of one planned image (k_plan's lists; host planning's route masks): unstuffing (-1 for
// progressive images), entropy variant by the Huffman tables in use (slots as load_tables counts
// them), resample variant as plan_image chose it (-1 for an empty crop).
SDSJ_HD inline void image_routes(const ImgDesc& d, int* ru, int* re, int* rr) {
  const int ns = huff_slots(d);
  *ru = d.progressive ? -1 : (d.ntiles > kUsSerialTiles || d.lat ? kRtUsBig : kRtUsSmall);
  *re = d.progressive ? kRtProg : ns > 4 ? kRtEnt10 : (d.ent_groups > 1 ? kRtEnt11M : kRtEnt11);
  *rr = d.geo == kGeoZeros ? -1
        : !d.fused ? kRtUnfused
                   : (d.rs_fast ? rs_route(d.rs_lay, d.rs_fast) : gen_route(d.need_h ? d.ksh : 1));
}

// k_plan, in two kernels.  k_plan_scan (one workgroup): exclusive scan of the images' scratch needs
// from the previous lane's total (each image's plan_base, the lane's total), route counters zeroed.
// k_plan_apply (one thread per image): capacity check, the image's scratch offsets, its route-list
// entries -- counted per workgroup in LDS, one global atomic per route and workgroup (the lists'
// order is the workgroups' arrival order; every image still lands in exactly its lists).
__global__ void __launch_bounds__(1024) k_plan_scan(int n, ImgDesc* __restrict__ descs, const int64_t* __restrict__ base,
                                                    int64_t* __restrict__ total_out, int32_t* __restrict__ routes) {
  __shared__ int64_t part[1024];
  __shared__ int64_t carry;
  const int t = threadIdx.x;
  if (t == 0) carry = base ? *base : 0;  // a second lane allocates after the first
  if (t < kRouteSlots) routes[t] = 0;    // route counts, then work counters
  __syncthreads();
  for (int b0 = 0; b0 < n; b0 += 1024) {
    const int i = b0 + t;
    int64_t need = 0;
    if (i < n && descs[i].status == SDSJ_OK) need = descs[i].need;
    part[t] = need;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int64_t v = t >= off ? part[t - off] : 0;
      __syncthreads();
      part[t] += v;
      __syncthreads();
    }
    if (i < n) descs[i].plan_base = carry + part[t] - need;
    __syncthreads();
    if (t == 1023) carry += part[1023];
    __syncthreads();
  }
  if (t == 0) *total_out = carry;
}

constexpr int kPlanThreads = 256;
__global__ void __launch_bounds__(kPlanThreads) k_plan_apply(int n, ImgDesc* __restrict__ descs, int64_t capacity,
                                                             int32_t* __restrict__ routes, int cap) {
  __shared__ int lcnt[kNumRoutes], gbase[kNumRoutes];
  const int t = threadIdx.x, i = blockIdx.x * kPlanThreads + t;
  if (t < kNumRoutes) lcnt[t] = 0;
  __syncthreads();
  int ru = -1, re = -1, rr = -1, iu = 0, ie = 0, ir = 0, ig = 0, ng = 0;
  if (i < n && descs[i].status == SDSJ_OK) {
    ImgDesc& d = descs[i];
    const int64_t start = d.plan_base;
    if (start + d.need > capacity) {
      d.status = SDSJ_ECAPACITY;
    } else {
      d.off_ustream += start;
      d.off_seg += start;
      d.off_tiles += start;
      d.off_sub += start;
      d.off_rec += start;
      d.off_ptab += start;
      d.off_coef += start;
      d.off_planes += start;
      d.off_rgb += start;
      d.off_tmp += start;
      d.off_kh += start;
      d.off_kv += start;
      // routes (image_routes): unstuffing -- one workgroup per small image, tile-parallel passes for
      // the rest --, entropy variant, resample variant
      image_routes(d, &ru, &re, &rr);
      if (ru >= 0) iu = atomicAdd(&lcnt[ru], 1);
      ie = atomicAdd(&lcnt[re], 1);
      if (re == kRtEnt11M) {
        ng = d.ent_groups;
        ig = atomicAdd(&lcnt[kRtEnt11G], ng);
      }
      if (rr >= 0) ir = atomicAdd(&lcnt[rr], 1);
    }
  }
  __syncthreads();
  if (t < kNumRoutes) gbase[t] = lcnt[t] ? atomicAdd(&routes[t], lcnt[t]) : 0;
  __syncthreads();
  if (ru >= 0) routes[kRouteSlots + ru * cap + gbase[ru] + iu] = i;
  if (re >= 0) routes[kRouteSlots + re * cap + gbase[re] + ie] = i;
  if (ng) {
    int32_t* gt = group_tasks(routes, cap);
    for (int q = 0; q < ng; q++) gt[gbase[kRtEnt11G] + ig + q] = (i << kGroupShift) | q;
  }
  if (rr >= 0) routes[kRouteSlots + rr * cap + gbase[rr] + ir] = i;
}

// k_finish: publishes every sample's status and accumulates the engine's per-process counters
// (SDSJ_CTR_*): one thread per sample, counters summed in LDS, one 64-bit atomic per counter and
// workgroup (lengths == null: the frames path).  k_zerofill then writes the zeros of failed samples and empty crops
// (presets.py:160-162 normalise maps them to -1.0 through the LUT, as zeros would).
__global__ void __launch_bounds__(256) k_finish(int n, const ImgDesc* __restrict__ descs, sdsj_op op,
                                                int32_t* __restrict__ status, const int32_t* __restrict__ lengths,
                                                unsigned long long* __restrict__ counters) {
  __shared__ unsigned long long acc[SDSJ_NUM_COUNTERS];
  const int t = threadIdx.x, img = blockIdx.x * 256 + t;
  if (t < SDSJ_NUM_COUNTERS) acc[t] = 0;
  __syncthreads();
  const int64_t total = (int64_t)op.out_h * op.out_w * 3;
  if (img < n) {
    const ImgDesc* d = &descs[img];
    const int st = d->status;  // (k_parse: EINVAL for a sample outside the blob / a negative length)
    status[img] = st;
    if (counters) {
      const int k = st == SDSJ_OK ? SDSJ_CTR_OK
                    : st == SDSJ_UNSUPPORTED ? SDSJ_CTR_UNSUPPORTED
                    : st == SDSJ_CORRUPT ? SDSJ_CTR_CORRUPT
                    : st == SDSJ_ECAPACITY ? SDSJ_CTR_CAPACITY : SDSJ_CTR_OTHER;
      atomicAdd(&acc[lengths ? SDSJ_CTR_IMAGES : SDSJ_CTR_FRAMES], 1ull);
      atomicAdd(&acc[k], 1ull);
      if (lengths && lengths[img] > 0) atomicAdd(&acc[SDSJ_CTR_BYTES_IN], (unsigned long long)lengths[img]);
      atomicAdd(&acc[SDSJ_CTR_BYTES_OUT], (unsigned long long)(total * (op.out_dtype == SDSJ_DTYPE_F32 ? 4 : 1)));
      if (lengths && st == SDSJ_OK && d->progressive) atomicAdd(&acc[SDSJ_CTR_PROGRESSIVE], 1ull);
    }
  }
  __syncthreads();
  if (counters && t < SDSJ_NUM_COUNTERS && acc[t]) atomicAdd(&counters[t], acc[t]);
}

// k_zerofill: zeros of failed samples and empty crops.  Work items = (image, chunk of 1/kZeroChunks of
// its output); a capped grid strides over them.  A workgroup reads the status of its next 256 items at
// once (one per thread) into LDS and then fills the flagged ones, so a batch without failures costs one
// coalesced descriptor pass (item by item, the status reads were a dependent chain: 84 us per 16,384
// images), and a batch of failures is still filled by the whole grid.
constexpr int kZeroChunks = 16;
constexpr int kZeroGrid = 2048;
__global__ void __launch_bounds__(256) k_zerofill(int n, const ImgDesc* __restrict__ descs, sdsj_op op,
                                                  void* __restrict__ out, const float* __restrict__ lut) {
  __shared__ int32_t fill[256];  // the window's flagged items, compacted
  __shared__ int nfill;
  const int t = threadIdx.x;
  const int64_t total = (int64_t)op.out_h * op.out_w * 3, per = (total + kZeroChunks - 1) / kZeroChunks;
  const int64_t items = (int64_t)n * kZeroChunks;
  for (int64_t k0 = 0; blockIdx.x + k0 * gridDim.x < items; k0 += 256) {
    const int64_t w = blockIdx.x + (k0 + t) * gridDim.x;  // this thread's item of the window
    bool f = false;
    if (w < items) {
      const ImgDesc* d = &descs[w / kZeroChunks];
      f = d->status != SDSJ_OK || d->geo == kGeoZeros;
    }
    if (t == 0) nfill = 0;
    __syncthreads();
    if (f) fill[atomicAdd(&nfill, 1)] = t;  // (a window without failures: one barrier, no loop -- the scan
    __syncthreads();                         //  of all 256 flags cost a single-image call ~10 us)
    for (int q = 0; q < nfill; q++) {
      const int k = fill[q];
      const int64_t wk = blockIdx.x + (k0 + k) * gridDim.x;
      const int img = (int)(wk / kZeroChunks), ch = (int)(wk % kZeroChunks);
      const int64_t e0 = ch * per, e1 = e0 + per < total ? e0 + per : total;
      if (op.out_dtype == SDSJ_DTYPE_F32) {
        float* o = reinterpret_cast<float*>(out) + (int64_t)img * total;
        const float z = lut[0];
        for (int64_t i = e0 + t; i < e1; i += blockDim.x) o[i] = z;
      } else {
        uint8_t* o = reinterpret_cast<uint8_t*>(out) + (int64_t)img * total;
        for (int64_t i = e0 + t; i < e1; i += blockDim.x) o[i] = 0;
      }
    }
    __syncthreads();  // fill reused
  }
}

// ------------------------------------------------------------------------------------------
// Unstuffing: removes FF00 stuffing and fill bytes, splits at RSTn markers and stops at the first
// other marker (jdhuff.c jpeg_fill_bit_buffer semantics).  The entropy-coded data is cut into 8 KiB
// tiles; each thread classifies 32 consecutive bytes (read as realigned dwords).  Three passes over
// the tiles of all images at once:
//   k_us_count  per tile: bytes emitted and split markers before the tile's end marker
//   k_us_scan   per image: exclusive prefixes over its tiles, the tile the scan ends in, lengths
//   k_us_write  per tile: one packed (emitted, split) scan places the bytes, the tile is assembled
//               in LDS and leaves as aligned 16-byte stores (byte stores for the two boundary chunks
//               it shares with its neighbours)
// ------------------------------------------------------------------------------------------
constexpr int kUnstuffThreads = 256;
constexpr int kUsBytes = 32;
constexpr int kUsTile = kUnstuffThreads * kUsBytes;
static_assert(kUsTile == kUsTileBytes, "tile table granularity");
constexpr int kUsGrid = 16;  // virtual workgroups per kRtUsBig image in k_us_count / k_us_write
constexpr int kUsLaunch = 1024;  // workgroups of the route-striding unstuff kernels
constexpr int kUsNone = 0x7fffffff;
constexpr int kUsSkip = 2, kUsFinal = 1;  // UsTile.code after k_us_scan

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int a = __shfl_up(v, o, 64);
    v += lane >= o ? a : 0;
  }
  return v;
}

// jdmarker.c read_markers after the scan, up to EOI, from the marker whose last FF is raw[pos]
// (thread-serial; normally one step: EOI).
__device__ int post_scan_markers(const uint8_t* raw, int64_t n, int64_t pos) {
  for (int guard = 0; guard < 4096; guard++) {
    if (pos + 1 >= n) return SDSJ_OK;
    const int m = raw[pos + 1];
    const int64_t body = pos + 2;
    if (m == 0xD9) return SDSJ_OK;
    if ((m >= 0xD0 && m <= 0xD7) || m == 0x01) {
      pos = body;
    } else {
      const bool is_seg = (m >= 0xE0 && m <= 0xEF) || m == 0xFE || m == 0xDC || m == 0xCC || m == 0xDD || m == 0xC4 ||
                          m == 0xDB;
      if (!is_seg) return SDSJ_CORRUPT;  // second SOI/SOF/SOS, JPGn, unknown (JERR_*)
      if (body + 2 > n) return SDSJ_OK;
      const int64_t len = (raw[body] << 8) | raw[body + 1];
      if (len < 2) return SDSJ_CORRUPT;
      if (body + len > n) return SDSJ_OK;
      const uint8_t* q = raw + body + 2;
      const int64_t sl = len - 2;
      if (m == 0xDD && len != 4) return SDSJ_CORRUPT;
      if (m == 0xC4) {
        for (int64_t k = 0; k < sl;) {
          if (k + 17 > sl || (q[k] >> 4) > 1 || (q[k] & 15) > 3) return SDSJ_CORRUPT;
          int64_t cnt = 0;
          for (int l = 1; l <= 16; l++) cnt += q[k + l];
          if (cnt > 256 || k + 17 + cnt > sl) return SDSJ_CORRUPT;
          k += 17 + cnt;
        }
      }
      if (m == 0xDB) {
        for (int64_t k = 0; k < sl;) {
          if ((q[k] & 15) > 3) return SDSJ_CORRUPT;
          const int64_t need = 1 + 64 * ((q[k] >> 4) ? 2 : 1);
          if (k + need > sl) return SDSJ_CORRUPT;
          k += need;
        }
      }
      pos = body + len;
    }
    // next_marker: skip data bytes, fill bytes and FF00 pairs
    for (;;) {
      while (pos < n && raw[pos] != 0xFF) pos++;
      if (pos >= n) return SDSJ_OK;
      int64_t p = pos + 1;
      while (p < n && raw[p] == 0xFF) p++;
      if (p >= n) return SDSJ_OK;
      if (raw[p] != 0) {
        pos = p - 1;
        break;
      }
      pos = p + 1;
    }
  }
  return SDSJ_CORRUPT;
}

// Restart intervals -> data segments, then the markers after the scan (one thread; kept out of line
// so its registers do not weigh on the tile loop).
__device__ void finish_scan(ImgDesc* d, const SegView sv, const uint8_t* raw, int64_t L, int m, int end_code,
                                       int64_t end_raw, int64_t out_pos, int overflow) {
  const int nseg = d->nseg;
  int status = SDSJ_OK;
  if (overflow) status = SDSJ_CORRUPT;
  // the input ended inside the scan (no marker): Pillow reports "image file is truncated"
  if (end_code < 0) status = SDSJ_CORRUPT;
  // Restart intervals -> data segments D_0 = [0, mk_out[0]), D_i = [mk_out[i-1], mk_out[i]),
  // D_m = [mk_out[m-1], out_pos); the marker after D_i is mk[i] (i < m) or the end marker.
  // jdhuff.c process_restart -> jdmarker.c read_restart_marker / jpeg_resync_to_restart.
  auto d_lo = [&](int i) { return i == 0 ? 0 : sv.mk_out[i - 1]; };
  auto d_hi = [&](int i) { return i < m ? sv.mk_out[i] : (int32_t)out_pos; };
  int cand = 0;  // the data segment being read / the marker after it
  sv.lo[0] = 0;
  sv.hi[0] = d_hi(0);
  sv.flag[0] = 0;
  for (int k = 1; k < nseg && status == SDSJ_OK; k++) {
    const int desired = (k - 1) & 7;
    for (;;) {
      const int mc = cand < m ? sv.mk_code[cand] : end_code;
      int action;
      if (mc == 0xD0 + desired) action = 1;
      else if (mc < 0xC0) action = 2;
      else if (mc < 0xD0 || mc > 0xD7) action = 3;
      else if (mc == 0xD0 + ((desired + 1) & 7) || mc == 0xD0 + ((desired + 2) & 7)) action = 3;
      else if (mc == 0xD0 + ((desired - 1) & 7) || mc == 0xD0 + ((desired - 2) & 7)) action = 2;
      else action = 1;
      if (action == 1) {  // marker consumed: the interval decodes the next data segment
        cand++;
        sv.lo[k] = d_lo(cand);
        sv.hi[k] = d_hi(cand);
        sv.flag[k] = 0;
        break;
      }
      if (action == 3) {  // marker left unread: an empty segment
        sv.lo[k] = sv.hi[k] = d_hi(cand);
        sv.flag[k] = kSegEmpty;
        break;
      }
      if (cand >= m) {  // (unreachable: the end marker is >= SOF0, an end of input failed above)
        status = SDSJ_CORRUPT;
        break;
      }
      cand++;  // action 2: skip to the next marker
    }
  }
  // jpeg_finish_decompress: markers from the one after the last decoded data up to EOI
  for (; status == SDSJ_OK && cand < m; cand++) {
    const int mc = sv.mk_code[cand];
    if (!((mc >= 0xD0 && mc <= 0xD7) || mc == 0x01)) status = SDSJ_CORRUPT;  // unknown marker
  }
  if (status == SDSJ_OK)
    status = post_scan_markers(raw, d->entropy_off + L, d->entropy_off + end_raw);
  sv.lo[nseg] = sv.hi[nseg] = (int32_t)out_pos;
  if (status != SDSJ_OK) d->status = status;
}

// Bytes [my0, my0 + 32) of the entropy-coded data classified as bit masks (bit k = byte k): FF bytes
// are skipped (fill / stuffing prefix); a byte after FF is a stuffed zero (emitted as 0xFF) or a
// marker code; markers split the data (RSTn, and codes below SOF0: the restart logic decides) or end
// it (any other marker, or the end of the input).  u[1..8] hold the 32 bytes, u[0] the 4 before
// (entropy_off >= 4, so they are header bytes of the same image).
struct UsClass {
  uint32_t u[9];
  uint32_t emit, stuffed, split, endm, vmask;
  uint32_t fillstuff;  // stuffed zeros preceded by two or more FF bytes (FF FF .. 00)
};
__device__ __forceinline__ int us_byte(const UsClass& c, int k) {
  uint32_t dw = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) dw = q == (k >> 2) ? c.u[1 + q] : dw;
  return (int)(dw >> (8 * (k & 3))) & 0xFF;
}
// Bytes past the input are never emitted (us_classify's vmask), so their values do not matter; the 4
// bytes before the entropy-coded data are header bytes.
struct UsRaw {
  uint32_t v[10];
};
// The ten dwords holding bytes [my0 - 4, my0 + 32), from four aligned 16-byte loads covering them:
// (e + my0) & 15 is the same for every thread of the image (tiles and threads start at multiples of
// 16), so the ten dwords sit at a wave-uniform offset into the sixteen loaded.  (Ten dword loads at a
// 32-byte lane stride measured 1.5x slower in k_us_count, profiles/r04_ab.txt.)  Chunks past the one
// holding the input's last byte read that one (same page); a chunk before the one holding byte -4
// (only for my0 = 0 and (e & 15) >= 4, and then unused) reads that one, so nothing before the image's
// headers is touched.  Loads go through the global address space as a native vector (HIP's uint4
// struct is loaded as flat, and flat loads also count on lgkmcnt, i.e. on every LDS wait).
typedef uint32_t us_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void us_load(const uint8_t* e, int64_t L, int64_t my0, UsRaw& r) {
  const uintptr_t a = (uintptr_t)(e + my0) & 15;
  const us_u32x4* A = reinterpret_cast<const us_u32x4*>((uintptr_t)(e + my0) - a - 16);
  const us_u32x4* first = reinterpret_cast<const us_u32x4*>(((uintptr_t)e - 4) & ~(uintptr_t)15);
  const us_u32x4* last = reinterpret_cast<const us_u32x4*>(((uintptr_t)(e + L) - 1) & ~(uintptr_t)15);
  uint32_t D[16];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const us_u32x4* p = A + i < first ? first : A + i;
    const us_u32x4 q = *(const __attribute__((address_space(1))) us_u32x4*)(p < last ? p : last);
    D[4 * i] = q.x;
    D[4 * i + 1] = q.y;
    D[4 * i + 2] = q.z;
    D[4 * i + 3] = q.w;
  }
  switch (__builtin_amdgcn_readfirstlane((int)(a >> 2))) {  // (uniform: static register indices)
#define US_CASE(S)                                                       \
  case S:                                                                \
    _Pragma("unroll") for (int k = 0; k < 10; k++) r.v[k] = D[S + 3 + k]; \
    break;
    US_CASE(0)
    US_CASE(1)
    US_CASE(2)
    default:
    US_CASE(3)
#undef US_CASE
  }
}
__device__ __forceinline__ void us_classify(const uint8_t* e, int64_t L, int64_t my0, const UsRaw& r, UsClass& c) {
  const int sh = (int)((uintptr_t)(e + my0) & 3);
#pragma unroll
  for (int k = 0; k < 9; k++) c.u[k] = (uint32_t)((((uint64_t)r.v[k + 1] << 32) | r.v[k]) >> (8 * sh));
  // per byte (SWAR, bit 7 of each byte lane): zero, 0xFF, and "a marker code that splits the data"
  // (RSTn, or below SOF0), then packed to bit masks (bit k = byte k)
  auto pack = [](uint32_t m) { return ((m >> 7) & 1) | ((m >> 14) & 2) | ((m >> 21) & 4) | ((m >> 28) & 8); };
  auto zbytes = [](uint32_t x) { return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u; };
  uint32_t isff = 0, isz = 0, issp = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint32_t x = c.u[1 + q];
    const uint32_t ge_c0 = x & (x << 1) & 0x80808080u;               // top two bits set
    const uint32_t rst = zbytes((x ^ 0xD0D0D0D0u) & 0xF8F8F8F8u);    // 0xD0..0xD7
    isz |= pack(zbytes(x)) << (4 * q);
    isff |= pack(zbytes(~x)) << (4 * q);
    issp |= pack((~ge_c0 & 0x80808080u) | rst) << (4 * q);
  }
  const uint32_t prevff = (isff << 1) | ((my0 > 0 && (c.u[0] >> 24) == 0xFF) ? 1u : 0u);
  const int64_t nvalid = L - my0;
  c.vmask = nvalid >= kUsBytes ? 0xFFFFFFFFu : (nvalid <= 0 ? 0u : ((1u << nvalid) - 1u));
  const uint32_t marker = prevff & ~isz & ~isff & c.vmask;
  c.stuffed = prevff & isz;
  // FF FF .. 00 (fill bytes before a stuffed zero; not valid JPEG, jdhuff.c jpeg_fill_bit_buffer reads it
  // as one FF data byte): libjpeg-turbo's decode_mcu_fast takes the first FF FF for a marker, decodes the
  // rest of that MCU from zero bits into the coefficient blocks, then decode_mcu_slow re-decodes the MCU
  // over them -- coefficients the slow path leaves zero keep the fast path's values.  Streams that hold it
  // are reported SDSJ_CORRUPT (the transforms rerun them on PIL).
  const uint32_t prev2ff = (isff << 2) | ((my0 > 0 && (c.u[0] >> 24) == 0xFF) ? 2u : 0u) |
                           ((my0 > 0 && ((c.u[0] >> 16) & 0xFF) == 0xFF) ? 1u : 0u);
  c.fillstuff = c.stuffed & prev2ff;
  c.emit = ~isff & ~marker & c.vmask;
  c.split = marker & issp;
  c.endm = (marker & ~issp) | ~c.vmask;  // the first byte past the input ends the data as well
}

// Tile end: the first ending byte of the tile (kUsNone: none), from every thread's classification
// (one barrier; wmin is free again after the caller's next barrier).
__device__ __forceinline__ int us_my_end(const UsClass& c, int t) {
  return c.endm ? t * kUsBytes + __builtin_ctz(c.endm) : kUsNone;
}
__device__ __forceinline__ int us_tile_end(int my_end, int t, int* wmin) {
  int m = my_end;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = min(m, __shfl_xor(m, o, 64));
  if ((t & 63) == 0) wmin[t >> 6] = m;
  __syncthreads();
  int r = wmin[0];
#pragma unroll
  for (int q = 1; q < kUnstuffThreads / 64; q++) r = min(r, wmin[q]);
  return r;
}
// The ending marker's code (-1: the end of the input), from the thread that holds it.
__device__ __forceinline__ int us_end_code(const UsClass& c, int t, int tile_end) {
  const int k = tile_end - t * kUsBytes;
  return ((c.vmask >> k) & 1) ? us_byte(c, k) : -1;
}

__device__ __forceinline__ uint32_t us_below(int tile_end, int t) {
  int lim = tile_end - t * kUsBytes;
  lim = lim < 0 ? 0 : (lim > kUsBytes ? kUsBytes : lim);
  return lim >= kUsBytes ? 0xFFFFFFFFu : ((1u << lim) - 1u);
}

// Places one tile's bytes at output offset obase and its split markers from entry sbase: one packed
// (emitted, split) scan, assembly in LDS, aligned 16-byte stores (byte stores for the boundary chunks
// shared with the neighbouring tiles).  The final tile is followed by kUPad zero bytes (the bit reader
// over-reads) to a 16-byte end.  Returns the tile's packed total.  Block-uniform call; buf and wsum are
// free again after the caller's next barrier.
// buf: [16 + kUsTile + kUPad + 16] bytes; the last 16 take the skipped bytes' stores
__device__ int us_place(const UsClass& c, int64_t my0, int t, int tile_end, int64_t obase, int sbase, bool final,
                        uint8_t* out, const SegView& sv, uint8_t* buf, int* wsum) {
  const int lane = t & 63, wv = t >> 6;
  const uint32_t below = us_below(tile_end, t);
  const uint32_t em = c.emit & below, sp = c.split & below;
  const int packed = __popc(em) | (__popc(sp) << 16);
  const int incl = wave_incl_scan(packed);
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  int before = 0, total = 0;
#pragma unroll
  for (int q = 0; q < kUnstuffThreads / 64; q++) {
    before += q < wv ? wsum[q] : 0;
    total += wsum[q];
  }
  const int excl = before + incl - packed;
  const int head = (int)(obase & 15);  // buf[i] is output byte (obase & ~15) + i
  // an emitted byte is itself, or 0xFF for the stuffed 0x00 of an FF00 pair; every byte is stored
  // (branch-free), the skipped ones to a dummy slot past the tile
  constexpr int kDummy = 16 + kUsTile + kUPad;
  int pos = head + (excl & 0xFFFF);
#pragma unroll
  for (int q = 0; q < kUsBytes / 4; q++) {
    const uint32_t sm = (c.stuffed >> (4 * q)) & 0xF;
    const uint32_t wq = c.u[1 + q] | (((sm * 0x00204081u) & 0x01010101u) * 0xFFu);
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const int k = 4 * q + b;
      const int bit = (int)((em >> k) & 1);
      buf[bit ? pos : kDummy] = (uint8_t)(wq >> (8 * b));
      pos += bit;
    }
  }
  int m = sbase + (excl >> 16);
  for (uint32_t mk = sp; mk; m++) {  // rare: the split markers, in order
    const int k = __builtin_ctz(mk);
    mk &= mk - 1;
    if (m < sv.cap) {  // (the image is marked corrupt otherwise)
      sv.mk_out[m] = (int32_t)(obase + (excl & 0xFFFF) + __popc(em & ((1u << k) - 1u)));
      sv.mk_raw[m] = (int32_t)(my0 + k - 1);
      sv.mk_code[m] = us_byte(c, k);
    }
  }
  const int len = head + (total & 0xFFFF);
  const int stop = final ? ((len + kUPad + 15) & ~15) : len;
  for (int i = len + t; i < stop; i += kUnstuffThreads) buf[i] = 0;
  __syncthreads();
  uint8_t* dst = out + (obase & ~(int64_t)15);
  const int first_full = (head + 15) >> 4, end_full = stop >> 4;
  for (int i = first_full + t; i < end_full; i += kUnstuffThreads)
    reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(buf)[i];
  if (end_full < first_full) {  // the tile's bytes lie inside one chunk
    if (t >= head && t < stop) dst[t] = buf[t];
  } else {
    if (t < 16 && t >= head && first_full > 0) dst[t] = buf[t];              // chunk shared with the previous tile
    if (t < (stop & 15)) dst[end_full * 16 + t] = buf[end_full * 16 + t];  // chunk shared with the next tile
  }
  return total;
}

// The scan's bookkeeping once its length is known: split-marker overflow, restart-interval ends; the
// padding of an empty scan.
__device__ void us_finish(ImgDesc* d, const SegView& sv, int t, int64_t ulen, int nsplit, int end_code,
                          int64_t end_raw, uint8_t* out) {
  if (t == 0) {
    d->ulen = ulen;
    d->useg_found = 1 + nsplit;
    d->scan_end_code = end_code;
    d->scan_end_raw = end_raw;
    if (nsplit > sv.cap) d->status = SDSJ_CORRUPT;  // more split markers than slots
  }
  if (d->ntiles == 0)  // no entropy-coded data: an empty stream and its padding
    for (int i = t; i < (kUPad >> 4); i += kUnstuffThreads) reinterpret_cast<uint4*>(out)[i] = make_uint4(0, 0, 0, 0);
  const int nseg = d->nseg;
  const int64_t bps = d->restart_interval ? (int64_t)d->restart_interval * d->bpm : d->total_blocks;
  for (int k = t; k < nseg; k += kUnstuffThreads) {
    const int64_t ge = (int64_t)(k + 1) * bps;
    sv.vend[k] = (int32_t)(ge < d->total_blocks ? ge : d->total_blocks);
  }
}

// Images of at most kUsSerialTiles tiles (route kRtUsSmall): one workgroup per image, tile after tile.
// 6 waves per SIMD (80 VGPRs, from 84 at the default 5): -2 % per launch (8: 64 VGPRs with spills, +6 %;
// profiles/r05_ab.txt)
#ifndef SDSJ_US_WAVES
#define SDSJ_US_WAVES 6
#endif
#define SDSJ_US_OCC __attribute__((amdgpu_waves_per_eu(SDSJ_US_WAVES)))
__global__ void __launch_bounds__(kUnstuffThreads) SDSJ_US_OCC k_us_serial(const uint8_t* __restrict__ blob,
                                                               const int64_t* __restrict__ offsets,
                                                               ImgDesc* __restrict__ descs, uint8_t* __restrict__ scratch,
                                                               const int32_t* __restrict__ routes, int cap) {
  __shared__ alignas(16) uint8_t buf[16 + kUsTile + kUPad + 16];
  __shared__ int wsum[kUnstuffThreads / 64];
  __shared__ int wmin[kUnstuffThreads / 64];
  __shared__ int s_code;
  const int t = threadIdx.x;
  const int cnt = routes[kRtUsSmall];
  const int32_t* lst = route_list(routes, cap, kRtUsSmall);
  for (int q = blockIdx.x; q < cnt; q += gridDim.x) {
    const int img = lst[q];
    ImgDesc* d = &descs[img];
    const uint8_t* e = blob + offsets[img] + d->entropy_off;
    const int64_t L = d->entropy_len;
    const int ntiles = d->ntiles;
    uint8_t* out = scratch + d->off_ustream;  // 256-byte aligned
    const SegView sv = seg_view(scratch + d->off_seg, d->nseg);
    int64_t obase = 0, end_raw = -1;
    int nsplit = 0, end_code = -1;
    UsRaw raw;
    if (ntiles > 0) us_load(e, L, t * kUsBytes, raw);
    for (int j = 0; j < ntiles; j++) {
      const int64_t my0 = (int64_t)j * kUsTile + t * kUsBytes;
      UsClass c;
      us_classify(e, L, my0, raw, c);
      if (j + 1 < ntiles) us_load(e, L, my0 + kUsTile, raw);  // the next tile's loads fly meanwhile
      const int my_end = us_my_end(c, t);
      const int tile_end = us_tile_end(my_end, t, wmin);
      const bool ends = tile_end != kUsNone;
      if (ends && my_end == tile_end) s_code = us_end_code(c, t, tile_end);
      // (restart intervals: libjpeg-turbo decodes every MCU with decode_mcu_slow, no divergence)
      if ((c.fillstuff & us_below(tile_end, t)) && d->restart_interval == 0) d->status = SDSJ_CORRUPT;
      const int tot = us_place(c, my0, t, tile_end, obase, nsplit, ends || j == ntiles - 1, out, sv, buf, wsum);
      obase += tot & 0xFFFF;
      nsplit += tot >> 16;
      if (ends) {
        end_code = s_code;  // (written before us_place's barriers)
        end_raw = (int64_t)j * kUsTile + tile_end - 1;
        break;
      }
    }
    us_finish(d, sv, t, obase, nsplit, end_code, end_raw, out);
  }
}

// Larger images (route kRtUsBig): kUsGrid virtual workgroups per image stride over its tiles.
// Pass 1 -- per tile: bytes emitted and split markers before the tile's end, the end and its code.
__global__ void __launch_bounds__(kUnstuffThreads) k_us_count(const uint8_t* __restrict__ blob,
                                                              const int64_t* __restrict__ offsets,
                                                              ImgDesc* __restrict__ descs, uint8_t* __restrict__ scratch,
                                                              const int32_t* __restrict__ routes, int cap) {
  __shared__ int wsum[kUnstuffThreads / 64];
  __shared__ int wmin[kUnstuffThreads / 64];
  __shared__ int s_code;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int cnt = routes[kRtUsBig];
  const int32_t* lst = route_list(routes, cap, kRtUsBig);
  for (int v = blockIdx.x; v < cnt * kUsGrid; v += gridDim.x) {
    const int img = lst[v / kUsGrid];
    const ImgDesc* d = &descs[img];
    const int ntiles = d->ntiles;
    const uint8_t* e = blob + offsets[img] + d->entropy_off;
    const int64_t L = d->entropy_len;
    UsTile* tiles = reinterpret_cast<UsTile*>(scratch + d->off_tiles);
    for (int j = v % kUsGrid; j < ntiles; j += kUsGrid) {
      const int64_t my0 = (int64_t)j * kUsTile + t * kUsBytes;
      UsRaw raw;
      UsClass c;
      us_load(e, L, my0, raw);
      us_classify(e, L, my0, raw, c);
      const int my_end = us_my_end(c, t);
      const int tile_end = us_tile_end(my_end, t, wmin);
      if (tile_end != kUsNone && my_end == tile_end) s_code = us_end_code(c, t, tile_end);
      const uint32_t below = us_below(tile_end, t);
      int packed = __popc(c.emit & below) | (__popc(c.split & below) << 16);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) packed += __shfl_xor(packed, o, 64);
      if (lane == 0) wsum[wv] = packed;
      __syncthreads();
      if (t == 0) {
        int tot = 0;
#pragma unroll
        for (int q = 0; q < kUnstuffThreads / 64; q++) tot += wsum[q];
        UsTile r;
        r.emit = tot & 0xFFFF;
        r.split = tot >> 16;
        r.end = tile_end == kUsNone ? -1 : tile_end;
        r.code = tile_end == kUsNone ? -1 : s_code;
        tiles[j] = r;
      }
      __syncthreads();  // wsum, wmin and s_code read
    }
  }
}

// Pass 2 -- one workgroup per image: tile records -> {bytes before, split markers before, end,
// kUsFinal / kUsSkip / 0}; the scan's length, split count and end marker.
__global__ void __launch_bounds__(kUnstuffThreads) k_us_scan(ImgDesc* __restrict__ descs, uint8_t* __restrict__ scratch,
                                                             const int32_t* __restrict__ routes, int cap) {
  __shared__ int wsum[3][kUnstuffThreads / 64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int cnt = routes[kRtUsBig];
  const int32_t* lst = route_list(routes, cap, kRtUsBig);
  for (int q = blockIdx.x; q < cnt; q += gridDim.x) {
    ImgDesc* d = &descs[lst[q]];
    const int ntiles = d->ntiles;
    const SegView sv = seg_view(scratch + d->off_seg, d->nseg);
    UsTile* tiles = reinterpret_cast<UsTile*>(scratch + d->off_tiles);
    int ebase = 0, sbase = 0, ended = 0;  // totals over the chunks before this one
    int64_t ulen = 0, end_raw = -1;
    int nsplit = 0, end_code = -1;
    for (int j0 = 0; j0 < ntiles; j0 += kUnstuffThreads) {
      const int j = j0 + t;
      const UsTile r = j < ntiles ? tiles[j] : UsTile{0, 0, -1, -1};
      const int hasend = r.end >= 0 ? 1 : 0;
      const int ie = wave_incl_scan(r.emit), is = wave_incl_scan(r.split), ih = wave_incl_scan(hasend);
      if (lane == 63) {
        wsum[0][wv] = ie;
        wsum[1][wv] = is;
        wsum[2][wv] = ih;
      }
      __syncthreads();
      int be = 0, bs = 0, bh = 0, te = 0, ts = 0, th = 0;
#pragma unroll
      for (int w = 0; w < kUnstuffThreads / 64; w++) {
        be += w < wv ? wsum[0][w] : 0;
        bs += w < wv ? wsum[1][w] : 0;
        bh += w < wv ? wsum[2][w] : 0;
        te += wsum[0][w];
        ts += wsum[1][w];
        th += wsum[2][w];
      }
      const int ends_before = ended + bh + ih - hasend;
      if (j < ntiles) {
        UsTile o;
        o.emit = ebase + be + ie - r.emit;
        o.split = sbase + bs + is - r.split;
        o.end = r.end >= 0 ? r.end : kUsNone;
        const bool final = ends_before == 0 && (hasend || j == ntiles - 1);
        o.code = ends_before > 0 ? kUsSkip : (final ? kUsFinal : 0);
        tiles[j] = o;
        if (final) {  // (one thread of the image)
          ulen = o.emit + r.emit;
          nsplit = o.split + r.split;
          end_code = hasend ? r.code : -1;
          end_raw = hasend ? (int64_t)j * kUsTile + r.end - 1 : -1;
          d->ulen = ulen;
          d->useg_found = 1 + nsplit;
          d->scan_end_code = end_code;
          d->scan_end_raw = end_raw;
          if (nsplit > sv.cap) d->status = SDSJ_CORRUPT;  // more split markers than slots
        }
      }
      ebase += te;
      sbase += ts;
      ended += th;
      __syncthreads();  // wsum read
    }
    const int nseg = d->nseg;
    const int64_t bps = d->restart_interval ? (int64_t)d->restart_interval * d->bpm : d->total_blocks;
    for (int k = t; k < nseg; k += kUnstuffThreads) {
      const int64_t ge = (int64_t)(k + 1) * bps;
      sv.vend[k] = (int32_t)(ge < d->total_blocks ? ge : d->total_blocks);
    }
  }
}

// Pass 3 -- per tile: places the bytes and markers at the offsets pass 2 found.
__global__ void __launch_bounds__(kUnstuffThreads) k_us_write(const uint8_t* __restrict__ blob,
                                                              const int64_t* __restrict__ offsets,
                                                              ImgDesc* __restrict__ descs, uint8_t* __restrict__ scratch,
                                                              const int32_t* __restrict__ routes, int cap) {
  __shared__ alignas(16) uint8_t buf[16 + kUsTile + kUPad + 16];
  __shared__ int wsum[kUnstuffThreads / 64];
  const int t = threadIdx.x;
  const int cnt = routes[kRtUsBig];
  const int32_t* lst = route_list(routes, cap, kRtUsBig);
  for (int v = blockIdx.x; v < cnt * kUsGrid; v += gridDim.x) {
    const int img = lst[v / kUsGrid];
    ImgDesc* d = &descs[img];
    if (d->status != SDSJ_OK) continue;  // (split-marker overflow found by pass 2)
    const int ntiles = d->ntiles;
    const uint8_t* e = blob + offsets[img] + d->entropy_off;
    const int64_t L = d->entropy_len;
    uint8_t* out = scratch + d->off_ustream;
    const SegView sv = seg_view(scratch + d->off_seg, d->nseg);
    const UsTile* tiles = reinterpret_cast<const UsTile*>(scratch + d->off_tiles);
    for (int j = v % kUsGrid; j < ntiles; j += kUsGrid) {
      const UsTile r = tiles[j];
      if (r.code == kUsSkip) break;  // the scan ended in an earlier tile (so it did for the later ones)
      const int64_t my0 = (int64_t)j * kUsTile + t * kUsBytes;
      UsRaw raw;
      UsClass c;
      us_load(e, L, my0, raw);
      us_classify(e, L, my0, raw, c);
      if ((c.fillstuff & us_below(r.end, t)) && d->restart_interval == 0)
        d->status = SDSJ_CORRUPT;  // FF FF .. 00 (us_classify)
      us_place(c, my0, t, r.end, r.emit, r.split, r.code == kUsFinal, out, sv, buf, wsum);
      if (r.code == kUsFinal) break;
      __syncthreads();  // buf and wsum reused
    }
  }
}

// k_scanmap: one thread per image -- restart intervals -> data segments and the markers after the scan
// (finish_scan), from what k_unstuff recorded.
__global__ void __launch_bounds__(64) k_scanmap(int n, const uint8_t* __restrict__ blob, const int64_t* __restrict__ offsets,
                                                ImgDesc* __restrict__ descs, uint8_t* __restrict__ scratch) {
  const int img = blockIdx.x * 64 + threadIdx.x;
  if (img >= n) return;
  ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK || d->progressive) return;  // progressive: k_prog reads the raw stream
  const SegView sv = seg_view(scratch + d->off_seg, d->nseg);
  finish_scan(d, sv, blob + offsets[img], d->entropy_len, d->useg_found - 1, d->scan_end_code, d->scan_end_raw, d->ulen, 0);
}

// ------------------------------------------------------------------------------------------
// k_idct: dequantisation + ISLOW IDCT with the SIMD version's 16-bit semantics (sdsj_idct.h); one block per
// thread, 256 blocks per iteration.
// ------------------------------------------------------------------------------------------
constexpr int kIdctThreads = 256;
#ifndef SDSJ_IDCT_GRID
#define SDSJ_IDCT_GRID 8
#endif
constexpr int kIdctGrid = SDSJ_IDCT_GRID;  // workgroups per image (each strides over 8-block groups)
// SDSJ_IDCT_GPW > 0 (0: kIdctGrid per image): batch launches take kIdctGridMax workgroups per image and an image uses
// ceil(total_blocks / 8 / SDSJ_IDCT_GPW) of them (1 .. kIdctGridMax; the rest exit at once), so a
// workgroup's setup is amortised over about the same number of groups whatever the image size.
#ifndef SDSJ_IDCT_GPW
#define SDSJ_IDCT_GPW 256
#endif
// (odd: workgroup k of the launch runs on XCD k mod 8, so with a grid row of 16 every image's first
// workgroups would land on the same XCDs; 17 rotates them by one XCD per image)
constexpr int kIdctGridMax = 17;

// Work unit = a group: 8 horizontally adjacent blocks of one component, one per thread, so each of
// a block's 8 row stores joins the group's other 7 in 64 contiguous bytes of a plane row.  The
// block stays in registers through both passes (64 values), so there is no LDS transpose.
#ifndef SDSJ_IDCT_WAVES
#define SDSJ_IDCT_WAVES 4  // waves per SIMD the register budget targets (124 VGPRs at 4)
#endif
__global__ void __launch_bounds__(kIdctThreads) __attribute__((amdgpu_waves_per_eu(SDSJ_IDCT_WAVES)))
k_idct(int n, const ImgDesc* __restrict__ descs,
                                                       const ImgTables* __restrict__ tables,
                                                       uint8_t* __restrict__ scratch) {
  const int img = blockIdx.y;
  if (img >= n) return;
  const ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK || d->geo == kGeoZeros) return;
  int nwg = gridDim.x;  // this image's workgroups
  if (SDSJ_IDCT_GPW > 0 && gridDim.x == kIdctGridMax) {
    const int64_t want = ((int64_t)d->total_blocks / 8 + SDSJ_IDCT_GPW - 1) / SDSJ_IDCT_GPW;
    nwg = want < 1 ? 1 : (want > kIdctGridMax ? kIdctGridMax : (int)want);
    if ((int)blockIdx.x >= nwg) return;
  }
  __shared__ alignas(16) int32_t qt[kMaxComp][64];
  __shared__ int32_t binv[kMaxComp][16];  // (dy * 4 + dx) -> MCU block index b (jdcoefct order)
  __shared__ int32_t gstart[kMaxComp + 1], ngx[kMaxComp], cbw[kMaxComp], ch_[kMaxComp], cv_[kMaxComp], cpitch[kMaxComp];
  __shared__ int32_t cgx0[kMaxComp], cby0[kMaxComp];  // first 8-block group column / block row needed
  __shared__ float rngx[kMaxComp], rch[kMaxComp], rcv[kMaxComp];  // reciprocals for the exact quotients below
  __shared__ int64_t cplane[kMaxComp];
  const int t = threadIdx.x;
  const int ncomp = d->ncomp, bpm = d->bpm, mcux = d->mcux;
  // quantisation tables in zigzag order (the coefficient blocks' order)
  for (int i = t; i < ncomp * 64; i += kIdctThreads) qt[i / 64][i % 64] = tables[img].qt[d->comp[i / 64].tq][natural_order(i % 64)];
  if (t < bpm) binv[d->blk_comp[t]][d->blk_dy[t] * 4 + d->blk_dx[t]] = t;
  if (t == 0) {
    // only the blocks whose pixels the colour/resample passes read (comp_block_rect: the crop's source
    // rectangle widened by one sample), in groups of 8 horizontally adjacent blocks aligned to 8 block
    // columns, so each group's row stores fill whole 64-byte plane segments (groups starting at the
    // first needed block column instead: k_idct 4.70 -> 5.18 ms per 16,384, profiles/r05_ab.txt)
    int acc = 0;
    for (int c = 0; c < ncomp; c++) {
      const CompDesc& cd = d->comp[c];
      int bx0, bx1, by0, by1;
      const bool any = comp_block_rect(*d, c, bx0, bx1, by0, by1);
      gstart[c] = acc;
      cgx0[c] = bx0 >> 3;
      ngx[c] = (bx1 >> 3) - cgx0[c] + 1;
      cby0[c] = by0;
      cbw[c] = cd.bw;
      ch_[c] = ncomp == 1 ? 1 : cd.h;
      cv_[c] = ncomp == 1 ? 1 : cd.v;
      cpitch[c] = cd.pitch;
      cplane[c] = cd.plane_off;
      rngx[c] = 1.0f / (float)ngx[c];
      rch[c] = 1.0f / (float)ch_[c];
      rcv[c] = 1.0f / (float)cv_[c];
      acc += any ? ngx[c] * (by1 - by0 + 1) : 0;
    }
    gstart[ncomp] = acc;
  }
  __syncthreads();
  const int lb = t & 7;  // this lane's block within its group
  const int16_t* coef = reinterpret_cast<const int16_t*>(scratch + d->off_coef);
  uint8_t* planes = scratch + d->off_planes;
  const int ngroups = gstart[ncomp];
  // blocks the entropy decoder left zero (jdhuff.c insufficient_data): from vend[k] to the end of
  // restart interval k, and all of an empty interval entered out of data
  const SegView sv = seg_view(scratch + d->off_seg, d->nseg);
  const int nseg = d->nseg;
  const int bps = d->restart_interval ? d->restart_interval * bpm : (int)d->total_blocks;
  const int vend0 = d->progressive ? 0 : sv.vend[0];
  const bool prog = d->progressive != 0;  // (k_prog decodes every block; no cut intervals)
  auto zero_block = [&](int g) {
    if (prog) return false;
    if (nseg == 1) return g >= vend0;
    const int k = g / bps;
    return g >= sv.vend[k] || (k > 0 && (sv.flag[k] & kSegEmpty) && (sv.flag[k - 1] & kSegIns));
  };
  // a / b for 0 <= a < 2^22, 1 <= b: float estimate, then one correction each way (exact)
  auto qdiv = [](int a, int b, float rb) {
    int q = (int)((float)a * rb);
    q -= q * b > a ? 1 : 0;
    q += (q + 1) * b <= a ? 1 : 0;
    return q;
  };
  // block lb of group grp: component, block coordinates, decode-order index (g < 0: none)
  auto locate = [&](int grp, int& c, int& by, int& bx, int& g) {
    c = ncomp > 1 && grp >= gstart[1] ? (ncomp > 2 && grp >= gstart[2] ? 2 : 1) : 0;
    const int local = grp - gstart[c];
    const int byl = qdiv(local, ngx[c], rngx[c]);
    by = cby0[c] + byl;
    bx = (cgx0[c] + local - byl * ngx[c]) * 8 + lb;
    g = -1;
    if (grp < ngroups && bx < cbw[c]) {
      const int h = ch_[c], v = cv_[c];
      const int mx = qdiv(bx, h, rch[c]), my = qdiv(by, v, rcv[c]);
      g = (my * mcux + mx) * bpm + binv[c][(by - my * v) * 4 + (bx - mx * h)];
    }
  };
  // One block per lane, held in registers: dequantise, columns (pass 1), rows (pass 2), each row's 8
  // bytes stored straight to the plane -- no LDS transposes.  The 8 lanes of a group write 64
  // contiguous bytes of a plane row per store.
  for (int grp = blockIdx.x * (kIdctThreads / 8) + (t >> 3); grp < ngroups; grp += nwg * (kIdctThreads / 8)) {
    int c, by, bx, g;
    locate(grp, c, by, bx, g);
    if (g < 0) continue;
    // the block (zigzag order, k_entwrite / k_prog), or zeros where the entropy decoder left it zero
    const uint4* src = reinterpret_cast<const uint4*>(coef + (int64_t)g * 64);
    const bool zb = zero_block(g);
    uint4 raw[8];
#pragma unroll
    for (int i = 0; i < 8; i++) raw[i] = zb ? make_uint4(0, 0, 0, 0) : src[i];
    // `ac`: any raw coefficient outside row 0 (the SIMD pass 1's zero test); row 0 is zigzag positions
    // 0, 1, 5, 6, 14, 15, 27 and 28
    uint32_t ac = raw[0].y | (raw[0].z & 0xFFFFu) | (raw[0].w & 0xFFFF0000u) | raw[1].x | raw[1].y | raw[1].z |
                  raw[3].x | (raw[3].y & 0xFFFFu) | (raw[3].z & 0xFFFF0000u) | raw[3].w;
#pragma unroll
    for (int i = 2; i < 8; i++) ac |= i == 3 ? 0u : (raw[i].x | raw[i].y | raw[i].z | raw[i].w);
    // DEQUANTIZE as vpmullw: the low 16 bits of coef * quantval, zigzag position k into row-major
    // natural_order(k)
    int x[64];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int4 q0 = *reinterpret_cast<const int4*>(&qt[c][i * 8]), q1 = *reinterpret_cast<const int4*>(&qt[c][i * 8 + 4]);
      const uint32_t w[4] = {raw[i].x, raw[i].y, raw[i].z, raw[i].w};
      const int q[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int cv = (int)(int16_t)((w[k >> 1] >> ((k & 1) * 16)) & 0xFFFF);
        x[natural_order(i * 8 + k)] = wrap16(cv * q[k]);
      }
    }
    // pass 1: columns.  A block whose rows 1..7 are all zero takes the SIMD shortcut (vpsllw: every
    // column is the dequantised DC << PASS1_BITS, wrapped to 16 bits); otherwise every column runs the
    // butterfly, saturated to 16 bits.  On such a block the butterfly of column k gives sat16(4 x[k]) in
    // every row, so the shortcut is the butterfly on x[k] = wrap16(4 x[k]) / 4 (exact: a multiple of 4).
    if (!ac) {
#pragma unroll
      for (int k = 0; k < 8; k++) x[k] = wrap16(x[k] * 4) >> 2;
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
      uint32_t o[8];
      islow_1d(x[k], x[8 + k], x[16 + k], x[24 + k], x[32 + k], x[40 + k], x[48 + k], x[56 + k], o);
#pragma unroll
      for (int j = 0; j < 8; j++) x[j * 8 + k] = descale_p1(o[j]);
    }
    // pass 2: rows -> 8 bytes of plane row by * 8 + r
    uint8_t* dst = planes + cplane[c] + (int64_t)(by * 8) * cpitch[c] + bx * 8;
#pragma unroll
    for (int r = 0; r < 8; r++) {
      uint32_t o[8];
      islow_1d(x[r * 8], x[r * 8 + 1], x[r * 8 + 2], x[r * 8 + 3], x[r * 8 + 4], x[r * 8 + 5], x[r * 8 + 6], x[r * 8 + 7], o);
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) lo |= descale_p2(o[k]) << (8 * k);
#pragma unroll
      for (int k = 0; k < 4; k++) hi |= descale_p2(o[k + 4]) << (8 * k);
      *reinterpret_cast<uint2*>(dst + (int64_t)r * cpitch[c]) = make_uint2(lo, hi);
    }
  }
}

// ------------------------------------------------------------------------------------------
// k_color: fancy upsampling (jdsample.c, context rows per jdmainct.c) + ycc_rgb_convert.
// One thread per RGB pixel of rows [src_y0, src_y1) x cols [src_x0, src_x0 + src_w).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int up_sample(const uint8_t* P, const CompDesc& c, int x, int y) {
  if (c.rh == 1 && c.rv == 1) return P[(int64_t)y * c.pitch + x];
  const int dw = c.dw, dh = c.dh;
  if (c.rv == 2) {
    const int i = y >> 1;
    int f = (y & 1) ? i + 1 : i - 1;
    f = f < 0 ? 0 : (f > dh - 1 ? dh - 1 : f);
    const uint8_t* r0 = P + (int64_t)i * c.pitch;
    const uint8_t* r1 = P + (int64_t)f * c.pitch;
    if (c.rh == 2) {
      const int jx = x >> 1;
      if (dw <= 2) return P[(int64_t)i * c.pitch + jx];  // h2v2_upsample (box)
      const int cs = r0[jx] * 3 + r1[jx];
      if ((x & 1) == 0) {
        const int k = jx > 0 ? jx - 1 : 0;
        const int cn = jx > 0 ? r0[k] * 3 + r1[k] : cs;
        return (cs * 3 + cn + 8) >> 4;
      } else {
        const int k = jx < dw - 1 ? jx + 1 : dw - 1;
        const int cn = jx < dw - 1 ? r0[k] * 3 + r1[k] : cs;
        return (cs * 3 + cn + 7) >> 4;
      }
    }
    // h1v2_fancy_upsample
    return (r0[x] * 3 + r1[x] + ((y & 1) ? 2 : 1)) >> 2;
  }
  // rh == 2, rv == 1: h2v1
  const uint8_t* row = P + (int64_t)y * c.pitch;
  const int jx = x >> 1;
  const int a = row[jx];
  if (dw <= 2) return a;
  if ((x & 1) == 0) return jx == 0 ? a : (a * 3 + row[jx - 1] + 1) >> 2;
  return jx == dw - 1 ? a : (a * 3 + row[jx + 1] + 2) >> 2;
}

__device__ __forceinline__ uint32_t clamp255(int v) { return (uint32_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

__device__ __forceinline__ void ycc_to_rgb(int y, int cb, int cr, uint32_t* r, uint32_t* g, uint32_t* b) {
  // jdcolor.c tables evaluated arithmetically (identical integer results)
  const int x_cb = cb - 128, x_cr = cr - 128;
  const int cr_r = (91881 * x_cr + 32768) >> 16;
  const int cb_b = (116130 * x_cb + 32768) >> 16;
  const int g_add = (-46802 * x_cr + (-22554 * x_cb + 32768)) >> 16;
  *r = clamp255(y + cr_r);
  *g = clamp255(y + g_add);
  *b = clamp255(y + cb_b);
}

__global__ void __launch_bounds__(256) k_color(int n, const ImgDesc* __restrict__ descs, uint8_t* __restrict__ scratch,
                                               const int32_t* __restrict__ routes, int cap) {
 const int32_t* rl = route_list(routes, cap, kRtUnfused);
 for (int li = blockIdx.y; li < routes[kRtUnfused]; li += gridDim.y) {
  const int img = rl[li];
  const ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK || d->geo == kGeoZeros || d->fused) continue;
  const int w = d->src_w, h = d->src_y1 - d->src_y0;
  const int64_t total = (int64_t)w * h;
  const uint8_t* planes = scratch + d->off_planes;
  uint8_t* rgb = scratch + d->off_rgb;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int yy = (int)(i / w), xx = (int)(i - (int64_t)yy * w);
    const int x = d->src_x0 + xx, y = d->src_y0 + yy;
    uint32_t R, G, B;
    const int Y = up_sample(planes + d->comp[0].plane_off, d->comp[0], x, y);
    if (d->ncomp == 1) {
      R = G = B = (uint32_t)Y;
    } else {
      const int cb = up_sample(planes + d->comp[1].plane_off, d->comp[1], x, y);
      const int cr = up_sample(planes + d->comp[2].plane_off, d->comp[2], x, y);
      ycc_to_rgb(Y, cb, cr, &R, &G, &B);
    }
    uint8_t* o = rgb + i * 3;
    o[0] = (uint8_t)R;
    o[1] = (uint8_t)G;
    o[2] = (uint8_t)B;
  }
 }
}

// ------------------------------------------------------------------------------------------
// k_coeffs: Pillow precompute_coeffs + normalize_coeffs_8bpc for both passes (doubles).
// ------------------------------------------------------------------------------------------
__device__ double filt_eval(int filter, double x) {
  switch (filter) {
    case SDSJ_FILTER_BOX:
      return (x > -0.5 && x <= 0.5) ? 1.0 : 0.0;
    case SDSJ_FILTER_BILINEAR:
      if (x < 0.0) x = -x;
      return x < 1.0 ? 1.0 - x : 0.0;
    case SDSJ_FILTER_HAMMING:
      if (x < 0.0) x = -x;
      if (x == 0.0) return 1.0;
      if (x >= 1.0) return 0.0;
      x = x * M_PI;
      return sin(x) / x * (0.54 + 0.46 * cos(x));
    case SDSJ_FILTER_BICUBIC: {
      const double a = -0.5;
      if (x < 0.0) x = -x;
      if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
      if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
      return 0.0;
    }
    default: {
      if (!(-3.0 <= x && x < 3.0)) return 0.0;
      double s1 = x == 0.0 ? 1.0 : sin(x * M_PI) / (x * M_PI);
      double x3 = x / 3;
      double s2 = x3 == 0.0 ? 1.0 : sin(x3 * M_PI) / (x3 * M_PI);
      return s1 * s2;
    }
  }
}

// NEAREST: one tap of weight 1.0 (ksize 1) at the source index of Pillow's running sum, or none (fill
// value 0).  One thread walks the whole axis (the running sum is sequential; a per-index restart
// would cost O(out^2)).
__device__ void nearest_axis(int in_size, int out_size, int32_t* bounds, int32_t* kk) {
  const double a = (double)in_size / out_size;
  double xo = 0.0 + a * 0.5;
  for (int xx = 0; xx < out_size; xx++, xo += a) {
    const int xin = xo < 0.0 ? -1 : (int)xo;
    const int s = (xin >= 0 && xin < in_size) ? xin : -1;
    kk[xx] = 1 << 22;
    bounds[2 * xx] = s < 0 ? 0 : s;
    bounds[2 * xx + 1] = s < 0 ? 0 : 1;
  }
}

__device__ void coeffs_one(int in_size, int out_size, int filter, int ksize, int xx, int32_t* bounds, int32_t* kk) {
  if (filter == SDSJ_FILTER_NEAREST) {
    if (xx == 0) nearest_axis(in_size, out_size, bounds, kk);
    return;
  }
  const double scale = (double)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = filter_support(filter) * filterscale;
  const double center = 0.0 + (xx + 0.5) * scale;
  double ww = 0.0;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  double w[64];
  int32_t* k = kk + (int64_t)xx * ksize;
  // two passes: the weights are recomputed rather than stored when ksize > 64
  for (int x = 0; x < xmax; x++) {
    double v = filt_eval(filter, (x + xmin - center + 0.5) * ss);
    if (x < 64) w[x] = v;
    ww += v;
  }
  for (int x = 0; x < xmax; x++) {
    double v = x < 64 ? w[x] : filt_eval(filter, (x + xmin - center + 0.5) * ss);
    if (ww != 0.0) v /= ww;
    double s = v * (double)(1 << 22);
    k[x] = v < 0 ? (int32_t)(-0.5 + s) : (int32_t)(0.5 + s);
  }
  for (int x = xmax; x < ksize; x++) k[x] = 0;
  bounds[2 * xx] = xmin;
  bounds[2 * xx + 1] = xmax;
}

__global__ void __launch_bounds__(256) k_coeffs(int n, ImgDesc* __restrict__ descs, sdsj_op op,
                                                uint8_t* __restrict__ scratch) {
  const int img = blockIdx.y;
  if (img >= n) return;
  ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK || d->geo != kGeoResize) return;
  // an image whose crop and passes equal the lane's first image's uses that image's tables (same
  // inputs, same Pillow coefficients): most batches hold one source size
  if (img > 0) {
    const ImgDesc* a = &descs[0];
    if (a->status == SDSJ_OK && a->geo == kGeoResize && a->cw == d->cw && a->ch == d->ch && a->need_h == d->need_h &&
        a->need_v == d->need_v && a->ksh == d->ksh && a->ksv == d->ksv) {
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        d->off_kh = a->off_kh;  // (absolute scratch offsets after k_plan_apply)
        d->off_kv = a->off_kv;
      }
      return;
    }
  }
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (d->need_h && i < op.out_w) {
    int32_t* b = reinterpret_cast<int32_t*>(scratch + d->off_kh);
    coeffs_one(d->cw, op.out_w, op.filter, d->ksh, i, b, b + 2 * op.out_w);
  }
  if (d->need_v && i < op.out_h) {
    int32_t* b = reinterpret_cast<int32_t*>(scratch + d->off_kv);
    coeffs_one(d->ch, op.out_h, op.filter, d->ksv, i, b, b + 2 * op.out_h);
  }
}

__device__ __forceinline__ uint32_t clip8(int32_t v) {
  v >>= 22;
  return (uint32_t)(v < 0 ? 0 : v > 255 ? 255 : v);
}

// ------------------------------------------------------------------------------------------
// k_hpass: rows [yf, yl) of the crop, out_w columns; taps clamp to the crop window.
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_hpass(int n, const ImgDesc* __restrict__ descs, sdsj_op op,
                                               uint8_t* __restrict__ scratch, const int32_t* __restrict__ routes, int cap) {
 const int32_t* rl = route_list(routes, cap, kRtUnfused);
 for (int li = blockIdx.y; li < routes[kRtUnfused]; li += gridDim.y) {
  const int img = rl[li];
  const ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK || !d->need_h || d->fused) continue;
  const int rows = d->yl - d->yf, ow = op.out_w;
  const int64_t total = (int64_t)rows * ow;
  const int32_t* bounds = reinterpret_cast<const int32_t*>(scratch + d->off_kh);
  const int32_t* kk = bounds + 2 * ow;
  const uint8_t* rgb = scratch + d->off_rgb;
  uint8_t* tmp = scratch + d->off_tmp;
  const int sw = d->rgb_pitch, ks = d->ksh;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int yy = (int)(i / ow), xx = (int)(i - (int64_t)yy * ow);
    const int xmin = bounds[2 * xx], xmax = bounds[2 * xx + 1];
    const int32_t* k = kk + (int64_t)xx * ks;
    const uint8_t* row = rgb + ((int64_t)yy * sw + xmin) * 3;
    int32_t s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
    for (int x = 0; x < xmax; x++) {
      const int32_t c = k[x];
      s0 += row[3 * x] * c;
      s1 += row[3 * x + 1] * c;
      s2 += row[3 * x + 2] * c;
    }
    uint8_t* o = tmp + i * 3;
    o[0] = (uint8_t)clip8(s0);
    o[1] = (uint8_t)clip8(s1);
    o[2] = (uint8_t)clip8(s2);
  }
 }
}

// ------------------------------------------------------------------------------------------
// k_vpass: vertical pass (or copy) + hflip + CHW/HWC layout + uint8 / float32 LUT output.
// Failed samples get zeros.  Also publishes the per-sample status.
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_vpass(int n, const ImgDesc* __restrict__ descs, sdsj_op op,
                                               const uint8_t* __restrict__ scratch, const uint8_t* __restrict__ flip,
                                               void* __restrict__ out, const int32_t* __restrict__ routes, int cap,
                                               const float* __restrict__ lut) {
 const int32_t* rl = route_list(routes, cap, kRtUnfused);
 for (int li = blockIdx.y; li < routes[kRtUnfused]; li += gridDim.y) {
  const int img = rl[li];
  const ImgDesc* d = &descs[img];
  const int oh = op.out_h, ow = op.out_w;
  const int64_t plane = (int64_t)oh * ow;
  const int64_t total = plane;
  // failed / empty-crop images are written (and every status published) by k_finish
  if (d->status != SDSJ_OK || d->geo == kGeoZeros || d->fused) continue;
  const bool zeros = false;
  const bool fl = flip ? flip[img] != 0 : false;
  const bool f32 = op.out_dtype == SDSJ_DTYPE_F32;
  const bool hwc = op.layout == SDSJ_LAYOUT_HWC;
  uint8_t* o8 = reinterpret_cast<uint8_t*>(out) + (f32 ? 0 : img * plane * 3);
  float* of = reinterpret_cast<float*>(out) + (f32 ? img * plane * 3 : 0);
  // source: H-pass output (need_h) or the materialised RGB rows (crop columns)
  const uint8_t* src = zeros ? nullptr : (d->need_h ? scratch + d->off_tmp : scratch + d->off_rgb);
  const int sw = d->need_h ? ow : d->rgb_pitch;
  const int32_t* bounds = d->need_v ? reinterpret_cast<const int32_t*>(scratch + d->off_kv) : nullptr;
  const int32_t* kk = bounds ? bounds + 2 * oh : nullptr;
  const int ks = d->ksv, yf = d->yf;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int yy = (int)(i / ow), xx = (int)(i - (int64_t)yy * ow);
    uint32_t v0 = 0, v1 = 0, v2 = 0;
    if (!zeros) {
      if (d->need_v) {
        const int ymin = bounds[2 * yy] - yf, ymax = bounds[2 * yy + 1];
        const int32_t* k = kk + (int64_t)yy * ks;
        int32_t s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
        for (int y = 0; y < ymax; y++) {
          const uint8_t* p = src + ((int64_t)(y + ymin) * sw + xx) * 3;
          const int32_t c = k[y];
          s0 += p[0] * c;
          s1 += p[1] * c;
          s2 += p[2] * c;
        }
        v0 = clip8(s0);
        v1 = clip8(s1);
        v2 = clip8(s2);
      } else {
        const uint8_t* p = src + ((int64_t)yy * sw + xx) * 3;
        v0 = p[0];
        v1 = p[1];
        v2 = p[2];
      }
    }
    const int ox = fl ? ow - 1 - xx : xx;
    const int64_t pix = (int64_t)yy * ow + ox;
    if (f32) {
      float* b = of;
      if (hwc) {
        b[pix * 3] = lut[v0];
        b[pix * 3 + 1] = lut[v1];
        b[pix * 3 + 2] = lut[v2];
      } else {
        b[pix] = lut[v0];
        b[plane + pix] = lut[v1];
        b[2 * plane + pix] = lut[v2];
      }
    } else {
      uint8_t* b = o8;
      if (hwc) {
        b[pix * 3] = (uint8_t)v0;
        b[pix * 3 + 1] = (uint8_t)v1;
        b[pix * 3 + 2] = (uint8_t)v2;
      } else {
        b[pix] = (uint8_t)v0;
        b[plane + pix] = (uint8_t)v1;
        b[2 * plane + pix] = (uint8_t)v2;
      }
    }
  }
 }
}

// ------------------------------------------------------------------------------------------
// Host-side launchers (called by the engine; all asynchronous on `stream`).
// ------------------------------------------------------------------------------------------
hipError_t launch_parse(int n, const uint8_t* blob, int64_t blob_bytes, const int64_t* offsets, const int32_t* lengths,
                        const sdsj_op& op, int warm_bits, bool small, ImgDesc* descs, ImgTables* tables, hipStream_t s) {
  hipLaunchKernelGGL(k_parse, dim3(n), dim3(64), 0, s, n, blob, blob_bytes, offsets, lengths, op, warm_bits, (int)small,
                     descs, tables);
  return hipGetLastError();
}
hipError_t launch_plan(int n, ImgDesc* descs, int64_t capacity, const int64_t* base, int64_t* total, int32_t* routes,
                       int cap, hipStream_t s) {
  hipLaunchKernelGGL(k_plan_scan, dim3(1), dim3(1024), 0, s, n, descs, base, total, routes);
  if (n > 0)
    hipLaunchKernelGGL(k_plan_apply, dim3((n + kPlanThreads - 1) / kPlanThreads), dim3(kPlanThreads), 0, s, n, descs,
                       capacity, routes, cap);
  return hipGetLastError();
}
hipError_t launch_unstuff(int n, const uint8_t* blob, const int64_t* offsets, ImgDesc* descs, uint8_t* scratch,
                          const int32_t* routes, int cap, hipStream_t s, uint64_t rm, uint64_t hint) {
  const int g = n < kUsLaunch ? n : kUsLaunch;
#ifndef SDSJ_US_TILE_GRID
#define SDSJ_US_TILE_GRID 16384
#endif
  const int gt = n * kUsGrid < SDSJ_US_TILE_GRID ? n * kUsGrid : SDSJ_US_TILE_GRID;
#ifndef SDSJ_US_SERIAL_GRID
#define SDSJ_US_SERIAL_GRID 16384
#endif
  const int gs = n < SDSJ_US_SERIAL_GRID ? n : SDSJ_US_SERIAL_GRID;
  if (route_on(rm, kRtUsSmall))
    hipLaunchKernelGGL(k_us_serial, dim3(route_grid(hint, kRtUsSmall, gs)), dim3(kUnstuffThreads), 0, s, blob, offsets, descs,
                       scratch, routes, cap);
  if (route_on(rm, kRtUsBig)) {  // (the three kernels stride over their work)
    hipLaunchKernelGGL(k_us_count, dim3(route_grid(hint, kRtUsBig, gt)), dim3(kUnstuffThreads), 0, s, blob, offsets, descs,
                       scratch, routes, cap);
    hipLaunchKernelGGL(k_us_scan, dim3(route_grid(hint, kRtUsBig, g)), dim3(kUnstuffThreads), 0, s, descs, scratch, routes,
                       cap);
    hipLaunchKernelGGL(k_us_write, dim3(route_grid(hint, kRtUsBig, gt)), dim3(kUnstuffThreads), 0, s, blob, offsets, descs,
                       scratch, routes, cap);
  }
  return hipGetLastError();
}
hipError_t launch_finish(int n, ImgDesc* descs, const sdsj_op& op, void* out, int32_t* status, const float* lut,
                         const int32_t* lengths, unsigned long long* counters, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_finish, dim3((n + 255) / 256), dim3(256), 0, s, n, descs, op, status, lengths, counters);
  const int zg = n * kZeroChunks < kZeroGrid ? n * kZeroChunks : kZeroGrid;
  hipLaunchKernelGGL(k_zerofill, dim3(zg), dim3(256), 0, s, n, descs, op, out, lut);
  return hipGetLastError();
}
hipError_t launch_scanmap(int n, const uint8_t* blob, const int64_t* offsets, ImgDesc* descs, uint8_t* scratch,
                          hipStream_t s) {
  hipLaunchKernelGGL(k_scanmap, dim3((n + 63) / 64), dim3(64), 0, s, n, blob, offsets, descs, scratch);
  return hipGetLastError();
}
hipError_t launch_idct(int n, const ImgDesc* descs, const ImgTables* tables, uint8_t* scratch, hipStream_t s) {
  // (a few images: more workgroups per image, for latency)
  hipLaunchKernelGGL(k_idct, dim3(n <= kSmallBatch ? 8 * kIdctGrid : (SDSJ_IDCT_GPW > 0 ? kIdctGridMax : kIdctGrid), n), dim3(kIdctThreads), 0, s, n, descs,
                     tables, scratch);
  return hipGetLastError();
}
hipError_t launch_color(int n, const ImgDesc* descs, uint8_t* scratch, const int32_t* routes, int cap, hipStream_t s,
                        uint64_t rm) {
  if (!route_on(rm, kRtUnfused)) return hipSuccess;
  hipLaunchKernelGGL(k_color, dim3(64, n < 64 ? n : 64), dim3(256), 0, s, n, descs, scratch, routes, cap);
  return hipGetLastError();
}
hipError_t launch_coeffs(int n, ImgDesc* descs, const sdsj_op& op, uint8_t* scratch, hipStream_t s) {
  int mx = op.out_w > op.out_h ? op.out_w : op.out_h;
  hipLaunchKernelGGL(k_coeffs, dim3((mx + 255) / 256, n), dim3(256), 0, s, n, descs, op, scratch);
  return hipGetLastError();
}
hipError_t launch_hpass(int n, const ImgDesc* descs, const sdsj_op& op, uint8_t* scratch, const int32_t* routes, int cap,
                        hipStream_t s, uint64_t rm) {
  if (!route_on(rm, kRtUnfused)) return hipSuccess;
  hipLaunchKernelGGL(k_hpass, dim3(32, n < 64 ? n : 64), dim3(256), 0, s, n, descs, op, scratch, routes, cap);
  return hipGetLastError();
}
hipError_t launch_vpass(int n, const ImgDesc* descs, const sdsj_op& op, const uint8_t* scratch, const uint8_t* flip,
                        void* out, const int32_t* routes, int cap, const float* lut, hipStream_t s, uint64_t rm) {
  if (!route_on(rm, kRtUnfused)) return hipSuccess;
  hipLaunchKernelGGL(k_vpass, dim3(32, n < 64 ? n : 64), dim3(256), 0, s, n, descs, op, scratch, flip, out, routes, cap, lut);
  return hipGetLastError();
}

}  // namespace sdsj

namespace sdsj {
struct HostReader {
  const uint8_t* p;
  int operator()(int64_t i) const { return p[i]; }
};

int64_t host_plan_frame(ImgDesc* d, int width, int height, const sdsj_op& op) {
  *d = ImgDesc{};
  d->status = SDSJ_OK;
  d->width = width;
  d->height = height;
  d->ncomp = 3;
  return plan_image(d, op, true);
}

int64_t host_plan_need(const uint8_t* jpg, int64_t n, const sdsj_op& op, int* status, uint64_t* routes, bool small) {
  ImgDesc d;
  static thread_local ImgTables t;
  HostReader rd{jpg};
  int st = parse_headers(rd, n, &d, &t, CopySink<HostReader>{rd});
  if (st == SDSJ_OK) st = setup_geometry(&d, &t);
  int64_t need = 0;
  if (st == SDSJ_OK) need = plan_image(&d, op, false, small);
  *status = st;
  if (routes) {
    *routes = kAllRoutes;
    if (st == SDSJ_OK) {
      int ru, re, rr;
      image_routes(d, &ru, &re, &rr);
      *routes = (ru >= 0 ? 1ull << ru : 0) | (1ull << re) | (rr >= 0 ? 1ull << rr : 0);
    }
  }
  return need;
}
}  // namespace sdsj
