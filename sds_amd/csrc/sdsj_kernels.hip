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
__device__ __host__ inline int64_t plan_image(ImgDesc* d, const sdsj_op& op, bool frames = false) {
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
  double sup = filter_support(op.filter);
  d->ksh = d->need_h ? resample_ksize(d->cw, op.out_w, sup) : 0;
  d->ksv = d->need_v ? resample_ksize(d->ch, op.out_h, sup) : 0;
  if (d->geo == kGeoZeros) {
    d->yf = d->yl = 0;
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
  d->ring_rows = 1;
  while (d->ring_rows < d->ksv) d->ring_rows *= 2;  // vertical window rows kept per column
  if (d->geo != kGeoZeros && d->ring_rows <= kRingMaxRows) {
    const double scale = d->need_h ? (double)d->cw / op.out_w : 1.0;
    const double supp = d->need_h ? sup * (scale < 1.0 ? 1.0 : scale) : 0.0;
    int tw = op.out_w < 256 ? op.out_w : 256;
    if (tw > kRingDW / d->ring_rows) tw = kRingDW / d->ring_rows;
    for (;;) {
      if ((double)tw * scale + 2.0 * supp + 4.0 <= (double)kMaxSpan) {
        d->fused = 1;
        d->tile_w = tw;
        break;
      }
      if (tw == 1) break;
      tw = (tw + 1) / 2;
    }
  }
  if (frames) d->fused = 0;
  // specialised fused kernel: 4:2:0 (h2v2 fancy chroma), horizontal and vertical passes, odd tap
  // counts 3..11 (sdsj_resample420.hip); everything else takes the generic k_resample
  d->rs_fast = 0;
  if (d->fused && d->ncomp == 3 && d->need_h && d->need_v && d->ksh >= 3 && d->ksh <= 11 && (d->ksh & 1) &&
      d->ring_rows <= kRingMaxRows && d->comp[0].rh == 1 && d->comp[0].rv == 1 && d->comp[1].rh == 2 &&
      d->comp[1].rv == 2 && d->comp[2].rh == 2 && d->comp[2].rv == 2 && d->comp[1].dw > 2 &&
      d->comp[2].dw == d->comp[1].dw && d->comp[2].dh == d->comp[1].dh)
    d->rs_fast = d->ksh;
  {
    const int64_t bits = d->entropy_len * 8, per_group = (int64_t)kDecodeThreads * kGroupBits;
    int64_t g = (bits + per_group - 1) / per_group;
    g = g < 1 ? 1 : (g > kMaxEntGroups ? kMaxEntGroups : g);
    d->ent_groups = frames ? 1 : (int32_t)g;
    const int64_t lanes = (int64_t)kDecodeThreads * d->ent_groups;
    d->sub_bits = (int32_t)align_up((bits + lanes - 1) / lanes, 32);
  }
  if (d->sub_bits < kMinSubBits) d->sub_bits = kMinSubBits;
  // warm-up: kWarmBits, or sub_bits / kWarmDiv for long subsequences (large images: a few percent
  // more speculative work removes nearly every sync task, each of which is a serial re-decode)
  {
    const int64_t w = d->sub_bits / kWarmDiv > kWarmBits ? d->sub_bits / kWarmDiv : kWarmBits;
    d->warm_bits = (int)(d->sub_bits * 3 / 2 < w ? d->sub_bits * 3 / 2 : w);
  }
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

__global__ void __launch_bounds__(64) k_parse(int n, const uint8_t* __restrict__ blob, const int64_t* __restrict__ offsets,
                                              const int32_t* __restrict__ lengths, sdsj_op op, int warm_bits,
                                              ImgDesc* __restrict__ descs, ImgTables* __restrict__ tables) {
  const int img = blockIdx.x;
  if (img >= n) return;
  const int lane = threadIdx.x;
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
    if (status == SDSJ_OK) plan_image(&sd, op);
    if (warm_bits >= 0) sd.warm_bits = warm_bits;
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
__global__ void __launch_bounds__(1024) k_plan(int n, ImgDesc* __restrict__ descs, int64_t capacity,
                                               const int64_t* __restrict__ base, int64_t* __restrict__ total_out,
                                               int32_t* __restrict__ routes, int cap) {
  __shared__ int64_t part[1024];
  __shared__ int64_t carry;
  __shared__ int rcnt[kNumRoutes];
  if (threadIdx.x == 0) carry = base ? *base : 0;  // a second lane allocates after the first
  if (threadIdx.x < kNumRoutes) rcnt[threadIdx.x] = 0;
  __syncthreads();
  for (int base = 0; base < n; base += 1024) {
    int i = base + threadIdx.x;
    int64_t need = 0;
    if (i < n && descs[i].status == SDSJ_OK) need = descs[i].need;
    part[threadIdx.x] = need;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      int64_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
    }
    int64_t start = carry + part[threadIdx.x] - need;
    if (i < n && descs[i].status == SDSJ_OK) {
      ImgDesc& d = descs[i];
      if (start + need > capacity) {
        d.status = SDSJ_ECAPACITY;
      } else {
        d.off_ustream += start;
        d.off_seg += start;
        d.off_sub += start;
        d.off_rec += start;
        d.off_ptab += start;
        d.off_coef += start;
        d.off_planes += start;
        d.off_rgb += start;
        d.off_tmp += start;
        d.off_kh += start;
        d.off_kv += start;
        // routes: entropy variant by the Huffman tables in use (slots as load_tables counts them),
        // resample variant as plan_image chose it
        int keys[2 * kMaxComp], ns = 0;
        for (int c = 0; c < d.ncomp; c++)
          for (int k = 0; k < 2; k++) {
            const int key = k ? (4 | d.comp[c].ta) : d.comp[c].td;
            bool seen = false;
            for (int q = 0; q < ns; q++) seen |= keys[q] == key;
            if (!seen) keys[ns++] = key;
          }
        const int re = d.progressive ? kRtProg : ns > 4 ? kRtEnt10 : (d.ent_groups > 1 ? kRtEnt11M : kRtEnt11);
        int32_t* lst = routes + kRouteSlots + re * cap;
        lst[atomicAdd(&rcnt[re], 1)] = i;
        if (re == kRtEnt11M) {
          int32_t* gt = group_tasks(routes, cap);
          const int b = atomicAdd(&rcnt[kRtEnt11G], d.ent_groups);
          for (int q = 0; q < d.ent_groups; q++) gt[b + q] = (i << kGroupShift) | q;
        }
        if (d.geo != kGeoZeros) {
          const int rr = !d.fused ? kRtUnfused
                         : (d.rs_fast ? rs_route(d.rs_fast) : gen_route(d.need_h ? d.ksh : 1));
          lst = routes + kRouteSlots + rr * cap;
          lst[atomicAdd(&rcnt[rr], 1)] = i;
        }
      }
    }
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total_out = carry;
  if (threadIdx.x < kNumRoutes) routes[threadIdx.x] = rcnt[threadIdx.x];
  else if (threadIdx.x < kRouteSlots) routes[threadIdx.x] = 0;  // work counters
}

// k_finish: publishes every sample's status and writes the zeros of failed samples and of empty
// crops (presets.py:160-162 normalise maps them to -1.0 through the LUT, as zeros would).  Also
// accumulates the engine's per-process counters (SDSJ_CTR_*): one thread per sample, a few 64-bit
// atomics per sample (lengths == null: the frames path).
__global__ void __launch_bounds__(256) k_finish(int n, const ImgDesc* __restrict__ descs, sdsj_op op,
                                                void* __restrict__ out, int32_t* __restrict__ status,
                                                const float* __restrict__ lut, const int32_t* __restrict__ lengths,
                                                unsigned long long* __restrict__ counters) {
  const int img = blockIdx.x;
  if (img >= n) return;
  const ImgDesc* d = &descs[img];
  const int st = d->status;
  const int64_t plane = (int64_t)op.out_h * op.out_w, total = plane * 3;
  if (threadIdx.x == 0) {
    status[img] = st;
    if (counters) {
      const int k = st == SDSJ_OK ? SDSJ_CTR_OK
                    : st == SDSJ_UNSUPPORTED ? SDSJ_CTR_UNSUPPORTED
                    : st == SDSJ_CORRUPT ? SDSJ_CTR_CORRUPT
                    : st == SDSJ_ECAPACITY ? SDSJ_CTR_CAPACITY : SDSJ_CTR_OTHER;
      atomicAdd(&counters[lengths ? SDSJ_CTR_IMAGES : SDSJ_CTR_FRAMES], 1ull);
      atomicAdd(&counters[k], 1ull);
      if (lengths) atomicAdd(&counters[SDSJ_CTR_BYTES_IN], (unsigned long long)(uint32_t)lengths[img]);
      atomicAdd(&counters[SDSJ_CTR_BYTES_OUT], (unsigned long long)(total * (op.out_dtype == SDSJ_DTYPE_F32 ? 4 : 1)));
      if (lengths && st == SDSJ_OK && d->progressive) atomicAdd(&counters[SDSJ_CTR_PROGRESSIVE], 1ull);
    }
  }
  if (st == SDSJ_OK && d->geo != kGeoZeros) return;
  if (op.out_dtype == SDSJ_DTYPE_F32) {
    float* o = reinterpret_cast<float*>(out) + img * total;
    const float z = lut[0];
    for (int64_t i = threadIdx.x; i < total; i += blockDim.x) o[i] = z;
  } else {
    uint8_t* o = reinterpret_cast<uint8_t*>(out) + img * total;
    for (int64_t i = threadIdx.x; i < total; i += blockDim.x) o[i] = 0;
  }
}

// ------------------------------------------------------------------------------------------
// k_unstuff: one 256-thread workgroup per image.  Removes FF00 stuffing and fill bytes, splits at
// RSTn markers and stops at the first other marker (jdhuff.c jpeg_fill_bit_buffer semantics).
// Tiles of 8 KiB: each thread classifies 32 consecutive bytes (read as realigned dwords), one
// packed (emitted, RSTn) scan places them, the tile is assembled in LDS and leaves as aligned
// 16-byte stores (the unaligned tail rides into the next tile).
// ------------------------------------------------------------------------------------------
constexpr int kUnstuffThreads = 256;
constexpr int kUsBytes = 32;
constexpr int kUsTile = kUnstuffThreads * kUsBytes;

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

__global__ void __launch_bounds__(kUnstuffThreads) k_unstuff(int n, const uint8_t* __restrict__ blob,
                                                             const int64_t* __restrict__ offsets,
                                                             ImgDesc* __restrict__ descs, uint8_t* __restrict__ scratch) {
  const int img = blockIdx.x;
  if (img >= n) return;
  ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK || d->progressive) return;  // progressive: k_prog reads the raw stream
  __shared__ alignas(16) uint8_t buf[kUsTile + 32];  // [carried tail][this tile's output]
  __shared__ int wsum[kUnstuffThreads / 64];
  __shared__ int s_end, s_end_code, s_overflow;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint8_t* raw = blob + offsets[img];
  const uint8_t* e = raw + d->entropy_off;
  const int64_t L = d->entropy_len;
  const uintptr_t e_end = (uintptr_t)(e + L);  // dwords starting below this lie in mapped pages
  uint8_t* out = scratch + d->off_ustream;  // 256-byte aligned
  const int nseg = d->nseg;
  const SegView sv = seg_view(scratch + d->off_seg, nseg);
  if (t == 0) {
    s_overflow = 0;
    s_end_code = -1;
  }

  int64_t out_pos = 0;  // bytes emitted so far; [out_pos & ~15, out_pos) sit in buf[0, carry)
  int nmk = 0;          // split markers (RSTn, and codes below SOF0) met so far
  int64_t end_raw = -1; // entropy-relative index of the last FF of the terminating marker
  bool ended = false;
  for (int64_t base = 0; base < L && !ended; base += kUsTile) {
    if (t == 0) s_end = 0x7fffffff;
    // bytes [my0 - 4, my0 + 32) as 9 realigned dwords u[0..8] (u[0] holds the 4 preceding bytes;
    // entropy_off >= 4, so they are header bytes of the same image)
    const int64_t my0 = base + (int64_t)t * kUsBytes;
    const uintptr_t a = (uintptr_t)(e + my0);
    const uint32_t* w = reinterpret_cast<const uint32_t*>((a & ~(uintptr_t)3) - 4);
    const int sh = (int)(a & 3);
    uint32_t v[10];
#pragma unroll
    for (int k = 0; k < 10; k++) v[k] = (uintptr_t)(w + k) < e_end ? w[k] : 0u;
    uint32_t u[9];
#pragma unroll
    for (int k = 0; k < 9; k++) u[k] = (uint32_t)((((uint64_t)v[k + 1] << 32) | v[k]) >> (8 * sh));
    // classify the 32 bytes as bit masks (bit k = byte k): FF bytes are skipped (fill / stuffing
    // prefix); a byte after FF is a stuffed zero (emitted as 0xFF) or a marker code; markers split
    // the data (RSTn, and codes below SOF0: the restart logic decides) or end it (any other marker,
    // or the end of the input)
    uint32_t isff = 0, isz = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t x = u[1 + q], y = ~x;
      const uint32_t zz = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;  // zero bytes
      const uint32_t zf = ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;  // 0xFF bytes
      isz |= (((zz >> 7) & 1) | ((zz >> 14) & 2) | ((zz >> 21) & 4) | ((zz >> 28) & 8)) << (4 * q);
      isff |= (((zf >> 7) & 1) | ((zf >> 14) & 2) | ((zf >> 21) & 4) | ((zf >> 28) & 8)) << (4 * q);
    }
    const uint32_t prevff = (isff << 1) | ((my0 > 0 && (u[0] >> 24) == 0xFF) ? 1u : 0u);
    const int64_t nvalid = L - my0;
    const uint32_t vmask = nvalid >= kUsBytes ? 0xFFFFFFFFu : (nvalid <= 0 ? 0u : ((1u << nvalid) - 1u));
    const uint32_t marker = prevff & ~isz & ~isff & vmask;
    const uint32_t stuffed = prevff & isz;
    const uint32_t emit = ~isff & ~marker & vmask;
    uint32_t split = 0, endm = ~vmask;  // the first byte past the input ends it as well
    for (uint32_t mk = marker; mk;) {   // rare: one iteration per marker
      const int k = __builtin_ctz(mk);
      mk &= mk - 1;
      uint32_t dw = 0;
#pragma unroll
      for (int q = 0; q < 8; q++) dw = q == (k >> 2) ? u[1 + q] : dw;
      const int c = (int)(dw >> (8 * (k & 3))) & 0xFF;
      if ((c >= 0xD0 && c <= 0xD7) || c < 0xC0) split |= 1u << k;
      else endm |= 1u << k;
    }
    const int my_end = endm ? __builtin_ctz(endm) : kUsBytes;
    __syncthreads();  // s_end initialised; buf tail of the previous tile settled
    if (my_end < kUsBytes) atomicMin(&s_end, t * kUsBytes + my_end);
    __syncthreads();
    const int tile_end = s_end;
    if (my_end < kUsBytes && tile_end == t * kUsBytes + my_end) {  // the earliest end: its marker code
      uint32_t dw = 0;
#pragma unroll
      for (int q = 0; q < 8; q++) dw = q == (my_end >> 2) ? u[1 + q] : dw;
      s_end_code = ((vmask >> my_end) & 1) ? (int)(dw >> (8 * (my_end & 3))) & 0xFF : -1;
    }
    int lim = tile_end - t * kUsBytes;
    lim = lim < 0 ? 0 : (lim > kUsBytes ? kUsBytes : lim);
    const uint32_t below = lim >= kUsBytes ? 0xFFFFFFFFu : ((1u << lim) - 1u);
    const uint32_t em = emit & below, sp = split & below;
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
    const int carry = (int)(out_pos & 15);
    int pos = excl & 0xFFFF;
#pragma unroll
    for (int k = 0; k < kUsBytes; k++) {
      // an emitted byte is itself, or 0xFF for the stuffed 0x00 of an FF00 pair
      const uint32_t rawb = (u[1 + (k >> 2)] >> (8 * (k & 3))) & 0xFF;
      if ((em >> k) & 1) buf[carry + pos++] = (uint8_t)(((stuffed >> k) & 1) ? 0xFF : rawb);
    }
    int r = nmk + (excl >> 16);
    for (uint32_t mk = sp; mk; r++) {  // rare: the split markers, in order
      const int k = __builtin_ctz(mk);
      mk &= mk - 1;
      uint32_t dw = 0;
#pragma unroll
      for (int q = 0; q < 8; q++) dw = q == (k >> 2) ? u[1 + q] : dw;
      if (r < sv.cap) {
        sv.mk_out[r] = (int32_t)(out_pos + (excl & 0xFFFF) + __popc(em & ((1u << k) - 1u)));
        sv.mk_raw[r] = (int32_t)(my0 + k - 1);
        sv.mk_code[r] = (int32_t)(dw >> (8 * (k & 3))) & 0xFF;
      } else {
        s_overflow = 1;
      }
    }
    __syncthreads();
    const int temit = total & 0xFFFF;
    // full 16-byte chunks of [out_pos & ~15, out_pos + temit) leave; the tail is carried
    const int have = carry + temit, full = have >> 4;
    uint4* dst = reinterpret_cast<uint4*>(out + (out_pos & ~(int64_t)15));
    const uint4* src = reinterpret_cast<const uint4*>(buf);
    for (int i = t; i < full; i += kUnstuffThreads) dst[i] = src[i];
    const int rem = have & 15;
    uint8_t tail = t < rem ? buf[full * 16 + t] : 0;
    __syncthreads();
    if (t < rem) buf[t] = tail;
    out_pos += temit;
    nmk += total >> 16;
    if (tile_end != 0x7fffffff) {
      ended = true;
      end_raw = base + tile_end - 1;
    }
  }
  __syncthreads();
  // the carried tail, then zero padding so the bit reader can over-read safely
  {
    const int rem = (int)(out_pos & 15);
    const int64_t a0 = out_pos & ~(int64_t)15;
    const int nchunks = (rem + kUPad + 15) >> 4;
    for (int i = t; i < nchunks; i += kUnstuffThreads) {
      uint32_t wds[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        uint32_t x = 0;
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
          const int o = i * 16 + q * 4 + bb;
          x |= (uint32_t)(o < rem ? buf[o] : 0) << (8 * bb);
        }
        wds[q] = x;
      }
      reinterpret_cast<uint4*>(out + a0)[i] = make_uint4(wds[0], wds[1], wds[2], wds[3]);
    }
  }
  const int64_t bps = d->restart_interval ? (int64_t)d->restart_interval * d->bpm : d->total_blocks;
  for (int k = t; k < nseg; k += kUnstuffThreads) {
    const int64_t ge = (int64_t)(k + 1) * bps;
    sv.vend[k] = (int32_t)(ge < d->total_blocks ? ge : d->total_blocks);
  }
  __syncthreads();
  if (t == 0) {
    d->ulen = out_pos;
    d->useg_found = 1 + nmk;
    d->scan_end_code = ended ? s_end_code : -1;
    d->scan_end_raw = end_raw;
    if (s_overflow) d->status = SDSJ_CORRUPT;
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
// k_idct: dequantisation + jpeg_idct_islow; 8 threads per block, 32 blocks per iteration.
// ------------------------------------------------------------------------------------------
constexpr int kIdctThreads = 256;
constexpr int kIdctBlocks = kIdctThreads / 8;
#ifndef SDSJ_IDCT_GRID
#define SDSJ_IDCT_GRID 8
#endif
constexpr int kIdctGrid = SDSJ_IDCT_GRID;  // workgroups per image (each strides over 8-block groups)
constexpr int kWsStride = 72;  // ints per block in LDS (conflict-free column reads per half-wave)

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
  int z1 = (z2 + z3) * SDSJ_FIX_0_541196100;
  int t2 = z1 + z3 * (-SDSJ_FIX_1_847759065);
  int t3 = z1 + z2 * SDSJ_FIX_0_765366865;
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
  int z5 = (z3 + z4) * SDSJ_FIX_1_175875602;
  t0 *= SDSJ_FIX_0_298631336;
  t1 *= SDSJ_FIX_2_053119869;
  t2 *= SDSJ_FIX_3_072711026;
  t3 *= SDSJ_FIX_1_501321110;
  z1 *= -SDSJ_FIX_0_899976223;
  z2 *= -SDSJ_FIX_2_562915447;
  z3 *= -SDSJ_FIX_1_961570560;
  z4 *= -SDSJ_FIX_0_390180644;
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

// Work unit = one wave: 8 horizontally adjacent blocks of one component (a "group"), so each of
// the 8 row stores of the wave writes 64 contiguous bytes of a plane row.  8 threads per block
// (thread r: row r, then column r); the 8 threads of a block share a wave, so the LDS transposes
// need only in-wave ordering, no workgroup barrier.
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__global__ void __launch_bounds__(kIdctThreads) k_idct(int n, const ImgDesc* __restrict__ descs,
                                                       const ImgTables* __restrict__ tables,
                                                       uint8_t* __restrict__ scratch) {
  const int img = blockIdx.y;
  if (img >= n) return;
  const ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK || d->geo == kGeoZeros) return;
  __shared__ alignas(16) int ws[kIdctBlocks * kWsStride];
  __shared__ alignas(16) int32_t qt[kMaxComp][64];
  __shared__ int32_t binv[kMaxComp][16];  // (dy * 4 + dx) -> MCU block index b (jdcoefct order)
  __shared__ int32_t gstart[kMaxComp + 1], ngx[kMaxComp], cbw[kMaxComp], ch_[kMaxComp], cv_[kMaxComp], cpitch[kMaxComp];
  __shared__ int32_t cgx0[kMaxComp], cby0[kMaxComp];  // first 8-block group column / block row needed
  __shared__ float rngx[kMaxComp], rch[kMaxComp], rcv[kMaxComp];  // reciprocals for the exact quotients below
  __shared__ int64_t cplane[kMaxComp];
  const int t = threadIdx.x;
  const int ncomp = d->ncomp, bpm = d->bpm, mcux = d->mcux;
  for (int i = t; i < ncomp * 64; i += kIdctThreads) qt[i / 64][i % 64] = tables[img].qt[d->comp[i / 64].tq][i % 64];
  if (t < bpm) binv[d->blk_comp[t]][d->blk_dy[t] * 4 + d->blk_dx[t]] = t;
  if (t == 0) {
    // only the blocks whose pixels the colour/resample passes read: the source rectangle
    // [src_x0, src_x0 + src_w) x [src_y0, src_y1) in each component's sampling, widened by one
    // sample for the fancy upsampling's neighbours (the crop drops the rest of the image)
    const int x0 = d->src_x0, x1 = d->src_x0 + d->src_w, y0 = d->src_y0, y1 = d->src_y1;
    int acc = 0;
    for (int c = 0; c < ncomp; c++) {
      const CompDesc& cd = d->comp[c];
      const int rh = ncomp == 1 ? 1 : d->hmax / cd.h, rv = ncomp == 1 ? 1 : d->vmax / cd.v;
      int cx0 = x0 / rh - 1, cx1 = (x1 - 1) / rh + 1, cy0 = y0 / rv - 1, cy1 = (y1 - 1) / rv + 1;
      cx0 = cx0 < 0 ? 0 : cx0;
      cy0 = cy0 < 0 ? 0 : cy0;
      cx1 = cx1 > cd.bw * 8 - 1 ? cd.bw * 8 - 1 : cx1;
      cy1 = cy1 > cd.bh * 8 - 1 ? cd.bh * 8 - 1 : cy1;
      gstart[c] = acc;
      cgx0[c] = cx0 >> 6;
      ngx[c] = (cx1 >> 6) - cgx0[c] + 1;
      cby0[c] = cy0 >> 3;
      cbw[c] = cd.bw;
      ch_[c] = ncomp == 1 ? 1 : cd.h;
      cv_[c] = ncomp == 1 ? 1 : cd.v;
      cpitch[c] = cd.pitch;
      cplane[c] = cd.plane_off;
      rngx[c] = 1.0f / (float)ngx[c];
      rch[c] = 1.0f / (float)ch_[c];
      rcv[c] = 1.0f / (float)cv_[c];
      acc += x1 > x0 && y1 > y0 ? ngx[c] * ((cy1 >> 3) - cby0[c] + 1) : 0;
    }
    gstart[ncomp] = acc;
  }
  __syncthreads();
  const int lane = t & 63, wv = t >> 6, lb = lane >> 3, r = lane & 7;
  int* W = ws + (wv * 8 + lb) * kWsStride;
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
  // block of this lane in group grp: component, block coordinates, decode-order index
  // a / b for 0 <= a < 2^22, 1 <= b: float estimate, then one correction each way (exact)
  auto qdiv = [](int a, int b, float rb) {
    int q = (int)((float)a * rb);
    q -= q * b > a ? 1 : 0;
    q += (q + 1) * b <= a ? 1 : 0;
    return q;
  };
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
  const int gstride = gridDim.x * 4;
  // transform + store the block of this lane (g < 0: none) from its coefficient row `raw`
  auto process = [&](const uint4& raw, int c, int by, int bx, int g) {
    const bool valid = g >= 0;
    if (valid) {
      // row r of the block, dequantised (DEQUANTIZE: coef * quantval), stored as two 16-byte writes
      const uint4 v = zero_block(g) ? make_uint4(0, 0, 0, 0) : raw;
      const int4 q0 = *reinterpret_cast<const int4*>(&qt[c][r * 8]), q1 = *reinterpret_cast<const int4*>(&qt[c][r * 8 + 4]);
      auto lo16 = [](uint32_t x) { return (int)(int16_t)(x & 0xFFFF); };
      auto hi16 = [](uint32_t x) { return (int)(int16_t)(x >> 16); };
      *reinterpret_cast<int4*>(W + r * 8) = make_int4(lo16(v.x) * q0.x, hi16(v.x) * q0.y, lo16(v.y) * q0.z, hi16(v.y) * q0.w);
      *reinterpret_cast<int4*>(W + r * 8 + 4) =
          make_int4(lo16(v.z) * q1.x, hi16(v.z) * q1.y, lo16(v.w) * q1.z, hi16(v.w) * q1.w);
    }
    wave_lds_sync();
    // pass 1: column r
    int col[8];
    if (valid) {
      int x[8];
      for (int k = 0; k < 8; k++) x[k] = W[k * 8 + r];
      if ((x[1] | x[2] | x[3] | x[4] | x[5] | x[6] | x[7]) == 0) {
        for (int k = 0; k < 8; k++) col[k] = x[0] * 4;  // << PASS1_BITS
      } else {
        int o[8];
        islow_1d(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], o);
        for (int k = 0; k < 8; k++) col[k] = (o[k] + (1 << 10)) >> 11;  // DESCALE(, CONST_BITS-PASS1_BITS)
      }
    }
    wave_lds_sync();
    if (valid)
      for (int k = 0; k < 8; k++) W[k * 8 + r] = col[k];
    wave_lds_sync();
    // pass 2: row r -> 8 bytes of plane row by * 8 + r
    if (valid) {
      const int4 w0 = *reinterpret_cast<const int4*>(W + r * 8), w1 = *reinterpret_cast<const int4*>(W + r * 8 + 4);
      int o[8];
      islow_1d(w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, o);
      uint32_t lo = 0, hi = 0;
      for (int k = 0; k < 4; k++) lo |= range_limit((o[k] + (1 << 17)) >> 18) << (8 * k);
      for (int k = 0; k < 4; k++) hi |= range_limit((o[k + 4] + (1 << 17)) >> 18) << (8 * k);
      *reinterpret_cast<uint2*>(planes + cplane[c] + (int64_t)(by * 8 + r) * cpitch[c] + bx * 8) = make_uint2(lo, hi);
    }
    wave_lds_sync();
  };
  // two groups in flight per wave (ping-pong registers: a loop-carried copy would force the wait)
  int c0, by0, bx0, g0, c1, by1, bx1, g1;
  int grp = blockIdx.x * 4 + wv;
  locate(grp, c0, by0, bx0, g0);
  uint4 rawA, rawB;
  rawA = *reinterpret_cast<const uint4*>(coef + (int64_t)(g0 >= 0 ? g0 : 0) * 64 + r * 8);
  for (; grp < ngroups; grp += 2 * gstride) {
    locate(grp + gstride, c1, by1, bx1, g1);
    rawB = *reinterpret_cast<const uint4*>(coef + (int64_t)(g1 >= 0 ? g1 : 0) * 64 + r * 8);  // unconditional: keeps vmcnt countable
    process(rawA, c0, by0, bx0, g0);
    if (grp + gstride >= ngroups) break;
    locate(grp + 2 * gstride, c0, by0, bx0, g0);
    rawA = *reinterpret_cast<const uint4*>(coef + (int64_t)(g0 >= 0 ? g0 : 0) * 64 + r * 8);
    process(rawB, c1, by1, bx1, g1);
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

__device__ void coeffs_one(int in_size, int out_size, int filter, int ksize, int xx, int32_t* bounds, int32_t* kk) {
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

__global__ void __launch_bounds__(256) k_coeffs(int n, const ImgDesc* __restrict__ descs, sdsj_op op,
                                                uint8_t* __restrict__ scratch) {
  const int img = blockIdx.y;
  if (img >= n) return;
  const ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK || d->geo != kGeoResize) return;
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
hipError_t launch_parse(int n, const uint8_t* blob, const int64_t* offsets, const int32_t* lengths, const sdsj_op& op,
                        int warm_bits, ImgDesc* descs, ImgTables* tables, hipStream_t s) {
  hipLaunchKernelGGL(k_parse, dim3(n), dim3(64), 0, s, n, blob, offsets, lengths, op, warm_bits, descs, tables);
  return hipGetLastError();
}
hipError_t launch_plan(int n, ImgDesc* descs, int64_t capacity, const int64_t* base, int64_t* total, int32_t* routes,
                       int cap, hipStream_t s) {
  hipLaunchKernelGGL(k_plan, dim3(1), dim3(1024), 0, s, n, descs, capacity, base, total, routes, cap);
  return hipGetLastError();
}
hipError_t launch_unstuff(int n, const uint8_t* blob, const int64_t* offsets, ImgDesc* descs, uint8_t* scratch,
                          hipStream_t s) {
  hipLaunchKernelGGL(k_unstuff, dim3(n), dim3(kUnstuffThreads), 0, s, n, blob, offsets, descs, scratch);
  return hipGetLastError();
}
hipError_t launch_finish(int n, const ImgDesc* descs, const sdsj_op& op, void* out, int32_t* status, const float* lut,
                         const int32_t* lengths, unsigned long long* counters, hipStream_t s) {
  hipLaunchKernelGGL(k_finish, dim3(n), dim3(256), 0, s, n, descs, op, out, status, lut, lengths, counters);
  return hipGetLastError();
}
hipError_t launch_scanmap(int n, const uint8_t* blob, const int64_t* offsets, ImgDesc* descs, uint8_t* scratch,
                          hipStream_t s) {
  hipLaunchKernelGGL(k_scanmap, dim3((n + 63) / 64), dim3(64), 0, s, n, blob, offsets, descs, scratch);
  return hipGetLastError();
}
hipError_t launch_idct(int n, const ImgDesc* descs, const ImgTables* tables, uint8_t* scratch, hipStream_t s) {
  hipLaunchKernelGGL(k_idct, dim3(kIdctGrid, n), dim3(kIdctThreads), 0, s, n, descs, tables, scratch);
  return hipGetLastError();
}
hipError_t launch_color(int n, const ImgDesc* descs, uint8_t* scratch, const int32_t* routes, int cap, hipStream_t s) {
  hipLaunchKernelGGL(k_color, dim3(64, n < 64 ? n : 64), dim3(256), 0, s, n, descs, scratch, routes, cap);
  return hipGetLastError();
}
hipError_t launch_coeffs(int n, const ImgDesc* descs, const sdsj_op& op, uint8_t* scratch, hipStream_t s) {
  int mx = op.out_w > op.out_h ? op.out_w : op.out_h;
  hipLaunchKernelGGL(k_coeffs, dim3((mx + 255) / 256, n), dim3(256), 0, s, n, descs, op, scratch);
  return hipGetLastError();
}
hipError_t launch_hpass(int n, const ImgDesc* descs, const sdsj_op& op, uint8_t* scratch, const int32_t* routes, int cap,
                        hipStream_t s) {
  hipLaunchKernelGGL(k_hpass, dim3(32, n < 64 ? n : 64), dim3(256), 0, s, n, descs, op, scratch, routes, cap);
  return hipGetLastError();
}
hipError_t launch_vpass(int n, const ImgDesc* descs, const sdsj_op& op, const uint8_t* scratch, const uint8_t* flip,
                        void* out, const int32_t* routes, int cap, const float* lut, hipStream_t s) {
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

int64_t host_plan_need(const uint8_t* jpg, int64_t n, const sdsj_op& op, int* status) {
  ImgDesc d;
  static thread_local ImgTables t;
  HostReader rd{jpg};
  int st = parse_headers(rd, n, &d, &t, CopySink<HostReader>{rd});
  if (st == SDSJ_OK) st = setup_geometry(&d, &t);
  int64_t need = 0;
  if (st == SDSJ_OK) need = plan_image(&d, op);
  *status = st;
  return need;
}
}  // namespace sdsj
