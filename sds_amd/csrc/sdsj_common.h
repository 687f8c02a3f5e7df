// sdsj_common.h -- structures and the JPEG header parser shared by host (probe) and device
// (parse kernel).  One implementation, compiled for both sides.
//
// The parser restates libjpeg-turbo's jdmarker.c for the subset this path decodes (SOF0/SOF1
// 8-bit sequential with one interleaved scan holding every component, SOF2 progressive -- whose
// scans k_prog parses --, Huffman coding, optional DRI): the decoder Pillow calls from
// sds/transforms/functional.py:100.  Everything else is reported as SDSJ_UNSUPPORTED (non-JPEG
// input, lossless, arithmetic, 12-bit, CMYK, Adobe-RGB, multi-scan sequential).
#pragma once
#include <stdint.h>

#include "sdsj.h"

#if defined(__HIPCC__)
#define SDSJ_HD __host__ __device__
#else
#define SDSJ_HD
#endif

namespace sdsj {

constexpr int kMaxComp = 3;
constexpr int kMaxBlocksPerMcu = 10;  // D_MAX_BLOCKS_IN_MCU
constexpr int kRec = 64;              // block-boundary records kept per subsequence by k_entsync
#ifndef SDSJ_DECODE_THREADS
#define SDSJ_DECODE_THREADS 256
#endif
constexpr int kDecodeThreads = SDSJ_DECODE_THREADS;  // threads (subsequences) per image in the entropy kernels
static_assert((kDecodeThreads & (kDecodeThreads - 1)) == 0 && kDecodeThreads >= 64 && kDecodeThreads <= 256,
              "a power of two number of waves");
constexpr int kMinSubBits = 1024;     // minimum entropy subsequence length (bits)
#ifndef SDSJ_WARM_BITS
#define SDSJ_WARM_BITS 2500
#endif
constexpr int kWarmBits = SDSJ_WARM_BITS;  // speculative warm-up before each subsequence (bits, <= 1.5 x sub_bits)
constexpr int kWarmBitsSmall = 4000;  // ... for lanes of fewer than kWarmSmallLane images (the sync pass is
constexpr int kWarmSmallLane = 512;   //     hidden by less concurrent work there, so it pays to shorten it)
constexpr int kWarmDiv = 3;           // ... or sub_bits / kWarmDiv when that is larger
// Latency mode (host-path chunks of at most kSmallBatch images, e.g. the per-sample drop-in's single
// image): the entropy work of an image spreads over up to kMaxEntGroups workgroups of short
// subsequences (kLatSubBits) with a fixed warm-up (kLatWarm), and its unstuffing goes tile-parallel,
// so one image's serial chains are short -- at the price of more warm-up work per image.
constexpr int kSmallBatch = 32;
#ifndef SDSJ_LAT_SUB
#define SDSJ_LAT_SUB 1024
#endif
#ifndef SDSJ_LAT_WARM
#define SDSJ_LAT_WARM 4000
#endif
constexpr int kLatSubBits = SDSJ_LAT_SUB;
constexpr int kLatWarm = SDSJ_LAT_WARM;
// Latency mode, multi-hypothesis (SDSJ_MH): every subsequence is decoded under each MCU phase
// (bpm lanes) from a short warm-up (kMhWarm bits) instead of one lane from kLatWarm bits; the phase
// whose entry matches its predecessor's exit is chosen afterwards (k_mh_select).
#ifndef SDSJ_MH
#define SDSJ_MH 1
#endif
#ifndef SDSJ_MH_WARM
#define SDSJ_MH_WARM 2048
#endif
constexpr int kMhWarm = SDSJ_MH_WARM;
constexpr int kMhMaxPhases = 10;  // bpm <= 10 (D_MAX_BLOCKS_IN_MCU)
// large images: ent_groups = ceil(bits / (kDecodeThreads x kGroupBits)) workgroups (<= kMaxEntGroups)
// share the subsequences, so one lane's serial decode stays near kGroupBits
#ifndef SDSJ_GROUP_BITS
#define SDSJ_GROUP_BITS 8192
#endif
constexpr int kGroupBits = SDSJ_GROUP_BITS;
constexpr int kMaxEntGroups = 16;
constexpr int kGroupShift = 4;  // (image << kGroupShift) | group in the group-task list
static_assert((1 << kGroupShift) >= kMaxEntGroups, "group index must fit the task encoding");
constexpr int kUPad = 128;            // zero bytes after each unstuffed stream (bit-reader prefetch)
constexpr int kUsTileBytes = 8192;    // unstuffing tile: 256 threads x 32 bytes
constexpr int kUsSerialTiles = 64;    // images of at most this many tiles are unstuffed by one workgroup
constexpr int kMaxSpan = 960;         // source columns per fused-resample tile (LDS row width)
constexpr int kRingDW = 3072;         // fused-resample ring (dwords): ring_rows x (3072 / ring_rows) columns
constexpr int kRingMaxRows = 16;      // vertical windows longer than this use the unfused path
#ifndef SDSJ_VTAPS_F
#define SDSJ_VTAPS_F 16
#endif
constexpr int kVTapsF = SDSJ_VTAPS_F;  // vertical taps the specialised fused kernels (k_rs420) stage; more: k_resample
// k_rs420<KT> with KT <= 7 horizontal taps (downscales up to ~3x with bilinear) carry a smaller ring and
// weight table (8 rows / 8 vertical taps: 6 KB less LDS, 5 workgroups per CU instead of 4; 6 with rs_span's
// narrower rows below); images whose
// vertical window needs more take k_resample
SDSJ_HD constexpr int rs_ring_rows(int kt) { return kt <= 7 ? 8 : kRingMaxRows; }
SDSJ_HD constexpr int rs_vtaps(int kt) { return kt <= 7 ? 8 : kVTapsF; }
SDSJ_HD constexpr int rs_ring_dw(int kt) { return kt <= 7 ? 8 * 256 : kRingDW; }
// ... and narrower staged rows: 768 source columns bring the 4:2:0 / 4:2:2 / gray kernels' LDS to
// 26.1 KB, 6 workgroups per CU instead of 5 (27.0 KB rows of 784 columns measured no faster: 5 still).
// KT <= 7 means ceil(support) <= 3, so a 256-column tile spans at most 256 x 3 + 2 x 3 + 4 = 778
// columns; plan_image halves the tile of the few images above 768 (bilinear scales in (2.97, 3]).
SDSJ_HD constexpr int rs_span(int kt) { return kt <= 7 ? 768 : kMaxSpan; }

// Raw DHT content (bits[1..16], huffval) -- jdmarker.c get_dht.
struct HuffSpec {
  uint8_t bits[17];
  uint8_t defined;
  uint8_t pad[14];
  uint8_t vals[256];
};

// Per-image table block in device scratch: quantisation tables (natural order) + the raw Huffman
// specs.  The entropy kernels derive their decode tables (jdhuff.c jpeg_make_d_derived_tbl plus a
// lookahead table) from the specs in LDS, in parallel.
struct ImgTables {
  uint16_t qt[4][64];
  uint8_t qt_defined[4];
  uint8_t pad[12];
  HuffSpec dc_spec[4], ac_spec[4];
};

// jdhuff.c jpeg_make_d_derived_tbl validation of a table the scan uses: the canonical code
// assignment must not overflow, and DC symbols must lie in 0..15 (JERR_BAD_HUFF_TABLE otherwise).
// Tables the scan does not use are never validated (start_pass_huff_decoder).
SDSJ_HD inline bool huff_table_ok(const HuffSpec& h, bool dc) {
  int code = 0, p = 0;
  for (int l = 1; l <= 16; l++) {
    code += h.bits[l];
    p += h.bits[l];
    if (code >= (1 << l)) return false;  // codes of length <= l overflow (the all-ones code is reserved)
    code <<= 1;
  }
  if (p > 256) return false;
  if (dc)
    for (int i = 0; i < p; i++)
      if (h.vals[i] > 15) return false;
  return true;
}

struct CompDesc {
  int32_t h, v, tq, td, ta;
  int32_t rh, rv;     // upsampling ratio hmax/h, vmax/v (1 or 2)
  int32_t dw, dh;     // downsampled width / height (jdinput.c)
  int32_t bw, bh;     // coded blocks per row / column (MCU padded when interleaved)
  int32_t pitch;      // plane row pitch in bytes (bw * 8)
  int64_t plane_off;  // byte offset of this plane inside the image's plane area
};

enum GeoMode : int32_t { kGeoResize = 0, kGeoIdentity = 1, kGeoZeros = 2 };

struct ImgDesc {
  int32_t status;
  int32_t width, height, ncomp;
  int32_t hmax, vmax, mcux, mcuy, bpm;
  int32_t restart_interval, nseg;
  int32_t saw_jfif, saw_adobe, adobe_transform;
  int32_t comp_id[kMaxComp];
  int64_t entropy_off;   // relative to the image's first byte
  int64_t entropy_len;   // bytes from entropy_off to the end of the input
  int64_t total_blocks;  // blocks in the scan (mcux*mcuy*bpm)
  int32_t blk_comp[kMaxBlocksPerMcu], blk_dx[kMaxBlocksPerMcu], blk_dy[kMaxBlocksPerMcu];
  CompDesc comp[kMaxComp];
  // pipeline geometry (functional.py:42-86, :118-147; Pillow ImagingResampleInner)
  int32_t geo;                  // GeoMode
  int32_t cx0, cy0, cw, ch;     // crop box (image coordinates)
  int32_t need_h, need_v;
  int32_t ksh, ksv;             // resampling kernel sizes
  int32_t yf, yl;               // crop rows [yf, yl) feeding the vertical pass
  int32_t src_y0, src_y1;       // image rows whose RGB is materialised
  int32_t src_x0, src_w;        // image columns whose RGB is materialised
  // entropy subsequences
  int32_t sub_bits;
  int32_t nsub_cap;
  // scratch layout (bytes from the scratch base)
  int64_t off_ustream, ustream_cap;
  int64_t off_seg;      // int32 [nseg + 2]: segment start bytes, then the stream length
  int64_t off_sub;      // SubState [nsub_cap]
  int64_t off_rec;      // SyncRec [nsub_cap][kRec]
  int64_t off_coef;     // int16 [total_blocks * 64], zigzag order within a block
  int64_t off_planes;
  int64_t off_rgb;      // uint8 RGB rows [src_y0, src_y1) x [src_x0, src_x0 + src_w)
  int64_t off_tmp;      // uint8 horizontal-pass output (yl - yf) x out_w x 3
  int64_t off_kh, off_kv;  // int32 resampling tables: [2 * out] bounds then [out * ks] coefficients
  int64_t need;         // total scratch bytes for this image
  int32_t nsub;         // actual subsequences (set by the entropy kernel)
  int32_t useg_found;   // segments found by the unstuff kernel
  int64_t ulen;         // unstuffed entropy bytes
  // entropy-kernel statistics (diagnostics): sync rounds, symbols decoded per phase
  int32_t sync_rounds;
  int32_t pad0;
  int64_t sym_spec, sym_sync, sym_write;
  // lane utilisation / phase timing diagnostics (s_memtime ticks, wave-loop iterations x 64)
  int64_t t_spec, t_sync, t_scan, t_write;
  int64_t it_spec, it_sync, it_write;
  // fused resample (sdsj_resample.hip): 1 when every tile of tile_w output columns needs at most
  // kMaxSpan source columns; 0 -> the unfused colour / h-pass / v-pass kernels
  int32_t fused, tile_w, ring_rows;
  int32_t rs_fast;  // > 0: tap count of the specialised 4:2:0 kernel (k_rs420<rs_fast>), 0: generic k_resample
  // k_resample phase ticks (s_memtime, summed over the image's workgroups; experiment builds only)
  int64_t t_rs[4];
  // entropy warm-up: a subsequence's speculative decode starts up to warm_bits before its first bit
  // (inside its segment) and takes the first block boundary at or after that bit as its entry
  int32_t warm_bits;
  // how the entropy-coded data ended (k_unstuff): the marker code (-1: end of input) and the
  // entropy-relative index of its last FF byte
  int32_t scan_end_code;
  int64_t scan_end_raw;
  int32_t rgb_pitch;   // pixels per row of the RGB rows the unfused passes read (frames: the frame width)
  int32_t ent_groups;  // workgroups sharing the image's subsequences in the spec / write passes
  // progressive JPEG (SOF2): every scan is decoded by k_prog from sos_pos (the first SOS segment's
  // length field) into the zeroed coefficient array; ProgTables at off_ptab hold its table state
  int32_t progressive;
  int32_t lat;  // latency-mode plan (kSmallBatch)
  int64_t sos_pos;
  int64_t off_ptab;
  // k_unstuff: per 8 KiB tile of the entropy-coded data, the counts its first pass found (UsTile)
  int64_t off_tiles;
  int32_t ntiles;
  int32_t rs_lay;  // chroma layout of the specialised fused kernel (RsLay) when rs_fast > 0
  int64_t plan_base;  // k_plan_scan: the image's first scratch byte (the offsets above are relative until k_plan_apply)
  // progressive block smoothing (jdcoefct.c smoothing_ok / decompress_smooth_data), set by k_prog at
  // EOI and applied by k_idct: smooth != 0 when some coefficient 1..9 is still inexact; per component
  // the scans' coef_bits for coefficients 0..9 after the last scan (sm_bits[0]) and before the
  // component's last scan (sm_bits[1], -1 = never coded), the latter for iMCU rows past sm_good (the
  // last scan ran out of data in row sm_good: jdcoefct.c last_good_iMCU_row)
  int32_t smooth, sm_good;
  int8_t sm_bits[2][kMaxComp][10];
  int8_t mh;  // latency mode: the multi-hypothesis speculative pass (k_entspec_mh) takes the image
  int8_t sm_pad[3];
  int32_t etab;  // k_enttab: the image whose EntTables it decodes with (itself, or image 0 of the lane when equal)
  int32_t etab_pad;
};

// One tile of k_unstuff's first pass: bytes it emits and split markers (RSTn, codes below SOF0) it
// holds before the tile's end, where its data ends (first other marker or the end of the input; -1:
// not in this tile) and that marker's code (-1: the end of the input).
struct UsTile {
  int32_t emit, split, end, code;
};

// Entropy decoder state of one subsequence (Weissenberger & Schmidt style self-synchronisation).
// Subsequence j owns the blocks whose DC symbol starts in [entry_j, exit_j): entry_j = the first
// block boundary at or after start_bit, exit_j = the first at or after end_bit.  State at a block
// boundary = (bit position p, MCU block index blk); bz packs (blk << 8) | z (z = 0 at entry/exit,
// non-zero only in a suspended sync stage).  "spec" = the speculative decode (warm-up from
// start_bit - warm_bits, then the subsequence), "cur" = the
// decode from the current entry estimate; after k_entsync, entry is verified and nblk_ex / dc_ex
// hold the exclusive (segmented) prefix of blocks and DC differences before the entry.
struct SubState {
  uint32_t start_bit, end_bit;
  uint32_t entry_p, cur_exit_p, spec_exit_p, new_exit_p, new_entry_p, res_p;
  uint16_t entry_bz, cur_exit_bz, spec_exit_bz, new_exit_bz, new_entry_bz, res_bz;
  int32_t cur_nblk, spec_nblk, new_nblk, nrec, res_nblk, res_ri;
  int32_t cur_dc[kMaxComp], spec_dc[kMaxComp], new_dc[kMaxComp], res_dc[kMaxComp], res_q[kMaxComp];
  int32_t nblk_ex, dc_ex[kMaxComp];
  int32_t first, seg;
  uint32_t lim_bit;  // end of the interval's data: bits at or beyond it read as zeros (jpeg_fill_bit_buffer)
  int32_t pad;
};

// Table state of the progressive decoder (k_prog), one per progressive image in scratch: the
// Huffman specs of the 4 DC and 4 AC slots as DHT segments define them (the scan's lookahead tables
// live in LDS, its canonical bounds here), the current DQT tables and which components have
// latched theirs (jdinput.c latch_quant_tables).
struct ProgTables {
  int32_t maxcode[8][17];  // the scan's derived tables (jdhuff.c jpeg_make_d_derived_tbl): [slot][l],
  int32_t valoff[8][17];   // l = 1..16, for codes longer than the LDS lookahead's 9 bits
  uint8_t vals[8][256];
  uint8_t bits[8][17];
  uint8_t defined[8];
  uint16_t qt[4][64];
  int32_t qt_defined[4];
  int32_t latched[kMaxComp];
};

// One block boundary met by the speculative decode (for early sync detection).
struct alignas(8) SyncRec {
  uint32_t p;       // bit position after the block's last symbol
  int16_t dc;       // DC difference decoded for that block
  uint8_t blk;      // MCU block index of the completed block
  uint8_t pad;
};

// Restart-interval table (scratch at off_seg).  Interval k = the k-th restart interval (the whole
// scan without DRI).  k_unstuff fills [lo[k], hi[k]) = the unstuffed bytes it decodes, chosen the way
// libjpeg's read_restart_marker / jpeg_resync_to_restart consume the markers it found (flag kEmpty:
// the marker was left unread, libjpeg decodes an empty segment).  k_entwrite sets vend[k] (blocks
// from vend[k] on stay zero: jdhuff.c insufficient_data) and kIns when the interval ran out of data.
constexpr int kMarkerSlack = 64;  // marker-list entries beyond one per restart
constexpr int32_t kSegEmpty = 1, kSegIns = 2;
struct SegView {
  int32_t *lo, *hi, *vend, *flag, *mk_out, *mk_raw, *mk_code;
  int cap;
};
SDSJ_HD inline int64_t seg_bytes(int nseg) { return ((int64_t)(nseg + 1) * 2 + (int64_t)nseg * 2 + (int64_t)(nseg + kMarkerSlack) * 3) * 4; }
SDSJ_HD inline SegView seg_view(uint8_t* base, int nseg) {
  int32_t* p = reinterpret_cast<int32_t*>(base);
  SegView v;
  v.cap = nseg + kMarkerSlack;
  v.lo = p;
  v.hi = v.lo + nseg + 1;
  v.vend = v.hi + nseg + 1;
  v.flag = v.vend + nseg;
  v.mk_out = v.flag + nseg;
  v.mk_raw = v.mk_out + v.cap;
  v.mk_code = v.mk_raw + v.cap;
  return v;
}

// Work routes: k_plan sorts the batch's images into per-variant lists.  A variant kernel maps its
// workgroups to its own list (the main variants: one workgroup column per entry, the surplus exits
// at once; the rare unfused path: a small grid striding over its list), so no workgroup is spent
// on an image another variant decodes.  Layout of the engine's route buffer (int32):
// [counts (kRouteSlots)][kNumRoutes lists of cap entries].
enum Route : int32_t {
  kRtUnfused = 0,  // k_color -> k_hpass -> k_vpass
  kRtGen0,         // k_resample<0>: any horizontal tap count (coefficients from the table)
  kRtGen1,         // k_resample<1>: no horizontal pass
  kRtGen3, kRtGen5, kRtGen7, kRtGen9, kRtGen11,  // k_resample<KT>
  kRtF,                           // k_rs420<KT, LAY>: 4 layouts x 5 tap counts from here (rs_route)
  kRtFLast = kRtF + 19,
  kRtEnt10, kRtEnt11,             // entropy kernels by lookahead width
  kRtEnt11M,                      // LB = 11 images decoded by several workgroups (ent_groups > 1)
  kRtProg,                        // progressive images (k_prog)
  kRtEnt11G,                      // (count only) (image, group) tasks of the kRtEnt11M images: group_tasks()
  kRtUsSmall, kRtUsBig,           // unstuffing: k_us_serial / the tile-parallel passes (kUsSerialTiles)
  kNumRoutes
};
constexpr int kRouteSlots = 48;  // counts [0, kNumRoutes), the rest zero
static_assert(kNumRoutes <= kRouteSlots, "route counts must fit the count slots");
SDSJ_HD inline const int32_t* route_list(const int32_t* routes, int cap, int r) { return routes + kRouteSlots + r * cap; }
// After the lists: one entry (image << kGroupShift | group) per workgroup task of a multi-group image, so the
// spec / write passes give every (image, group) its own workgroup (count in routes[kRtEnt11G]).
SDSJ_HD inline int32_t* group_tasks(int32_t* routes, int cap) { return routes + kRouteSlots + (int64_t)kNumRoutes * cap; }
SDSJ_HD inline int64_t route_ints(int cap) { return kRouteSlots + (int64_t)(kNumRoutes + kMaxEntGroups) * cap; }
// chroma layouts of the specialised fused resample (sdsj_resample420.hip)
enum RsLay : int32_t { kRs420 = 0, kRs422 = 1, kRs444 = 2, kRsGray = 3 };
SDSJ_HD inline int rs_route(int lay, int kt) { return kRtF + lay * 5 + (kt - 3) / 2; }
constexpr int kRsfEntries = 4096;  // workgroup columns of a specialised-resample launch (they stride over its list)
// generic fused resample route of an image whose horizontal pass has kt taps (1: none)
SDSJ_HD inline int gen_route(int kt) {
  return kt == 1 ? kRtGen1 : (kt >= 3 && kt <= 11 && (kt & 1) ? kRtGen3 + (kt - 3) / 2 : kRtGen0);
}

SDSJ_HD inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
SDSJ_HD inline int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

// jutils.c jpeg_natural_order (+16 guard entries)
#if defined(__HIPCC__)
__host__ __device__
#endif
inline int natural_order(int k) {
  constexpr int8_t t[80] = {
      0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
      41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
      30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63,
      63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};
  return t[k];
}

// Copies DHT values / DQT entries as the parser meets them (host probe and host planning).  The
// device parser substitutes a sink that records the copies and runs them on all lanes.
template <class Reader>
struct CopySink {
  const Reader& rd;
  SDSJ_HD void dht(HuffSpec* h, int64_t src, int cnt) const {
    for (int q = 0; q < 256; q++) h->vals[q] = q < cnt ? (uint8_t)rd(src + q) : 0;
  }
  SDSJ_HD void dqt(uint16_t* qt, int pq, int64_t src) const {
    for (int q = 0; q < 64; q++)
      qt[natural_order(q)] = (uint16_t)(pq ? ((rd(src + 2 * q) << 8) | rd(src + 2 * q + 1)) : rd(src + q));
  }
};

// Parses markers up to the first SOS (jdmarker.c subset).  `rd(i)` returns byte i; `t` must be
// non-null (no null checks: on the device it points into LDS).  Bulk table bytes go through `sink`.
template <class Reader, class Sink>
SDSJ_HD int parse_headers(const Reader& rd, int64_t n, ImgDesc* d, ImgTables* t, const Sink& sink) {
  d->status = SDSJ_OK;
  d->width = d->height = d->ncomp = 0;
  d->progressive = 0;
  d->sos_pos = 0;
  d->restart_interval = 0;
  d->saw_jfif = d->saw_adobe = d->adobe_transform = 0;
  for (int q = 0; q < 4; q++) {
    t->qt_defined[q] = 0;
    t->dc_spec[q].defined = 0;
    t->ac_spec[q].defined = 0;
  }
  // not a JPEG stream (PNG, WebP, GIF, ... every other IMAGE_EXT format PIL opens, sds/structs.py:42):
  // outside this path, reported as unsupported; a JPEG cut inside its first marker is corrupt
  if (n < 2 || rd(0) != 0xFF || rd(1) != 0xD8) return SDSJ_UNSUPPORTED;
  if (n < 4) return SDSJ_CORRUPT;
  int64_t i = 2;
  bool saw_sof = false;
  for (;;) {
    while (i < n && rd(i) != 0xFF) i++;  // next_marker: skip garbage
    while (i < n && rd(i) == 0xFF) i++;  // and fill bytes
    if (i >= n) return SDSJ_CORRUPT;
    int m = rd(i++);
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
    if (m == 0xD9) return SDSJ_CORRUPT;  // EOI before SOS
    if (i + 2 > n) return SDSJ_CORRUPT;
    int len = (rd(i) << 8) | rd(i + 1);
    if (len < 2 || i + len > n) return SDSJ_CORRUPT;
    int64_t s = i + 2;
    int sl = len - 2;
    switch (m) {
      case 0xC0:
      case 0xC1:
      case 0xC2: {  // baseline, extended sequential, progressive (Huffman)
        if (saw_sof) return SDSJ_CORRUPT;
        saw_sof = true;
        d->progressive = m == 0xC2;
        if (sl < 6) return SDSJ_CORRUPT;
        if (rd(s) != 8) return SDSJ_UNSUPPORTED;
        d->height = (rd(s + 1) << 8) | rd(s + 2);
        d->width = (rd(s + 3) << 8) | rd(s + 4);
        d->ncomp = rd(s + 5);
        if (d->height == 0 || d->width == 0) return SDSJ_UNSUPPORTED;  // DNL
        if (sl != 6 + 3 * d->ncomp) return SDSJ_CORRUPT;                // get_sof: JERR_BAD_LENGTH
        if (d->ncomp != 1 && d->ncomp != 3) return SDSJ_UNSUPPORTED;
        d->hmax = d->vmax = 1;
        for (int c = 0; c < d->ncomp; c++) {
          CompDesc& cp = d->comp[c];
          d->comp_id[c] = rd(s + 6 + 3 * c);
          int hv = rd(s + 7 + 3 * c);
          cp.h = hv >> 4;
          cp.v = hv & 15;
          cp.tq = rd(s + 8 + 3 * c);
          if (cp.h < 1 || cp.h > 4 || cp.v < 1 || cp.v > 4 || cp.tq > 3) return SDSJ_CORRUPT;
          if (cp.h > d->hmax) d->hmax = cp.h;
          if (cp.v > d->vmax) d->vmax = cp.v;
        }
        break;
      }
      case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9:
      case 0xCA: case 0xCB: case 0xCD: case 0xCE: case 0xCF:
        return SDSJ_UNSUPPORTED;
      case 0xC4: {  // DHT
        int k = 0;
        while (k < sl) {
          if (k + 17 > sl) return SDSJ_CORRUPT;
          int tc = rd(s + k) >> 4, th = rd(s + k) & 15;
          if (tc > 1 || th > 3) return SDSJ_CORRUPT;
          int cnt = 0;
          HuffSpec* h = tc ? &t->ac_spec[th] : &t->dc_spec[th];
          for (int l = 1; l <= 16; l++) {
            int b = rd(s + k + l);
            cnt += b;
            h->bits[l] = (uint8_t)b;
          }
          if (cnt > 256 || k + 17 + cnt > sl) return SDSJ_CORRUPT;
          h->bits[0] = 0;
          sink.dht(h, s + k + 17, cnt);
          h->defined = 1;
          k += 17 + cnt;
        }
        break;
      }
      case 0xDB: {  // DQT
        int k = 0;
        while (k < sl) {
          int pq = rd(s + k) >> 4, tq = rd(s + k) & 15;
          if (tq > 3 || pq > 1) return SDSJ_CORRUPT;
          int need = 1 + 64 * (pq ? 2 : 1);
          if (k + need > sl) return SDSJ_CORRUPT;
          sink.dqt(t->qt[tq], pq, s + k + 1);
          t->qt_defined[tq] = 1;
          k += need;
        }
        break;
      }
      case 0xDD:
        if (sl < 2) return SDSJ_CORRUPT;
        d->restart_interval = (rd(s) << 8) | rd(s + 1);
        break;
      case 0xE0:
        if (sl >= 5 && rd(s) == 'J' && rd(s + 1) == 'F' && rd(s + 2) == 'I' && rd(s + 3) == 'F' && rd(s + 4) == 0)
          d->saw_jfif = 1;
        break;
      case 0xEE:
        if (sl >= 12 && rd(s) == 'A' && rd(s + 1) == 'd' && rd(s + 2) == 'o' && rd(s + 3) == 'b' && rd(s + 4) == 'e') {
          d->saw_adobe = 1;
          d->adobe_transform = rd(s + 11);
        }
        break;
      case 0xDC:
        return SDSJ_UNSUPPORTED;  // DNL
      case 0xDA: {  // SOS
        if (!saw_sof || sl < 1) return SDSJ_CORRUPT;
        int ns = rd(s);
        if (ns < 1 || ns > 4 || sl != 2 * ns + 4) return SDSJ_CORRUPT;  // get_sos: JERR_BAD_LENGTH
        if (d->progressive) {  // every scan is parsed by k_prog
          d->sos_pos = i;
          d->entropy_off = i + len;
          d->entropy_len = n - d->entropy_off;
          return SDSJ_OK;
        }
        if (ns != d->ncomp) return SDSJ_UNSUPPORTED;  // multi-scan sequential
        for (int q = 0; q < ns; q++) {
          int cid = rd(s + 1 + 2 * q);
          int c = 0;
          while (c < d->ncomp && d->comp_id[c] != cid) c++;
          if (c != q) return SDSJ_UNSUPPORTED;
          int tt = rd(s + 2 + 2 * q);
          d->comp[c].td = tt >> 4;
          d->comp[c].ta = tt & 15;
          if (d->comp[c].td > 3 || d->comp[c].ta > 3) return SDSJ_CORRUPT;
        }
        int ss = rd(s + 1 + 2 * ns), se = rd(s + 2 + 2 * ns), ahal = rd(s + 3 + 2 * ns);
        if (ss != 0 || se != 63 || ahal != 0) return SDSJ_UNSUPPORTED;
        d->entropy_off = i + len;
        d->entropy_len = n - d->entropy_off;
        return SDSJ_OK;
      }
      default:
        break;
    }
    i += len;
  }
}

// Colour space (jdapimin.c default_decompress_parms) and geometry (jdinput.c).
SDSJ_HD inline int setup_geometry(ImgDesc* d, const ImgTables* t) {
  if (d->ncomp == 3) {
    if (!d->saw_jfif) {
      if (d->saw_adobe) {
        if (d->adobe_transform == 0) return SDSJ_UNSUPPORTED;  // Adobe RGB
      } else if (d->comp_id[0] == 82 && d->comp_id[1] == 71 && d->comp_id[2] == 66) {
        return SDSJ_UNSUPPORTED;  // 'R','G','B' component ids
      }
    }
  }
  int bpm = 0;
  for (int c = 0; c < d->ncomp; c++) {
    CompDesc& cp = d->comp[c];
    if (d->hmax % cp.h || d->vmax % cp.v) return SDSJ_UNSUPPORTED;
    cp.rh = d->hmax / cp.h;
    cp.rv = d->vmax / cp.v;
    if (cp.rh > 2 || cp.rv > 2) return SDSJ_UNSUPPORTED;
    cp.dw = ceil_div(d->width * cp.h, d->hmax);
    cp.dh = ceil_div(d->height * cp.v, d->vmax);
    if (d->progressive) continue;  // tables are checked per scan (k_prog)
    if (!t->qt_defined[cp.tq]) return SDSJ_CORRUPT;
    if (!t->dc_spec[cp.td].defined || !t->ac_spec[cp.ta].defined) return SDSJ_CORRUPT;
  }
  if (d->ncomp == 1) {
    CompDesc& cp = d->comp[0];
    cp.bw = ceil_div(cp.dw, 8);
    cp.bh = ceil_div(cp.dh, 8);
    d->mcux = cp.bw;
    d->mcuy = cp.bh;
    d->bpm = 1;
    d->blk_comp[0] = 0;
    d->blk_dx[0] = 0;
    d->blk_dy[0] = 0;
  } else {
    d->mcux = ceil_div(d->width, 8 * d->hmax);
    d->mcuy = ceil_div(d->height, 8 * d->vmax);
    for (int c = 0; c < d->ncomp; c++) {
      d->comp[c].bw = d->mcux * d->comp[c].h;
      d->comp[c].bh = d->mcuy * d->comp[c].v;
      for (int v = 0; v < d->comp[c].v; v++)
        for (int h = 0; h < d->comp[c].h; h++) {
          if (bpm >= kMaxBlocksPerMcu) return SDSJ_CORRUPT;
          d->blk_comp[bpm] = c;
          d->blk_dx[bpm] = h;
          d->blk_dy[bpm] = v;
          bpm++;
        }
    }
    d->bpm = bpm;
  }
  int64_t plane = 0;
  for (int c = 0; c < d->ncomp; c++) {
    CompDesc& cp = d->comp[c];
    cp.pitch = cp.bw * 8;
    cp.plane_off = plane;
    plane += align_up((int64_t)cp.pitch * cp.bh * 8, 256);
  }
  d->total_blocks = (int64_t)d->mcux * d->mcuy * d->bpm;
  if (d->total_blocks >= (int64_t)1 << 24) return SDSJ_UNSUPPORTED;  // > ~700 MP (block indices are 24-bit)
  int64_t mcus = (int64_t)d->mcux * d->mcuy;
  d->nseg = d->restart_interval ? (int32_t)((mcus + d->restart_interval - 1) / d->restart_interval) : 1;
  return SDSJ_OK;
}

// functional.py:118-140 crop_to_aspect_ratio (Python doubles, int() truncation, floor-div).
SDSJ_HD inline void crop_box(int w, int h, int out_h, int out_w, int* x0, int* y0, int* cw, int* ch) {
  double cur = (double)w / (double)h;
  double tgt = (double)out_w / (double)out_h;
  if (cur > tgt) {
    int nw = (int)((double)h * tgt);
    *x0 = (w - nw) / 2;
    *y0 = 0;
    *cw = nw;
    *ch = h;
  } else {
    int nh = (int)((double)w / tgt);
    *x0 = 0;
    *y0 = (h - nh) / 2;
    *cw = w;
    *ch = nh;
  }
}

// Pillow Resample.c precompute_coeffs: kernel size for a 1-D resample in -> out.
SDSJ_HD inline int resample_ksize(int in_size, int out_size, double filter_support) {
  double scale = (double)in_size / out_size;
  double fs = scale < 1.0 ? 1.0 : scale;
  double support = filter_support * fs;
  int c = (int)support;
  if ((double)c < support) c++;  // ceil
  return c * 2 + 1;
}

// Pillow _imaging.c _resize, NEAREST branch -> ImagingTransform(AFFINE, fill = 1) -> Geometry.c
// ImagingScaleAffine: output index xx samples source index COORD(xo), xo = scale * 0.5 advanced by
// `xo += scale` per index (a running double sum, kept as such: (xx + 0.5) * scale can round
// differently), COORD(v) = v < 0 ? -1 : (int)v; -1 = outside [0, in): the pixel keeps the fill value 0.
SDSJ_HD inline int nearest_src(int in_size, int out_size, int xx) {
  const double a = (double)in_size / out_size;
  double xo = 0.0 + a * 0.5;
  for (int i = 0; i < xx; i++) xo += a;
  const int xin = xo < 0.0 ? -1 : (int)xo;
  return (xin >= 0 && xin < in_size) ? xin : -1;
}

// The blocks of component c the colour / resample passes read -- k_idct transforms exactly these and
// k_entwrite stores only these: the source rectangle [src_x0, src_x0 + src_w) x [src_y0, src_y1) in the
// component's sampling, widened by one sample for the fancy upsampling's neighbours, as inclusive block
// bounds.  False when the crop is empty (nothing is read).
SDSJ_HD inline bool comp_block_rect(const ImgDesc& d, int c, int& bx0, int& bx1, int& by0, int& by1) {
  const int x0 = d.src_x0, x1 = d.src_x0 + d.src_w, y0 = d.src_y0, y1 = d.src_y1;
  const CompDesc& cd = d.comp[c];
  const int rh = d.ncomp == 1 ? 1 : d.hmax / cd.h, rv = d.ncomp == 1 ? 1 : d.vmax / cd.v;
  int cx0 = x0 / rh - 1, cx1 = (x1 - 1) / rh + 1, cy0 = y0 / rv - 1, cy1 = (y1 - 1) / rv + 1;
  cx0 = cx0 < 0 ? 0 : cx0;
  cy0 = cy0 < 0 ? 0 : cy0;
  cx1 = cx1 > cd.bw * 8 - 1 ? cd.bw * 8 - 1 : cx1;
  cy1 = cy1 > cd.bh * 8 - 1 ? cd.bh * 8 - 1 : cy1;
  bx0 = cx0 >> 3;
  bx1 = cx1 >> 3;
  by0 = cy0 >> 3;
  by1 = cy1 >> 3;
  return x1 > x0 && y1 > y0 && d.geo != kGeoZeros;
}

SDSJ_HD inline double filter_support(int filter) {
  switch (filter) {
    case SDSJ_FILTER_BOX: return 0.5;
    case SDSJ_FILTER_BILINEAR: return 1.0;
    case SDSJ_FILTER_HAMMING: return 1.0;
    case SDSJ_FILTER_BICUBIC: return 2.0;
    default: return 3.0;
  }
}

}  // namespace sdsj
