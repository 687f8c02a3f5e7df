// sdsj_entropy.hip -- parallel Huffman decoding of baseline JPEG scans on gfx950.
//
// Restates libjpeg-turbo jdhuff.c decode_mcu (the decoder Pillow runs for
// sds/transforms/functional.py:100) with one image per 256-thread workgroup and the entropy
// segment split into subsequences decoded in parallel (self-synchronisation, after Weissenberger &
// Schmidt, "Massively Parallel Huffman Decoding on GPUs"):
//
//   k_entsync   1. speculative pass: subsequence j decodes from its first bit assuming (block 0,
//                  DC) and records its block boundaries (SyncRec);
//               2. sync: every j whose entry state differs from the exit state of j-1 re-decodes
//                  from that state and stops at the first boundary where it meets a record of its
//                  speculative pass (the paths have merged, the rest of that result is exact).  The
//                  re-decodes run as work stages with a doubling symbol budget: unfinished tasks
//                  save their state and are packed into the fewest waves for the next stage, so the
//                  few long re-decodes do not hold every wave of the workgroup.  Rounds repeat
//                  until every entry equals its predecessor's exit (Jacobi fixed point);
//               3. segmented exclusive scan of (blocks completed, DC differences) -> every
//                  subsequence's first block index and DC predictors (prediction resets at RSTn).
//   k_entwrite  4. verified decode: each lane assembles its current 8x8 block in LDS (zigzag order,
//                  positions past 63 at 63 like jpeg_natural_order's guard entries: k_idct reads
//                  zigzag blocks); the wave flushes completed blocks cooperatively as 128-byte stores.
//                  A block belongs to the subsequence in which its DC symbol starts (the owner
//                  decodes past its end to finish it).
//
// Symbol decoding: 2^LB-entry lookup of (code length, size, run) -- LB = 11 for images using at
// most 4 Huffman tables, LB = 10 otherwise (two kernel variants, each skips the other's images)
// -- and the canonical maxcode search of jpeg_huff_decode for longer codes.  The MCU position
// (block -> table slots, component) comes from per-image packed registers, so the per-symbol path
// is branch-free apart from the rare long-code search and the refill.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "sdsj_common.h"
#include "sdsj_kernels.h"

namespace sdsj {

#ifndef SDSJ_STATS
#define SDSJ_STATS 0  // 1: per-image symbol / tick / lane-utilisation statistics (tools/entropy_stats.py builds)
#endif
constexpr bool kStats = SDSJ_STATS != 0;

constexpr int kEntThreads = kDecodeThreads;
constexpr int kLutEntries = 1 << 13;  // LDS lookup capacity: 4 tables x 2^11 or 8 x 2^10
constexpr int kStageStride = 64;      // int16 per lane staging block (one 128-byte block)
template <int NT>
constexpr int max_tasks() { return 4 * NT; }  // sync tasks per round (more: picked up by the next round)
// k_entsync is latency-bound (a few serial re-decodes per image): one wave per image keeps more
// images in flight per CU than a 4-wave workgroup would (the LDS tables bound both)
constexpr int kSyncThreads = 64;
constexpr int kMaxSlots = 2 * kMaxComp;  // a DC and an AC table per component at most

// What a symbol adds to its block's zigzag position k (decode_mcu's k loop): 1 for a DC symbol, r + 1
// for an AC value or ZRL (r = 15), 64 for EOB -- a block ends when k passes 63.  The speculative and the
// write passes' tables carry it per entry, so a block end is one compare.
__device__ __forceinline__ uint32_t write_adv(bool ac, uint32_t s, uint32_t r) {
  return !ac ? 1u : ((s == 0 && r != 15) ? 64u : r + 1u);
}
// A decode-table entry (len | size << 4 | run << 8) in the write and sync passes' format:
// len | size << 4 | advance << 8.
__device__ __forceinline__ uint32_t write_entry(uint32_t e, bool ac) {
  const uint32_t l = e & 15, sz = (e >> 4) & 15, r = (e >> 8) & 15;
  return l == 0 ? 0u : (l | (sz << 4) | (write_adv(ac, sz, r) << 8));
}

// ------------------------------------------------------------------------------------------
// Per-image decode tables in LDS.
// ------------------------------------------------------------------------------------------
// Canonical bounds, symbols and the MCU context: shared by every table layout below.
struct TabCommon {
  int32_t maxcode[kMaxSlots][18];
  int32_t valoff[kMaxSlots][18];
  uint8_t vals[kMaxSlots][256];
  int32_t slot_src[kMaxSlots];  // (kind << 2) | id of the table in each slot (kind 0 = DC, 1 = AC)
  int32_t nslots;
  uint32_t pk_dc[2], pk_ac[2], pk_c;  // per MCU block: DC slot, AC slot (4 bits each), component (2)
  uint32_t pad[4];
};
static_assert(sizeof(TabCommon) % 16 == 0, "tables are copied in 16-byte units");

// Multi-symbol lookahead (the LB = 11 images' speculative pass): kMW bits per slot, 32-bit entries.
//   bits 0-11  the single symbol whose code fits kMW bits: len | size << 4 | run << 8 (0: a longer code)
//   bits 12-16 AC slots: the bits a group of >= 2 consecutive symbols consumes (codes and extra bits)
//              when every code of the group lies in the window; 0: no group
//   bits 17-23 the group's coefficient advance (sum of run + 1 over value symbols, 16 per ZRL), + 1
//              when it ends with an EOB: the group applies at block position z iff z + this <= 64,
//              so a block can only end at a group's last symbol
//   bit  24    the group ends with an EOB
//   bits 25-31 the single symbol's advance of the block position (write_adv)
// Groups skip the values, so only passes that need no AC values (warm-up, speculative) use them.
constexpr int kMW = 10;
constexpr int kMSlots = 4;  // LB = 11 images have at most 4 slots

// LDS copy with the single-symbol LUT (LB = 10 images; a prefix of EntTables).
struct LutTables : TabCommon {
  static constexpr bool kTwoLevel = false;
  uint16_t lut[kLutEntries];
};

static_assert(sizeof(LutTables) % 16 == 0, "LutTables is copied in 16-byte units");

// What k_enttab writes per image (HBM).
struct EntTables : LutTables {
  uint32_t mlut[kMSlots << kMW];
};
static_assert(sizeof(EntTables) % 16 == 0, "EntTables is copied in 16-byte units");

// The speculative pass's LDS copy for LB = 11 images: the multi-symbol table instead of the LUT.
struct SpecTables : TabCommon {
  static constexpr bool kTwoLevel = false;
  uint32_t mlut[kMSlots << kMW];
};

// Is this image decoded by the LB variant?  (LB = 11 when its tables fit 4 slots, else LB = 10.)
template <int LB>
__device__ __forceinline__ bool variant_owns(int ns) {
  return LB == 11 ? (ns << 11) <= kLutEntries : (ns << 11) > kLutEntries && (ns << 10) <= kLutEntries;
}

// k_enttab: one workgroup per image builds its decode tables once into HBM; every entropy kernel
// then copies the image's EntTables into LDS with 16-byte loads (one round trip) instead of
// rebuilding them.
__global__ void __launch_bounds__(kEntThreads) k_enttab(ImgDesc* __restrict__ descs,
                                                       const ImgTables* __restrict__ tables, EntTables* __restrict__ out) {
  ImgDesc* d = &descs[blockIdx.x];
  if (d->status != SDSJ_OK || d->progressive) return;
  const ImgTables* tb = &tables[blockIdx.x];
  __shared__ LutTables T;  // (the multi-symbol table goes straight to HBM: nothing here reads it back)
  __shared__ int32_t lim[kMaxSlots][12];
  const int t = threadIdx.x;
  if (blockIdx.x > 0) {
    // Shared tables: an image whose table inputs equal image 0's (same components' table selectors,
    // same block -> component map, byte-equal Huffman specs of the tables it uses) decodes with image
    // 0's EntTables (most JPEGs carry the standard tables), so only image 0 builds them.  Image 0's
    // status is read here as its own workgroup reads it (this kernel changes no status).
    const ImgDesc* a = &descs[0];
    const ImgTables* ta = &tables[0];
    __shared__ int same;
    const bool cand = a->status == SDSJ_OK && !a->progressive && a->ncomp == d->ncomp && a->bpm == d->bpm;
    if (t == 0) same = cand ? 1 : 0;
    __syncthreads();
    if (cand) {
      bool diff = false;
      if (t < d->ncomp) diff |= a->comp[t].td != d->comp[t].td || a->comp[t].ta != d->comp[t].ta;
      if (t < d->bpm) diff |= a->blk_comp[t] != d->blk_comp[t];
      // bits[0..16] and vals[0..255] of each component's DC and AC spec (273 bytes each)
      for (int i = t; i < 2 * d->ncomp * 273; i += kEntThreads) {
        const int c = i / (2 * 273), r = i % (2 * 273), ac = r >= 273, k = ac ? r - 273 : r;
        const HuffSpec& ha = ac ? ta->ac_spec[d->comp[c].ta & 3] : ta->dc_spec[d->comp[c].td & 3];
        const HuffSpec& hd = ac ? tb->ac_spec[d->comp[c].ta & 3] : tb->dc_spec[d->comp[c].td & 3];
        diff |= k < 17 ? ha.bits[k] != hd.bits[k] : ha.vals[k - 17] != hd.vals[k - 17];
      }
      if (diff) same = 0;  // (benign race: every writer stores 0)
    }
    __syncthreads();
    if (same) {
      if (t == 0) d->etab = 0;
      return;
    }
  }
  if (t == 0) d->etab = blockIdx.x;
  if (t == 0) {
    int ns = 0;
    auto slot_of = [&](int key) {
      for (int q = 0; q < ns; q++)
        if (T.slot_src[q] == key) return q;
      T.slot_src[ns] = key;
      return ns++;
    };
    int dcs[kMaxComp], acs[kMaxComp];
    for (int c = 0; c < d->ncomp; c++) {
      dcs[c] = slot_of(d->comp[c].td);
      acs[c] = slot_of(4 | d->comp[c].ta);
    }
    T.nslots = ns;
    uint64_t pdc = 0, pac = 0;
    uint32_t pc = 0;
    for (int b = 0; b < d->bpm; b++) {
      const int c = d->blk_comp[b];
      pdc |= (uint64_t)dcs[c] << (4 * b);
      pac |= (uint64_t)acs[c] << (4 * b);
      pc |= (uint32_t)c << (2 * b);
    }
    T.pk_dc[0] = (uint32_t)pdc;
    T.pk_dc[1] = (uint32_t)(pdc >> 32);
    T.pk_ac[0] = (uint32_t)pac;
    T.pk_ac[1] = (uint32_t)(pac >> 32);
    T.pk_c = pc;
    T.pad[0] = T.pad[1] = T.pad[2] = T.pad[3] = 0;
  }
  __syncthreads();
  const int ns = T.nslots;
  const int lb = (ns << 11) <= kLutEntries ? 11 : 10;  // the variant that will decode this image
  // canonical code bounds per slot (jdhuff.c jpeg_make_d_derived_tbl: maxcode / valoffset), and
  // lim[l] = (end of the length-l codes) << (lb - l): the lookahead indices below lim[l] and at or
  // above lim[l-1] hold length-l codes (canonical codes make lim non-decreasing in l)
  if (t < ns) {
    const int key = T.slot_src[t];
    const HuffSpec& h = (key & 4) ? tb->ac_spec[key & 3] : tb->dc_spec[key & 3];
    int code = 0, p = 0;
    for (int l = 1; l <= 16; l++) {
      const int cnt = h.bits[l];
      T.maxcode[t][l] = cnt ? code + cnt - 1 : -1;
      T.valoff[t][l] = cnt ? p - code : 0;
      if (l <= lb) lim[t][l] = (code + cnt) << (lb - l);
      p += cnt;
      code = (code + cnt) << 1;
    }
    T.maxcode[t][0] = -1;
    T.valoff[t][0] = 0;
    T.maxcode[t][17] = 0xFFFFF;  // sentinel: the search stops at length 17 (bad code)
    T.valoff[t][17] = 0;
    if (lb == 10) lim[t][11] = 1 << 30;
  }
  for (int i = t; i < ns * 256; i += kEntThreads) {
    const int q = i >> 8, k = i & 255;
    const int key = T.slot_src[q];
    T.vals[q][k] = (key & 4) ? tb->ac_spec[key & 3].vals[k] : tb->dc_spec[key & 3].vals[k];
  }
  __syncthreads();
  // 2^lb lookahead entries (len | size << 4 | run << 8); codes longer than lb bits (entry 0) take
  // the canonical search in decode_sym
  for (int i = t; i < (ns << lb); i += kEntThreads) {
    const int q = i >> lb, k = i & ((1 << lb) - 1);
    int l = 1;
#pragma unroll
    for (int m = 1; m <= 11; m++) l += k >= lim[q][m] ? 1 : 0;
    uint16_t e = 0;
    if (l <= lb) {
      const bool dc = (T.slot_src[q] & 4) == 0;
      const int sym = T.vals[q][((k >> (lb - l)) + T.valoff[q][l]) & 0xFF];
      const int sz = dc ? sym : (sym & 15), run = dc ? 0 : (sym >> 4);
      e = sz > 15 ? (uint16_t)0 : (uint16_t)(l | (sz << 4) | (run << 8));
    }
    T.lut[i] = e;
  }
  __syncthreads();
  if (lb == 11) {
    // the multi-symbol table (kMW bits): the single entry of codes <= kMW bits, and for AC slots the
    // group of symbols whose codes lie in the window, walked with the LUT above (each step reads
    // the window's remaining bits, zero-padded, so a code of <= kMW - used bits is decided by real bits)
    for (int i = t; i < (ns << kMW); i += kEntThreads) {
      const int q = i >> kMW, k = i & ((1 << kMW) - 1);
      const uint32_t e1 = T.lut[(q << 11) + (k << 1)];
      uint32_t e = (e1 & 15) <= kMW ? e1 : 0u;
      if (e & 15) e |= write_adv((T.slot_src[q] & 4) != 0, (e >> 4) & 15, (e >> 8) & 15) << 25;
      if (T.slot_src[q] & 4) {
        int used = 0, dz = 0, n = 0, eob = 0;
        while (used < kMW) {
          const uint32_t f = T.lut[(q << 11) + (((k << used) & ((1 << kMW) - 1)) << 1)];
          const int l = f & 15, s = (f >> 4) & 15, r = (f >> 8) & 15;
          if (l == 0 || l > kMW - used) break;
          if (s == 0 && r != 15) {  // EOB ends the group (and the block)
            eob = 1;
            used += l;
            n++;
            break;
          }
          const int step = s == 0 ? 16 : r + 1;
          if (dz + step > 63) break;
          used += l + s;
          dz += step;
          n++;
        }
        if (n >= 2) e |= ((uint32_t)used << 12) | ((uint32_t)(dz + eob) << 17) | ((uint32_t)eob << 24);
      }
      out[blockIdx.x].mlut[i] = e;
    }
  }
  const uint4* src = reinterpret_cast<const uint4*>(&T);
  uint4* dst = reinterpret_cast<uint4*>(&out[blockIdx.x]);
  for (int i = t; i < (int)(sizeof(LutTables) / 16); i += kEntThreads) dst[i] = src[i];
}

// The image's tables into LDS (the LUT part the variant uses, and everything after it).
template <int LB>
__device__ __forceinline__ int load_tables(LutTables& T, const EntTables* g) {
  const uint4* src = reinterpret_cast<const uint4*>(g);
  uint4* dst = reinterpret_cast<uint4*>(&T);
  constexpr int kCom16 = (int)(sizeof(TabCommon) / 16);
  const int ns = g->nslots;
  const int used16 = kCom16 + (variant_owns<LB>(ns) ? ((ns << LB) * 2 + 15) / 16 : 0);
  for (int i = threadIdx.x; i < used16; i += blockDim.x) dst[i] = src[i];
  __syncthreads();
  return ns;
}

// The speculative pass's tables for LB = 11 images: the common part and the multi-symbol table.
__device__ __forceinline__ int load_tables(SpecTables& T, const EntTables* g) {
  const uint4* src = reinterpret_cast<const uint4*>(g);
  const uint4* msrc = reinterpret_cast<const uint4*>(g->mlut);
  uint4* dst = reinterpret_cast<uint4*>(&T);
  uint4* mdst = reinterpret_cast<uint4*>(T.mlut);
  constexpr int kCom16 = (int)(sizeof(TabCommon) / 16);
  const int ns = g->nslots;
  const int m16 = variant_owns<11>(ns) ? (ns << kMW) * 4 / 16 : 0;
  for (int i = threadIdx.x; i < kCom16 + m16; i += blockDim.x) {
    if (i < kCom16) dst[i] = src[i];
    else mdst[i - kCom16] = msrc[i - kCom16];
  }
  __syncthreads();
  return ns;
}

// k_entsync's tables: a 2^9-entry lookahead per slot (codes of at most 9 bits; longer ones take the
// canonical search) so that about 10 KB of LDS per image lets ~15 images share a CU -- its few
// lanes per image are latency-bound, and more images in flight hide that latency.
constexpr int kSyncLB = 9;
struct SyncTables {
  static constexpr bool kTwoLevel = false;
  uint16_t lut[kMaxSlots << kSyncLB];
  int32_t maxcode[kMaxSlots][18];
  int32_t valoff[kMaxSlots][18];
  uint8_t vals[kMaxSlots][256];
  uint32_t pk_dc[2], pk_ac[2], pk_c;
};

// The 9-bit lookahead from the image's LB-bit one: entry k << (LB - 9) when its code fits 9 bits, in
// the write_entry format (size and advance).
template <int LB>
__device__ void load_sync_tables(SyncTables& T, const EntTables* g) {
  const int ns = g->nslots;
  for (int i = threadIdx.x; i < (ns << kSyncLB); i += blockDim.x) {
    const int q = i >> kSyncLB, k = i & ((1 << kSyncLB) - 1);
    const uint16_t e = g->lut[(q << LB) + (k << (LB - kSyncLB))];
    T.lut[i] = (e & 15) <= kSyncLB ? (uint16_t)write_entry(e, (g->slot_src[q] & 4) != 0) : (uint16_t)0;
  }
  for (int i = threadIdx.x; i < ns * 18; i += blockDim.x) {
    T.maxcode[i / 18][i % 18] = g->maxcode[i / 18][i % 18];
    T.valoff[i / 18][i % 18] = g->valoff[i / 18][i % 18];
  }
  const uint32_t* gv = reinterpret_cast<const uint32_t*>(g->vals);
  uint32_t* tv = reinterpret_cast<uint32_t*>(T.vals);
  for (int i = threadIdx.x; i < ns * 64; i += blockDim.x) tv[i] = gv[i];
  if (threadIdx.x == 0) {
    T.pk_dc[0] = g->pk_dc[0];
    T.pk_dc[1] = g->pk_dc[1];
    T.pk_ac[0] = g->pk_ac[0];
    T.pk_ac[1] = g->pk_ac[1];
    T.pk_c = g->pk_c;
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------------------
// Bit reader: 64-bit MSB-first window fed from a queue of kQ byte-swapped words held in
// registers.  The queue is refilled for every lane of a wave at once (bits_fill) when any lane
// has run dry; the byte swap consumes the loads there, so the decode loop itself carries no
// global loads.  (CDNA counts loads and stores on one vmcnt: a load waited on inside the loop
// would also wait for every coefficient/record store issued since.)
// ------------------------------------------------------------------------------------------
#ifndef SDSJ_Q
#define SDSJ_Q 8
#endif
constexpr int kQ = SDSJ_Q;
#ifndef SDSJ_SPEC_WAVES
#define SDSJ_SPEC_WAVES 7  // k_entspec<11> occupancy target (waves per SIMD; 8 spills 7 VGPRs and measured no faster)
#endif
#ifndef SDSJ_SPEC_GROUP
#define SDSJ_SPEC_GROUP 4
#endif
#ifndef SDSJ_WRITE_GROUP
#define SDSJ_WRITE_GROUP 4
#endif
constexpr int kSpecGroup = SDSJ_SPEC_GROUP;    // symbols decoded between two wave-uniform refill checks (spec pass)
constexpr int kWriteGroup = SDSJ_WRITE_GROUP;  // (write pass)
constexpr int kQW = kQ;                        // the write pass's queue (words)
static_assert(kSpecGroup < kQ && kWriteGroup < kQW, "a fresh refill must pass the group check");
// A symbol takes at most 27 bits (16-bit code + 11 extra bits; a bad code 17): a group of G symbols
// has a word to pull before each of them when nb + 32 nq >= 27 (G - 1) + 32 at its start.
constexpr int kRefillSpec = 27 * (kSpecGroup - 1) + 32;
#ifndef SDSJ_REC_STORE
#define SDSJ_REC_STORE 16
#endif
// Records the speculative pass keeps per subsequence (<= kRec): the first 16 block boundaries.  With
// the warm-up, a subsequence's entry is almost always right and k_entsync reads none of them; when
// it is not, paths merge within a few blocks.  16 instead of 64: k_entspec 7.45 -> 7.22 ms per 16,384
// (fewer scattered 8-byte stores; profiles/r03d_ab.txt).
constexpr int kRecStore = SDSJ_REC_STORE;
static_assert(kRecStore <= kRec, "records fit their scratch");
constexpr int kRefillWrite = 27 * (kWriteGroup - 1) + 32;
constexpr int kFlushEvery = kWriteGroup;  // write pass: steps between stage flushes (every 2: 12.9 ms, 4: 12.8)
static_assert(kWriteGroup % kFlushEvery == 0, "a group ends with a flush: nothing is pending across a refill");

template <int Q>
struct BitsQ {
  const uint32_t* src;
  uint64_t buf;
  int nb;
  uint32_t wend; // word index one past the queued words (wend - wi valid words in q)
  uint32_t wi;   // word index of q[0]
  uint32_t pos;  // absolute bit position of the next unconsumed bit
  uint32_t lim;  // bits at or beyond lim read as zeros (the data ran into a marker)
  uint32_t q[Q];
};
using Bits = BitsQ<kQ>;

// Word w of the stream (MSB-first bits [32w, 32w + 32)), zeroed from bit `lim` on.
__device__ __forceinline__ uint32_t load_word(const uint32_t* src, uint32_t w, uint32_t lim) {
  const uint32_t b0 = w * 32u;
  if (b0 >= lim) return 0u;
  const uint32_t v = __builtin_bswap32(src[w]), keep = lim - b0;
  return keep >= 32u ? v : (v & ~(0xFFFFFFFFu >> keep));
}

template <int Q>
__device__ __forceinline__ void bits_init(BitsQ<Q>& b, const uint32_t* src, uint32_t p, uint32_t lim) {
  b.src = src;
  b.lim = lim;
  const uint32_t w = p >> 5;
  const uint32_t hi = load_word(src, w, lim), lo = load_word(src, w + 1, lim);
  const int sh = p & 31;
  b.buf = (((uint64_t)hi << 32) | lo) << sh;
  b.nb = 64 - sh;
  b.wi = w + 2;
  b.wend = b.wi;
  b.pos = p;
#pragma unroll
  for (int k = 0; k < Q; k++) b.q[k] = 0;
}

// Wave-synchronous refill: re-reads kQ words from wi (the ustream carries kUPad bytes of slack), as
// dword-aligned 16-byte loads (global_load_dwordx4: a quarter of the load instructions, and of the
// per-lane cache-line requests, of one dword load per word).
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
template <int Q>
__device__ __forceinline__ void bits_fill(BitsQ<Q>& b) {
  static_assert(Q % 4 == 0, "the queue refills in 16-byte loads");
  if ((b.wi + Q) * 32u <= b.lim) {  // the common case: all kQ words lie before the limit
#pragma unroll
    for (int k = 0; k < Q; k += 4) {
      const u32x4a4 v = *reinterpret_cast<const u32x4a4*>(b.src + b.wi + k);
      b.q[k] = __builtin_bswap32(v.x);
      b.q[k + 1] = __builtin_bswap32(v.y);
      b.q[k + 2] = __builtin_bswap32(v.z);
      b.q[k + 3] = __builtin_bswap32(v.w);
    }
  } else {
#pragma unroll
    for (int k = 0; k < Q; k++) b.q[k] = load_word(b.src, b.wi + k, b.lim);
  }
  b.wend = b.wi + Q;
}

// Bits held (the window and the queue): a group of symbols may run without a refill check while this
// covers them (the refill thresholds kRefillSpec / kRefillWrite).
template <int Q>
__device__ __forceinline__ int bits_avail(const BitsQ<Q>& b) { return b.nb + 32 * (int)(b.wend - b.wi); }

// Can the next symbol (at most 32 bits) be decoded without a refill?
template <int Q>
__device__ __forceinline__ bool bits_can(const BitsQ<Q>& b) { return b.nb > 32 || b.wi < b.wend; }

template <int Q>
__device__ __forceinline__ void bits_pull(BitsQ<Q>& b) {
  // branch-free: a divergent branch here made the compiler copy the whole queue around it on every
  // symbol (phi copies on both paths); selects shift it in place
  const bool need = b.nb <= 32;
  b.buf |= need ? (uint64_t)b.q[0] << ((32 - b.nb) & 63) : 0ull;
  b.nb += need ? 32 : 0;
#pragma unroll
  for (int k = 0; k + 1 < Q; k++) b.q[k] = need ? b.q[k + 1] : b.q[k];
  b.wi += need ? 1u : 0u;
}

// MCU position -> table slots and component, from packed per-image registers.
struct BlkCtx {
  uint64_t pdc, pac;
  uint32_t pc;
  int bpm;
  uint64_t p6;  // images of <= 4 table slots (LB = 11): per MCU block 6 bits, DC slot | AC slot << 2 | comp << 4
  uint64_t p5;  // (the write pass, LB = 11) per MCU block 5 bits: DC slot | AC slot << 2 | the next block's
                // component differs << 4 (an MCU's blocks come component by component, so the predictors
                // can rotate through the components in MCU order instead of being selected by index)
};

__device__ __forceinline__ int ctx_dc(const BlkCtx& k, int blk) { return (int)(k.pdc >> (4 * blk)) & 15; }
__device__ __forceinline__ int ctx_ac(const BlkCtx& k, int blk) { return (int)(k.pac >> (4 * blk)) & 15; }
__device__ __forceinline__ int ctx_c(const BlkCtx& k, int blk) { return (int)(k.pc >> (2 * blk)) & 3; }

template <class TT>
__device__ __forceinline__ BlkCtx make_ctx(const TT& T, int bpm) {
  BlkCtx k;
  k.pdc = ((uint64_t)T.pk_dc[1] << 32) | T.pk_dc[0];
  k.pac = ((uint64_t)T.pk_ac[1] << 32) | T.pk_ac[0];
  k.pc = T.pk_c;
  k.bpm = bpm;
  k.p6 = 0;
  k.p5 = 0;
  for (int b = 0; b < bpm; b++) {
    const uint64_t c = (k.pc >> (2 * b)) & 3, cn = (k.pc >> (2 * (b + 1 == bpm ? 0 : b + 1))) & 3;
    k.p6 |= (uint64_t)(((k.pdc >> (4 * b)) & 3) | (((k.pac >> (4 * b)) & 3) << 2) | (c << 4)) << (6 * b);
    k.p5 |= (uint64_t)(((k.pdc >> (4 * b)) & 3) | (((k.pac >> (4 * b)) & 3) << 2) | ((uint64_t)(c != cn) << 4)) << (5 * b);
  }
  return k;
}

// The write pass's context of MCU block blk (LB = 11): table slots and whether the component changes after it.
__device__ __forceinline__ void ctx_w5(const BlkCtx& k, int blk, int& sdc, int& sac, bool& chg) {
  const uint32_t x = (uint32_t)(k.p5 >> __umul24((unsigned)blk, 5u));
  sdc = (int)(x & 3);
  sac = (int)((x >> 2) & 3);
  chg = (x >> 4) & 1;
}

// All three of an MCU block's context values from the 6-bit packing (<= 4 table slots): one 64-bit
// shift and three field extracts instead of three separate shifts of the 4- and 2-bit packings.
__device__ __forceinline__ void ctx_all6(const BlkCtx& k, int blk, int& c, int& sdc, int& sac) {
  const uint32_t x = (uint32_t)(k.p6 >> __umul24((unsigned)blk, 6u));  // (24-bit multiply: full rate)
  sdc = (int)(x & 3);
  sac = (int)((x >> 2) & 3);
  c = (int)((x >> 4) & 3);
}

// jpeg_huff_decode for a code longer than LB bits (lookahead entry 0): the canonical search --
// the first length whose code is <= maxcode.  Only lengths LB + 1 .. 16 can match: every code of at
// most LB bits has its lookahead entry (a zero entry for a short code would need a DC category > 15,
// and such tables are rejected at parse time, huff_table_ok).  The compares issue together.
// hi = the next 32 bits; gives the code length l (17 = bad code), category s and run r.
template <int LB, class TT>
__device__ __forceinline__ void long_code(const TT& T, int slot, bool isdc, uint32_t hi, int& l, int& s, int& r,
                                          int& bad) {
  const uint32_t peek = hi >> 16;
  int ll = 17;
#pragma unroll
  for (int k = 16; k > LB; k--) ll = (int32_t)(peek >> (16 - k)) <= T.maxcode[slot][k] ? k : ll;
  if (ll > 16) {
    bad = 1;  // JWRN_HUFF_BAD_CODE: 17 bits consumed, symbol 0 (libjpeg warns and goes on)
    l = 17;
    s = 0;
    r = 0;
  } else {
    const int sym = T.vals[slot][((int32_t)(peek >> (16 - ll)) + T.valoff[slot][ll]) & 0xFF];
    l = ll;
    s = isdc ? sym : (sym & 15);
    r = isdc ? 0 : (sym >> 4);
  }
}

// The write pass's tables for LB = 11 images (at most 4 slots), compact enough for 4 workgroups per
// CU: a 9-bit first level and, for each 9-bit prefix of a longer code, a 4-entry second level holding
// the LB = 11 table's entries for the next 2 bits (codes of 10 and 11 bits).  Longer codes (entry 0
// at both levels) take the canonical search as before.  First-level entry of such a prefix:
// (second-level subtable + 1) << 4 with length 0 (0: no subtable left -- the canonical search).
constexpr int kW1 = 9;
constexpr int kW2Cap = 256;  // second-level entries (64 subtables; a standard table needs ~8)
struct WriteTables {
  static constexpr bool kTwoLevel = true;
  uint16_t lut[4 << kW1];
  uint16_t l2[kW2Cap];
  int32_t maxcode[4][18];
  int32_t valoff[4][18];
  uint8_t vals[4][256];
  uint32_t pk_dc[2], pk_ac[2], pk_c;
  uint32_t pad[3];
};


template <int LB, class TT>
__device__ __forceinline__ uint32_t lookup(const TT& T, int slot, uint32_t hi) {
  if constexpr (TT::kTwoLevel) {
    uint32_t e = T.lut[(slot << kW1) + (hi >> (32 - kW1))];
    if ((e & 15) == 0) {  // code longer than 9 bits
      const uint32_t sub = e >> 4;
      e = sub ? T.l2[((sub - 1) << 2) + ((hi >> (32 - kW1 - 2)) & 3)] : 0u;
    }
    return e;
  } else {
    return T.lut[(slot << LB) + (hi >> (32 - LB))];
  }
}

// HUFF_EXTEND of the s extra bits that follow the code inside hi (l + s = tot <= 27): x < 2^(s-1) ->
// x - (2^s - 1); s = 0 -> 0 (a zero-width field extract, mask 0).  One bit-field extract for x.
__device__ __forceinline__ int huff_extend(uint32_t hi, int tot, int s) {
  const uint32_t x = __builtin_amdgcn_ubfe(hi, (uint32_t)(32 - tot), (uint32_t)s);
  const uint32_t msk = (1u << s) - 1u;
  return (x >> ((s - 1) & 31)) ? (int)x : (int)x - (int)msk;
}

// One symbol (jdhuff.c HUFF_DECODE + get_bits + HUFF_EXTEND): DC -> category s, r = 0;
// AC -> (r, s).  val = the extended value (0 when s = 0).
template <int LB, class TT, int Q>
__device__ __forceinline__ void decode_sym(const TT& T, BitsQ<Q>& b, int slot, bool isdc, int& s, int& r, int& val,
                                           int& bad) {
  bits_pull(b);
  const uint32_t hi = (uint32_t)(b.buf >> 32);
  const uint32_t e = lookup<LB>(T, slot, hi);
  int l = e & 15;
  s = (e >> 4) & 15;
  r = (e >> 8) & 15;
  // (two-level tables: a prefix without a second level -- more long prefixes than kW2Cap / 4 -- may
  // hold 10- and 11-bit codes too, so their search starts past the first level's width)
  if (l == 0) long_code<TT::kTwoLevel ? kW1 : LB>(T, slot, isdc, hi, l, s, r, bad);
  // HUFF_EXTEND without branches: the s extra bits follow the l code bits inside hi (l + s <= 27; a
  // bad code has s = 0), x < 2^(s-1) -> x - (2^s - 1); s = 0 -> x = 0, mask 0 -> 0
  const int tot = l + s;
  val = huff_extend(hi, tot, s);
  b.buf <<= tot;
  b.nb -= tot;
  b.pos += tot;
}

// decode_sym for tables in the write_entry format (the write and sync passes'): the symbol's size and its
// advance of the zigzag position instead of (size, run).  A bad code (JWRN_HUFF_BAD_CODE) sets `bad`.
template <int LB, class TT, int Q>
__device__ __forceinline__ void decode_wsym(const TT& T, BitsQ<Q>& b, int slot, bool isdc, int& s, int& adv, int& val,
                                            int& bad) {
  bits_pull(b);
  const uint32_t hi = (uint32_t)(b.buf >> 32);
  int l;
  if constexpr (TT::kTwoLevel) {
    // one branch for both rare cases (a code longer than the first level: its second level, and codes
    // longer than that the canonical search)
    const uint32_t e = T.lut[(slot << kW1) + (hi >> (32 - kW1))];
    l = e & 15;
    s = (e >> 4) & 15;
    adv = (e >> 8) & 127;
    if (l == 0) {
      const uint32_t sub = e >> 4;
      const uint32_t e2 = sub ? T.l2[((sub - 1) << 2) + ((hi >> (32 - kW1 - 2)) & 3)] : 0u;
      l = e2 & 15;
      s = (e2 >> 4) & 15;
      adv = (e2 >> 8) & 127;
      if (l == 0) {
        int r;
        long_code<kW1>(T, slot, isdc, hi, l, s, r, bad);
        adv = (int)write_adv(!isdc, (uint32_t)s, (uint32_t)r);
      }
    }
  } else {
    const uint32_t e = lookup<LB>(T, slot, hi);
    l = e & 15;
    s = (e >> 4) & 15;
    adv = (e >> 8) & 127;
    if (l == 0) {
      int r;
      long_code<LB>(T, slot, isdc, hi, l, s, r, bad);
      adv = (int)write_adv(!isdc, (uint32_t)s, (uint32_t)r);
    }
  }
  const int tot = l + s;
  val = huff_extend(hi, tot, s);
  b.buf <<= tot;
  b.nb -= tot;
  b.pos += tot;
}

// One step through the multi-symbol table (SpecTables::mlut): a group of AC symbols that ends inside
// the block (z + advance <= 64) at once, else one symbol -- the DC symbol (with its value when kVal),
// or an AC symbol near the block end.  Gives the (s, r) next_z takes for the step: a group of value /
// ZRL symbols advances like one symbol of run dz - 1, a group ending in EOB like an EOB.  The group's
// symbols are exactly the ones single decodes would give (k_enttab walks them with the same LUT).
// adv: the step's advance of the block position (write_adv; a group ending in EOB: 64), so the
// block ends when z + adv passes 63.
template <bool kVal, class TT, int Q>
__device__ __forceinline__ void decode_step(const TT& T, BitsQ<Q>& b, int slot, bool isdc, int z, int& adv,
                                            int& val, int& bad) {
  bits_pull(b);
  const uint32_t hi = (uint32_t)(b.buf >> 32);
  const uint32_t e = T.mlut[(slot << kMW) + (hi >> (32 - kMW))];
  int l = e & 15, sz = (e >> 4) & 15, a = (int)(e >> 25);
  const int mb = (e >> 12) & 31, mdz = (e >> 17) & 127, eob = (e >> 24) & 1;
  const bool multi = (mb != 0) & (z + mdz <= 64);
  if (!multi && l == 0) {
    int rr;
    long_code<kMW>(T, slot, isdc, hi, l, sz, rr, bad);
    a = (int)write_adv(!isdc, (uint32_t)sz, (uint32_t)rr);
  }
  if (kVal) val = huff_extend(hi, l + sz, sz);  // (only DC values are used: a group is never a DC step)
  const int tot = multi ? mb : l + sz;
  adv = multi ? (eob ? 64 : mdz) : a;
  b.buf <<= tot;
  b.nb -= tot;
  b.pos += tot;
}

// The block position after a step of advance adv; true when the step ended the block.
__device__ __forceinline__ bool adv_z(int& z, int adv) {
  const int zn = z + adv;
  const bool done = zn > 63;
  z = done ? 0 : zn;
  return done;
}

// decode_mcu's k loop: DC -> k = 1; AC value -> k += r + 1; ZRL -> k += 16; EOB -> done.
// Returns true when the block is complete (z wraps to 0).  Branch-free: the step is r + 1 for a DC
// symbol (r = 0), an AC value or ZRL (r = 15), and 64 for EOB.
__device__ __forceinline__ bool next_z(int& z, int s, int r) {
  const int m = (s != 0) | (r == 15) | (z == 0);
  const int zn = z + 64 - m * (63 - r);
  const bool done = zn >= 64;
  z = done ? 0 : zn;
  return done;
}

__device__ __forceinline__ void add_dc(int c, int v, int& d0, int& d1, int& d2) {
  d0 += c == 0 ? v : 0;
  d1 += c == 1 ? v : 0;
  d2 += c == 2 ? v : 0;
}

// Exclusive scan over the first NT threads (threads beyond NT -- the write pass's transform waves --
// take part in the barriers only and get 0).
template <int NT = kEntThreads>
__device__ inline int block_excl_scan(int v, int* tmp, int* total) {
  const int t = threadIdx.x;
  const bool in = t < NT;
  if (in) tmp[t] = v;
  __syncthreads();
  for (int off = 1; off < NT; off <<= 1) {
    int a = in && t >= off ? tmp[t - off] : 0;
    __syncthreads();
    if (in) tmp[t] += a;
    __syncthreads();
  }
  const int incl = in ? tmp[t] : v;
  *total = tmp[NT - 1];
  __syncthreads();
  return incl - v;
}

// ------------------------------------------------------------------------------------------
// k_entsync
// ------------------------------------------------------------------------------------------
template <int NT, class TT = LutTables>
struct LdsSyncT {
  TT T;
  int32_t tmp[NT];  // block_excl_scan scratch
  union {                    // sync rounds | final segmented scan (never live together)
    int32_t task[1][max_tasks<NT>()];
    struct {
      int32_t scan[4][NT];
      int32_t flag[NT];
    } fs;
  } u;
  int32_t nsub, rounds, stages;
  unsigned long long sym[2];
  unsigned long long t0, t1, t2;
  unsigned long long it[2];
  int32_t wmax[NT / 64];
};
using LdsSync = LdsSyncT<kEntThreads>;

// Speculative decode of subsequence S.  Warm-up: decode from `warm` bits before start_bit (not
// before the segment start) assuming (block 0, DC), and take the first block boundary at or after
// start_bit as the entry; by then the decode has almost always merged with the true path (JPEG's
// Huffman self-synchronisation; the MCU phase takes ~1k bits to lock on).  Then decode to the first
// block boundary at or after end_bit, recording every block boundary.  A segment's first
// subsequence starts exactly at its (known) state.
template <int LB, class TT>
// at: the subsequence is entered exactly at (at_p, MCU block at_blk) -- the speculative exit of its
// predecessor, decoded by the same lane just before (paired subsequences) -- with no warm-up.
// init_blk: the MCU block the warm-up assumes at its first bit (k_entspec_mh's phase hypotheses; 0
// otherwise); keep_rec: store block-boundary records.
__device__ int spec_pass(const TT& T, const BlkCtx& K, const uint32_t* src, SubState& S, SyncRec* rec,
                         uint32_t seg_start, uint32_t warm, bool at = false, uint32_t at_p = 0, int at_blk = 0,
                         int init_blk = 0, bool keep_rec = true) {
  constexpr bool kMulti = std::is_same_v<TT, SpecTables>;  // LB = 11: the multi-symbol table
  // (bits at or beyond S.lim_bit read as zeros)
  const uint32_t start = S.start_bit, end = S.end_bit;
  const uint32_t ws = at ? at_p : (S.first ? start : (start - seg_start > warm ? start - warm : seg_start));
  Bits b;
  bits_init(b, src, ws, S.lim_bit);
  int blk = at ? at_blk : init_blk, z = 0, nrec = 0, dcd = 0, bad = 0, nsym = 0;  // nrec: also the block count
  int d0 = 0, d1 = 0, d2 = 0;
  // MCU block context: for the LB = 11 images (<= 4 table slots) the 5-bit packing, whose third value
  // is whether the component changes after the block (the DC sums rotate through the MCU's component
  // cycle as the write pass's predictors do: d0 is the current block's component), else the 4-bit
  // packings and the component
  auto ctx = [&](int bk, int& cc, int& dc_slot, int& ac_slot) {
    if constexpr (kMulti) {
      bool chg;
      ctx_w5(K, bk, dc_slot, ac_slot, chg);
      cc = chg;
    } else {
      cc = ctx_c(K, bk);
      dc_slot = ctx_dc(K, bk);
      ac_slot = ctx_ac(K, bk);
    }
  };
  int c, sdc, sac;
  ctx(blk, c, sdc, sac);
  // the MCU's component cycle: succ[c] = the component after c's blocks; n3: three components in it
  int succ[kMaxComp] = {0, 0, 0};
  for (int bb = 0; bb < K.bpm; bb++) {
    const int cb = ctx_c(K, bb), cn = ctx_c(K, bb + 1 == K.bpm ? 0 : bb + 1);
    if (cn != cb) succ[cb] = cn;
  }
  const bool n3 = kMulti && succ[succ[ctx_c(K, 0)]] != ctx_c(K, 0) && succ[ctx_c(K, 0)] != ctx_c(K, 0);
  uint32_t entry = at ? at_p : start;
  int entry_blk = blk;
  bool warmup = !at && b.pos < start;
  // warm-up: only the MCU position matters (no values, no records): code length + size per symbol
  while (__builtin_amdgcn_ballot_w64(warmup)) {
    if (warmup) bits_fill(b);
    for (;;) {
#pragma unroll
      for (int u = 0; u < kSpecGroup; u++) {
        if (warmup) {
          const bool isdc = z == 0;
          const int slot = isdc ? sdc : sac;
          bool done;
          if constexpr (kMulti) {
            int adv, unused;
            decode_step<false>(T, b, slot, isdc, z, adv, unused, bad);
            done = adv_z(z, adv);
          } else {
            int sz, r;
            bits_pull(b);
            const uint32_t hi = (uint32_t)(b.buf >> 32);
            const uint32_t e = T.lut[(slot << LB) + (hi >> (32 - LB))];
            int l = e & 15;
            sz = (e >> 4) & 15;
            r = (e >> 8) & 15;
            if (l == 0) long_code<LB>(T, slot, isdc, hi, l, sz, r, bad);
            const int tot = l + sz;
            b.buf <<= tot;
            b.nb -= tot;
            b.pos += tot;
            done = next_z(z, sz, r);
          }
          if (kStats) nsym++;
          if (done) {
            blk = blk + 1 == K.bpm ? 0 : blk + 1;
            ctx(blk, c, sdc, sac);
            if (b.pos >= start) {
              warmup = false;
              entry = b.pos;
              entry_blk = blk;
            }
          }
        }
      }
      if (__builtin_amdgcn_ballot_w64(warmup && bits_avail(b) < kRefillSpec) ||
          !__builtin_amdgcn_ballot_w64(warmup))
        break;
    }
  }
  bool run = b.pos < end || z != 0;
  while (__builtin_amdgcn_ballot_w64(run)) {
    if (run) bits_fill(b);
    for (;;) {
      // kSpecGroup symbols per wave-uniform check: every running lane holds >= bits for them.  A lane
      // that completes a block waits for the group's end, where the block-end bookkeeping (record,
      // DC sums, MCU position and context, the stop test) runs once instead of as selects on every step
      bool pend = false;
#pragma unroll
      for (int u = 0; u < kSpecGroup; u++) {
        if (run && !pend) {
          int val;
          const bool isdc = z == 0;
          if constexpr (kMulti) {
            int adv;
            decode_step<true>(T, b, isdc ? sdc : sac, isdc, z, adv, val, bad);
            pend = adv_z(z, adv);
          } else {
            int s, r;
            decode_sym<LB>(T, b, isdc ? sdc : sac, isdc, s, r, val, bad);
            pend = next_z(z, s, r);
          }
          if (kStats) nsym++;
          dcd = isdc ? val : dcd;  // (the block's DC difference joins its component's sum at the block end)
        }
      }
      if (pend) {
        if (keep_rec && nrec < kRecStore)  // one 8-byte store (SyncRec: p, dc, blk, pad)
          reinterpret_cast<uint2*>(rec)[nrec] =
              make_uint2(b.pos, ((uint32_t)dcd & 0xFFFFu) | ((uint32_t)(blk & 0xFF) << 16));
        if constexpr (kMulti) {
          // (d0, d1, d2) -> (d1, d2, d0) after a block whose successor is of the next component (two
          // components: (d0, d1) -> (d1, d0))
          d0 += dcd;
          if (c != 0) {
            const int t0 = d0;
            d0 = d1;
            d1 = n3 ? d2 : t0;
            d2 = n3 ? t0 : d2;
          }
        } else {
          add_dc(c, dcd, d0, d1, d2);
        }
        nrec++;
        blk = blk + 1 == K.bpm ? 0 : blk + 1;
        ctx(blk, c, sdc, sac);
        run = b.pos < end;  // (at a block boundary)
      }
      // leave to refill when a running lane may not hold kSpecGroup more symbols (<= 32 bits each)
      if (__builtin_amdgcn_ballot_w64(run && bits_avail(b) < kRefillSpec) ||
          !__builtin_amdgcn_ballot_w64(run))
        break;
    }
  }
  if constexpr (kMulti) {  // the rotating sums back to component order
    const int ce = ctx_c(K, blk), c1 = succ[ce], c2 = succ[c1];
    int o0 = 0, o1 = 0, o2 = 0;
    add_dc(ce, d0, o0, o1, o2);
    if (c1 != ce) add_dc(c1, d1, o0, o1, o2);
    if (n3) add_dc(c2, d2, o0, o1, o2);
    d0 = o0;
    d1 = o1;
    d2 = o2;
  }
  S.entry_p = entry;
  S.entry_bz = (uint16_t)(entry_blk << 8);
  S.spec_exit_p = S.cur_exit_p = b.pos;
  S.spec_exit_bz = S.cur_exit_bz = (uint16_t)((blk << 8) | z);
  S.spec_nblk = S.cur_nblk = nrec;
  S.spec_dc[0] = S.cur_dc[0] = d0;
  S.spec_dc[1] = S.cur_dc[1] = d1;
  S.spec_dc[2] = S.cur_dc[2] = d2;
  S.nrec = nrec < kRecStore ? nrec : kRecStore;
  return nsym;
}

// Re-decode of subsequence S from its corrected entry (new_entry_*) to its end -- the first block
// boundary at or after end_bit, as in the speculative pass -- giving the exact exit state, block
// count and DC sums in new_*.  A lean loop like the speculative pass's; every kMergeBits of progress
// a lane that sits on a block boundary looks it up among the speculative pass's records (binary
// search): the same position and MCU block means the two paths have merged, and the rest of the
// speculative result is exact (large subsequences stop there instead of decoding to their end).
constexpr uint32_t kMergeBits = 768;
constexpr int kSyncQ = kQ;  // (a deeper queue measured slower: the pull shifts it)

template <int LB, class TT>
__device__ int sync_full(const TT& T, const BlkCtx& K, const uint32_t* src, SubState& S, const SyncRec* rec) {
  const uint32_t end = S.end_bit;
  const int nrec = S.nrec;
  BitsQ<kSyncQ> b;
  bits_init(b, src, S.new_entry_p, S.lim_bit);
  int blk = S.new_entry_bz >> 8, z = S.new_entry_bz & 0xFF;
  int nblk = 0, bad = 0, nsym = 0, d0 = 0, d1 = 0, d2 = 0, dcd = 0;
  uint32_t next_chk = nrec > 0 ? b.pos + kMergeBits : 0xFFFFFFFFu;
  bool merged = false;
  int c = ctx_c(K, blk), sdc = ctx_dc(K, blk), sac = ctx_ac(K, blk);
  bool run = b.pos < end || z != 0;
  while (__builtin_amdgcn_ballot_w64(run)) {
    if (run) bits_fill(b);
    for (;;) {
      bool pend = false;  // (a completed block's bookkeeping waits for the group's end, as in spec_pass)
#pragma unroll
      for (int u = 0; u < kSpecGroup; u++) {
        if (run && !pend) {
          int sy, adv, val;
          const bool isdc = z == 0;
          decode_wsym<LB>(T, b, isdc ? sdc : sac, isdc, sy, adv, val, bad);
          if (kStats) nsym++;
          dcd = isdc ? val : dcd;
          pend = adv_z(z, adv);
        }
      }
      if (pend) {
        add_dc(c, dcd, d0, d1, d2);
        nblk++;
        blk = blk + 1 == K.bpm ? 0 : blk + 1;
        c = ctx_c(K, blk);
        sdc = ctx_dc(K, blk);
        sac = ctx_ac(K, blk);
        run = b.pos < end;  // (at a block boundary)
      }
      if (run && z == 0 && b.pos >= next_chk) {
        // first record at or after b.pos; a record there for the block just completed = merged
        int lo = 0, hi = nrec;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (rec[mid].p < b.pos) lo = mid + 1;
          else hi = mid;
        }
        const int done_blk = blk == 0 ? K.bpm - 1 : blk - 1;
        if (lo < nrec && rec[lo].p == b.pos && rec[lo].blk == done_blk) {
          int q0 = 0, q1 = 0, q2 = 0;  // speculative DC sums up to and including that block
          for (int k = 0; k <= lo; k++) add_dc(ctx_c(K, rec[k].blk), rec[k].dc, q0, q1, q2);
          S.new_exit_p = S.spec_exit_p;
          S.new_exit_bz = S.spec_exit_bz;
          S.new_nblk = nblk + S.spec_nblk - (lo + 1);
          S.new_dc[0] = d0 + S.spec_dc[0] - q0;
          S.new_dc[1] = d1 + S.spec_dc[1] - q1;
          S.new_dc[2] = d2 + S.spec_dc[2] - q2;
          merged = true;
          run = false;
        } else {
          next_chk = lo < nrec ? b.pos + kMergeBits : 0xFFFFFFFFu;
        }
      }
      if (__builtin_amdgcn_ballot_w64(run && bits_avail(b) < kRefillSpec) ||
          !__builtin_amdgcn_ballot_w64(run))
        break;
    }
  }
  if (!merged) {
    S.new_exit_p = b.pos;
    S.new_exit_bz = (uint16_t)((blk << 8) | z);
    S.new_nblk = nblk;
    S.new_dc[0] = d0;
    S.new_dc[1] = d1;
    S.new_dc[2] = d2;
  }
  return nsym;
}

// The speculative pass's LDS: tables, the layout scan's scratch, statistics -- not the sync kernel's
// task / scan arrays (5 KB that cost it two workgroups per CU)
template <int LB, int NT>
struct LdsSpec {
  std::conditional_t<LB == 11, SpecTables, LutTables> T;
  int32_t tmp[NT];
  int32_t nsub;
  unsigned long long sym[1], it[1], t0, t1;
  int32_t wmax[NT / 64];
};

// NT threads per image: each lane takes kEntThreads / NT consecutive subsequences of the image's
// kEntThreads-lane layout, the first after its warm-up, the next ones entered exactly at the
// previous one's speculative exit (spec_pass `at`), so a pair shares one warm-up.
template <int LB, int NT = kEntThreads>
__device__ void entspec_image(int img, int grp, ImgDesc* __restrict__ descs, const EntTables* __restrict__ tables,
                              uint8_t* __restrict__ scratch) {
  constexpr int F = kEntThreads / NT;
  ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK || d->mh) return;  // (mh: k_entspec_mh + k_mh_select)
  __shared__ LdsSpec<LB, NT> L;
  const int t = threadIdx.x;
  int ns;
  if constexpr (LB == 11) ns = load_tables(L.T, &tables[d->etab]);
  else ns = load_tables<LB>(L.T, &tables[d->etab]);
  if (!variant_owns<LB>(ns)) return;
  if (t == 0) {
    L.sym[0] = 0;
    L.it[0] = 0;
  }
  const BlkCtx K = make_ctx(L.T, d->bpm);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(scratch + d->off_ustream);
  const SegView sv = seg_view(scratch + d->off_seg, d->nseg);
  SubState* sub = reinterpret_cast<SubState*>(scratch + d->off_sub);
  SyncRec* recs = reinterpret_cast<SyncRec*>(scratch + d->off_rec);
  const int nseg = d->nseg;
  const uint32_t SB = (uint32_t)d->sub_bits;

  // --- subsequence layout: restart interval s (bytes [lo[s], hi[s])) -> max(1, ceil(bits / SB)) ---
  {
    int carry = 0;
    for (int base = 0; base < nseg; base += NT) {
      const int s = base + t;
      int cnt = 0;
      uint32_t b0 = 0, b1 = 0;
      if (s < nseg) {
        b0 = (uint32_t)sv.lo[s] * 8u;
        b1 = (uint32_t)sv.hi[s] * 8u;
        if (b1 < b0) b1 = b0;
        cnt = b1 > b0 ? (int)((b1 - b0 + SB - 1) / SB) : 1;
      }
      int total;
      const int off = carry + block_excl_scan<NT>(cnt, L.tmp, &total);
      if (s < nseg) {
        for (int k = 0; k < cnt; k++) {
          const int j = off + k;
          if (j >= d->nsub_cap) break;
          SubState& S = sub[j];
          S.start_bit = b0 + (uint32_t)k * SB;
          const uint32_t e = S.start_bit + SB;
          S.end_bit = e < b1 ? e : b1;
          S.first = k == 0;
          S.seg = s;
          S.lim_bit = b1;
        }
      }
      carry += total;
    }
    if (t == 0) L.nsub = carry < d->nsub_cap ? carry : d->nsub_cap;
  }
  __syncthreads();
  const int nsub = L.nsub;
  unsigned long long nsym_spec = 0;

  // --- 1. speculative pass ---
  if (kStats && t == 0) L.t0 = __builtin_amdgcn_s_memtime();
  if (kStats && (t & 63) == 0) L.wmax[t >> 6] = 0;
  __syncthreads();
  // this workgroup's share of the subsequences (every group computes the same layout above)
  const int G = d->ent_groups, per = (nsub + G - 1) / G, j0 = grp * per, j1 = j0 + per < nsub ? j0 + per : nsub;
  for (int jb = j0 + F * t; jb < j1; jb += F * NT) {
    int k = 0;
#pragma unroll
    for (int q = 0; q < F; q++) {
      const int j = jb + q;
      if (j >= j1) break;
      // a later subsequence of the lane's run starts where the previous one stopped (same segment)
      const bool at = q > 0 && !sub[j].first;
      const uint32_t at_p = at ? sub[j - 1].spec_exit_p : 0u;
      const int at_blk = at ? sub[j - 1].spec_exit_bz >> 8 : 0;
      k += spec_pass<LB>(L.T, K, src, sub[j], recs + (int64_t)j * kRec, (uint32_t)sv.lo[sub[j].seg] * 8u,
                         (uint32_t)d->warm_bits, at, at_p, at_blk);
    }
    if (kStats) {
      nsym_spec += k;
      atomicMax(&L.wmax[t >> 6], k);
    }
  }
  __syncthreads();
  if (kStats && t == 0) {
    L.t1 = __builtin_amdgcn_s_memtime();
    for (int w = 0; w < NT / 64; w++) L.it[0] += 64ull * L.wmax[w];
  }
  if (kStats) atomicAdd(&L.sym[0], nsym_spec);
  __syncthreads();
  if (t == 0) d->nsub = nsub;
  if (kStats && t == 0 && grp == 0) {  // statistics: the first group's share
    d->sym_spec = (int64_t)L.sym[0];
    d->t_spec = (int64_t)(L.t1 - L.t0);
    d->it_spec = (int64_t)L.it[0];
  }
}

template <int LB, int NT>
__device__ void entsync_image(int img, ImgDesc* __restrict__ descs, const EntTables* __restrict__ tables,
                              uint8_t* __restrict__ scratch) {
  ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK) return;
  __shared__ LdsSyncT<NT, SyncTables> L;
  const int t = threadIdx.x;
  const int nsub = d->nsub;
  SubState* sub = reinterpret_cast<SubState*>(scratch + d->off_sub);
  SyncRec* recs = reinterpret_cast<SyncRec*>(scratch + d->off_rec);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(scratch + d->off_ustream);
  unsigned long long nsym_sync = 0;
  if (t == 0) {
    L.rounds = 0;
    L.stages = 0;
    L.sym[0] = L.sym[1] = 0;
    L.it[0] = L.it[1] = 0;
    if (kStats) L.t1 = __builtin_amdgcn_s_memtime();
  }
  // any subsequence whose entry differs from its predecessor's exit?  Only then are the decode
  // tables built (most images: none after the warm-up)
  bool need_any = false;
  for (int j = t; j < nsub; j += NT)
    if (!sub[j].first && (sub[j - 1].cur_exit_p != sub[j].entry_p || sub[j - 1].cur_exit_bz != sub[j].entry_bz))
      need_any = true;
  BlkCtx K{};
  if (__syncthreads_or(need_any)) {
    load_sync_tables<LB>(L.T, &tables[d->etab]);
    K = make_ctx(L.T, d->bpm);
    // --- 2. sync rounds until every entry equals its predecessor's exit ---
    for (;;) {
      // tasks of this round: j with entry != exit(j-1); new entry = exit(j-1) (previous values)
      int ntask = 0;
      for (int base = 0; base < nsub; base += NT) {
        const int j = base + t;
        bool need = false;
        uint32_t ep = 0;
        uint16_t ebz = 0;
        if (j < nsub && !sub[j].first) {
          ep = sub[j - 1].cur_exit_p;
          ebz = sub[j - 1].cur_exit_bz;
          need = ep != sub[j].entry_p || ebz != sub[j].entry_bz;
        }
        int tot;
        const int off = block_excl_scan<NT>(need ? 1 : 0, L.tmp, &tot);
        if (need && ntask + off < max_tasks<NT>()) {
          L.u.task[0][ntask + off] = j;
          SubState& S = sub[j];
          S.new_entry_p = ep;
          S.new_entry_bz = ebz;
        }
        ntask += tot;
      }
      if (ntask > max_tasks<NT>()) ntask = max_tasks<NT>();  // the rest are picked up by the next round
      __syncthreads();
      if (ntask == 0) break;
      if (t == 0) {
        L.rounds++;
        L.stages += ntask;  // (statistics: tasks over all rounds)
      }
      for (int i = t; i < ntask; i += NT) {
        const int j = L.u.task[0][i];
        const int k = sync_full<kSyncLB>(L.T, K, src, sub[j], recs + (int64_t)j * kRec);
        if (kStats) nsym_sync += k;
      }
      __syncthreads();
      // commit every task of the round (entries first: they were read from cur_exit of j-1)
      for (int i = t; i < ntask; i += NT) {
        SubState& S = sub[L.u.task[0][i]];
        S.entry_p = S.new_entry_p;
        S.entry_bz = S.new_entry_bz;
      }
      __syncthreads();
      for (int i = t; i < ntask; i += NT) {
        SubState& S = sub[L.u.task[0][i]];
        S.cur_exit_p = S.new_exit_p;
        S.cur_exit_bz = S.new_exit_bz;
        S.cur_nblk = S.new_nblk;
        S.cur_dc[0] = S.new_dc[0];
        S.cur_dc[1] = S.new_dc[1];
        S.cur_dc[2] = S.new_dc[2];
      }
      __syncthreads();
    }
  }
  // --- 3. segmented exclusive scan of (blocks, dc0, dc1, dc2) ---
  if (kStats && t == 0) L.t2 = __builtin_amdgcn_s_memtime();
  {
    int carry[4] = {0, 0, 0, 0};
    for (int base = 0; base < nsub; base += NT) {
      const int j = base + t;
      int v[4] = {0, 0, 0, 0};
      int f = 1;
      if (j < nsub) {
        const SubState& S = sub[j];
        v[0] = S.cur_nblk;
        v[1] = S.cur_dc[0];
        v[2] = S.cur_dc[1];
        v[3] = S.cur_dc[2];
        f = S.first;
      }
      for (int q = 0; q < 4; q++) L.u.fs.scan[q][t] = v[q];
      L.u.fs.flag[t] = f;
      __syncthreads();
      for (int off = 1; off < NT; off <<= 1) {
        int a[4] = {0, 0, 0, 0}, af = 0;
        const bool take = t >= off;
        if (take) {
          for (int q = 0; q < 4; q++) a[q] = L.u.fs.scan[q][t - off];
          af = L.u.fs.flag[t - off];
        }
        __syncthreads();
        if (take && !L.u.fs.flag[t])
          for (int q = 0; q < 4; q++) L.u.fs.scan[q][t] += a[q];
        if (take) L.u.fs.flag[t] |= af;
        __syncthreads();
      }
      if (j < nsub) {
        SubState& S = sub[j];
        const int hit = L.u.fs.flag[t];
        int ex[4];
        for (int q = 0; q < 4; q++) ex[q] = S.first ? 0 : L.u.fs.scan[q][t] - v[q] + (hit ? 0 : carry[q]);
        S.nblk_ex = ex[0];
        S.dc_ex[0] = ex[1];
        S.dc_ex[1] = ex[2];
        S.dc_ex[2] = ex[3];
      }
      __syncthreads();
      const int any = L.u.fs.flag[NT - 1];
      for (int q = 0; q < 4; q++) carry[q] = L.u.fs.scan[q][NT - 1] + (any ? 0 : carry[q]);
      __syncthreads();
    }
  }
  if (kStats) atomicAdd(&L.sym[1], nsym_sync);
  __syncthreads();
  if (t == 0) {
    d->sync_rounds = L.rounds;
    d->pad0 = L.stages;
  }
  if (kStats && t == 0) {
    d->sym_sync = (int64_t)L.sym[1];
    d->t_sync = (int64_t)(L.t2 - L.t1);
    d->t_scan = (int64_t)(__builtin_amdgcn_s_memtime() - L.t2);
    d->it_sync = (int64_t)L.it[1];
  }
}

// ------------------------------------------------------------------------------------------
// k_entwrite
// ------------------------------------------------------------------------------------------
// A 16-byte coefficient store, non-temporal: k_idct reads the coefficients back only after the whole
// lane's write pass (far more than the caches hold), so they should not displace the bit streams the
// entropy passes are reading (write pass 13.7 -> 13.4 ms per 32,768, +0.8 % images/s; profiles/r05_ab.txt).
__device__ __forceinline__ void store_coef16(void* p, uint4 v) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(v4u{v.x, v.y, v.z, v.w}, reinterpret_cast<v4u*>(p));
}
template <class TT>
struct LdsWriteT {
  unsigned long long t0, it;
  TT T;
  alignas(16) int16_t stage[kEntThreads * kStageStride];
  uint32_t flist[kEntThreads / 64][64];  // (thread << 24) | block index (total_blocks < 2^24)
  int32_t bad;
  unsigned long long sym;
};

// The compact two-level tables from the image's LB = 11 tables (HBM).  The staging area serves as
// the scan's scratch before it is cleared.
template <int NT = kEntThreads>
__device__ int load_write_tables(WriteTables& W, const EntTables* g, int32_t* tmp) {
  const int t = threadIdx.x;
  const int ns = g->nslots;
  if (!variant_owns<11>(ns)) return ns;
  // which 9-bit prefixes lead to longer codes: (4 << kW1) / NT consecutive prefixes per thread, one block scan
  constexpr int kPer = (4 << kW1) / NT;
  int cnt = 0;
  uint32_t longmask = 0;
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    const int i = t * kPer + j, q = i >> kW1, k = i & ((1 << kW1) - 1);
    const uint32_t e = q < ns ? g->lut[(q << 11) + (k << 2)] : 0u;
    const int l = e & 15;
    const bool lng = q < ns && (l == 0 || l > kW1);
    longmask |= lng ? 1u << j : 0u;
    cnt += lng ? 1 : 0;
  }
  int total;
  int base = block_excl_scan<NT>(cnt, tmp, &total);
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    const int i = t * kPer + j, q = i >> kW1, k = i & ((1 << kW1) - 1);
    const bool ac = q < ns && (g->slot_src[q] & 4);
    uint32_t e = q < ns ? write_entry(g->lut[(q << 11) + (k << 2)], ac) : 0u;
    if ((longmask >> j) & 1) {
      const int sub = base++;
      if (sub < kW2Cap / 4) {
        for (int m = 0; m < 4; m++) W.l2[sub * 4 + m] = (uint16_t)write_entry(g->lut[(q << 11) + (k << 2) + m], ac);
        e = (uint32_t)(sub + 1) << 4;
      } else {
        e = 0;  // no second level left: the canonical search
      }
    }
    W.lut[i] = (uint16_t)e;
  }
  for (int i = t; i < 4 * 18; i += NT) {
    W.maxcode[i / 18][i % 18] = g->maxcode[i / 18][i % 18];
    W.valoff[i / 18][i % 18] = g->valoff[i / 18][i % 18];
  }
  const uint32_t* gv = reinterpret_cast<const uint32_t*>(g->vals);
  uint32_t* wvls = reinterpret_cast<uint32_t*>(W.vals);
  for (int i = t; i < 4 * 64; i += NT) wvls[i] = gv[i];
  if (t == 0) {
    W.pk_dc[0] = g->pk_dc[0];
    W.pk_dc[1] = g->pk_dc[1];
    W.pk_ac[0] = g->pk_ac[0];
    W.pk_ac[1] = g->pk_ac[1];
    W.pk_c = g->pk_c;
  }
  __syncthreads();
  return ns;
}

template <int LB>
__device__ void entwrite_image(int img, int grp, ImgDesc* __restrict__ descs, const EntTables* __restrict__ tables,
                               uint8_t* __restrict__ scratch) {
  ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK) return;
  using TT = std::conditional_t<LB == 11, WriteTables, LutTables>;
  __shared__ LdsWriteT<TT> L;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  int ns;
  if constexpr (LB == 11) ns = load_write_tables(L.T, &tables[d->etab], reinterpret_cast<int32_t*>(L.stage));
  else ns = load_tables<LB>(L.T, &tables[d->etab]);
  if (!variant_owns<LB>(ns)) return;
  {
    uint4* z4 = reinterpret_cast<uint4*>(L.stage);
    for (int i = t; i < kEntThreads * kStageStride * 2 / 16; i += kEntThreads) z4[i] = make_uint4(0, 0, 0, 0);
  }
  if (t == 0) {
    L.bad = 0;
    L.sym = 0;
    L.it = 0;
    if (kStats) L.t0 = __builtin_amdgcn_s_memtime();
  }
  __syncthreads();
  const TT& T = L.T;
  const BlkCtx K = make_ctx(T, d->bpm);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(scratch + d->off_ustream);
  const SegView sv = seg_view(scratch + d->off_seg, d->nseg);
  const SubState* sub = reinterpret_cast<const SubState*>(scratch + d->off_sub);
  int16_t* coef = reinterpret_cast<int16_t*>(scratch + d->off_coef);
  const int nsub = d->nsub;
  const int blocks_per_seg = d->restart_interval ? d->restart_interval * K.bpm : (int)d->total_blocks;
  const int ncomp = d->ncomp;
  const int my_base = t * kStageStride;
  int bad = 0;
  unsigned long long nsym = 0, witers = 0;

  const int G = d->ent_groups, per = (nsub + G - 1) / G, j0 = grp * per, j1 = j0 + per < nsub ? j0 + per : nsub;
  for (int jb = j0; jb < j1; jb += kEntThreads) {  // uniform trip count for the whole workgroup
    const int j = jb + t;
    const bool active = j < j1;
    BitsQ<kQW> b;
    int blk = 0, z = 0, c = 0, p0 = 0, p1 = 0, p2 = 0, pc = 0, sdc = 0, sac = 0;
    bool chg = false;
    int g = 0, gend = 0;  // decode-order block indices (total_blocks < 2^24, setup_geometry)
    uint32_t end_bit = 0, lim = 0;
    int s_int = 0;
    bool last_of_seg = false, run = false;
    uint32_t stop_pos = 0, stop_blk = 0;
    if (active) {
      const SubState& S = sub[j];
      const int s = S.seg;
      const int g0 = s * blocks_per_seg;
      gend = g0 + blocks_per_seg;
      if (gend > (int)d->total_blocks) gend = (int)d->total_blocks;
      g = g0 + S.nblk_ex;
      p0 = S.dc_ex[0];
      p1 = S.dc_ex[1];
      p2 = S.dc_ex[2];
      // entries are block boundaries (z = 0): the speculative and the sync passes stop only there.  The
      // pass relies on that invariant (z starts at 0, no mid-block entry state); an entry that breaks it
      // fails the image (CORRUPT) instead of writing wrong coefficients
      blk = S.entry_bz >> 8;
      z = 0;
      if (S.entry_bz & 0xFF) d->status = SDSJ_CORRUPT;
      c = ctx_c(K, blk);
      if constexpr (LB == 11) {
        // predictors in component order from the entry block's component: pc = its own, p0 / p1 the
        // next ones (cyclically); a block after which the component changes rotates them (ctx_w5)
        // (the scan's component order, which the MCU follows, need not be the components' index order)
        ctx_w5(K, blk, sdc, sac, chg);
        int succ[kMaxComp] = {0, 0, 0};
        for (int b = 0; b < K.bpm; b++) {
          const int cb = ctx_c(K, b), cn = ctx_c(K, b + 1 == K.bpm ? 0 : b + 1);
          if (cn != cb) succ[cb] = cn;
        }
        auto pred = [&](int k) { return k == 0 ? p0 : (k == 1 ? p1 : p2); };
        const int c1 = succ[c], c2 = succ[c1];
        const int pa = pred(c), pb = pred(c1), pd = pred(c2);
        pc = pa;
        p0 = pb;
        p1 = pd;
      } else {
        sdc = ctx_dc(K, blk);
        sac = ctx_ac(K, blk);
        pc = c == 0 ? p0 : (c == 1 ? p1 : p2);  // the current block's component predictor
      }
      end_bit = S.end_bit;
      s_int = s;
      lim = S.lim_bit;
      last_of_seg = (j + 1 == nsub) || sub[j + 1].first;
      bits_init(b, src, S.entry_p, S.lim_bit);
      // the interval's last subsequence decodes every remaining block; when its data runs out
      // (bits past lim, read as zeros) it finishes that MCU and stops: jdhuff.c insufficient_data
      run = g < gend && (S.entry_bz & 0xFF) == 0 &&
            (last_of_seg ? !(z == 0 && blk == 0 && b.pos > lim) : (b.pos < end_bit || z != 0));
      // one stop rule for both kinds: at a block boundary (z = 0) whose MCU position blk is in stop_blk
      // (the interval's last subsequence: MCU boundaries only) once pos >= stop_pos
      stop_pos = last_of_seg ? lim + 1 : end_bit;
      stop_blk = last_of_seg ? 1u : 0xFFFFFFFFu;
    }
    // A completed block waits in its lane's stage for the next flush step (every kFlushEvery steps of
    // the group), and the lane decodes nothing until then: a flush per step cost as much as the
    // decode itself (some lane of the wave completes a block at almost every step).  The block-end
    // bookkeeping (predictors, MCU position and context, block index, stop rule) runs there too, once
    // per flush instead of as selects on every step.
    bool pending = false;
    while (__builtin_amdgcn_ballot_w64(run)) {
      if (run) bits_fill(b);
      for (;;) {
#pragma unroll
       for (int u = 0; u < kWriteGroup; u++) {
        if (kStats) witers++;
        if (run && !pending) {
          const bool isdc = z == 0;
          int val;
          bool done;
          if constexpr (LB == 11) {
            int s, adv;
            decode_wsym<11>(T, b, isdc ? sdc : sac, isdc, s, adv, val, bad);
            if (kStats) nsym++;
            // DC: predictor update (jdhuff.c last_dc_val); AC value at natural_order[k + r], k + r =
            // k + advance - 1 (jpeg_natural_order's guard entries send positions past 63 to 63).  EOB
            // (advance 64: position 63) and ZRL symbols (s = 0, val = 0) store a zero at a position of the
            // block not written yet (positions only grow within a block, and a clamped store ends it), so
            // every symbol stores
            pc += isdc ? val : 0;
            const int zn = z + adv, wpos = zn < 64 ? zn - 1 : 63;
            L.stage[my_base + wpos] = (int16_t)(isdc ? pc : val);
            // block end by selects (no branches): the component's predictor back, the next block's out
            done = zn > 63;
            z = done ? 0 : zn;
          } else {
            int s, r, sb = 0;
            decode_sym<LB>(T, b, isdc ? sdc : sac, isdc, s, r, val, sb);
            if (kStats) nsym++;
            bad |= sb;
            pc += isdc ? val : 0;
            const int zp = z + r, wpos = zp < 63 ? zp : 63;
            L.stage[my_base + wpos] = (int16_t)(isdc ? pc : val);
            done = next_z(z, s, r);
          }
          pending = done;
        }
        // cooperative flush of the blocks completed since the last flush: 8 lanes x 16 B per block
        const uint64_t m = u % kFlushEvery == kFlushEvery - 1 ? __builtin_amdgcn_ballot_w64(pending) : 0ull;
        if (m) {
          const int cnt = __popcll(m);
          if (pending) {
            const int idx = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            L.flist[wv][idx] = ((uint32_t)t << 24) | (uint32_t)g;
            // the block end: the component's predictor back, the next block's out
            if constexpr (LB == 11) {
              // (pc, p0, p1) -> (p0, p1, pc) with 3 components in the scan, (pc, p0) -> (p0, pc) with 2
              if (chg) {
                const int t0 = pc;
                pc = p0;
                p0 = ncomp == 3 ? p1 : t0;
                p1 = ncomp == 3 ? t0 : p1;
              }
              blk = blk + 1 == K.bpm ? 0 : blk + 1;
              ctx_w5(K, blk, sdc, sac, chg);
            } else {
              p0 = c == 0 ? pc : p0;
              p1 = c == 1 ? pc : p1;
              p2 = c == 2 ? pc : p2;
              blk = blk + 1 == K.bpm ? 0 : blk + 1;
              c = ctx_c(K, blk);
              sdc = ctx_dc(K, blk);
              sac = ctx_ac(K, blk);
              pc = c == 0 ? p0 : (c == 1 ? p1 : p2);
            }
            g++;
            // the stop rule at this block boundary (stop_blk: every block, or MCU starts)
            run = (g < gend) & !(((stop_blk != 1u) | (blk == 0)) & (b.pos >= stop_pos));
          }
          // (a wave's LDS accesses execute in issue order: the reads below see these writes, and the
          // owner's next stage writes land after the clears -- no waits beyond the data dependences)
          __builtin_amdgcn_wave_barrier();
          for (int b0 = 0; b0 < cnt; b0 += 8) {
            const int bi = b0 + (lane >> 3);
            if (bi < cnt) {
              const uint32_t f = L.flist[wv][bi];
              uint4* sp = reinterpret_cast<uint4*>(L.stage + (f >> 24) * kStageStride) + (lane & 7);
              const uint4 v = *sp;
              store_coef16(reinterpret_cast<uint4*>(coef + (int64_t)(f & 0xFFFFFF) * 64) + (lane & 7), v);
              *sp = make_uint4(0, 0, 0, 0);
            }
          }
          __builtin_amdgcn_wave_barrier();
          pending = false;
        }
       }
        if (__builtin_amdgcn_ballot_w64(run && bits_avail(b) < kRefillWrite) ||
            !__builtin_amdgcn_ballot_w64(run))
          break;
      }
    }
    if (active && last_of_seg) {
      if (g < gend) sv.vend[s_int] = g;                     // the rest of the interval stays zero
      if (b.pos > lim) sv.flag[s_int] |= kSegIns;          // ran out of data (JWRN_HIT_MARKER)
    }
  }
  if (bad) atomicOr(&L.bad, 1);  // bad Huffman codes: libjpeg warns and decodes symbol 0 (statistics only)
  if (kStats) {
    atomicAdd(&L.sym, nsym);
    if (lane == 0) atomicAdd(&L.it, 64ull * witers);
  }
  __syncthreads();
  if (kStats && t == 0 && grp == 0) {  // statistics: the first group's share
    d->sym_write = (int64_t)L.sym;
    d->it_write = (int64_t)L.it;
    d->t_write = (int64_t)(__builtin_amdgcn_s_memtime() - L.t0);
  }
}


template <int LB, int PHASE, int NTS = kSyncThreads, int NSPEC = kEntThreads>
__device__ __forceinline__ void ent_phase(int img, int grp, ImgDesc* descs, const EntTables* tables, uint8_t* scratch) {
  if (PHASE == 0) entspec_image<LB, NSPEC>(img, grp, descs, tables, scratch);
  else if (PHASE == 1) entsync_image<LB, NTS>(img, descs, tables, scratch);
  else entwrite_image<LB>(img, grp, descs, tables, scratch);
}

// The entropy kernels take images from a route list.  MODE 0: one workgroup per list entry (grid =
// batch size, surplus workgroups exit at once) -- the main route (LB = 11, one group per image).
// MODE 1: a small grid strides over the list and runs each image's groups in turn (LB = 10).  MODE 3:
// (image, group) tasks of the LB = 11 images with ent_groups > 1, a grid of at most kTaskGrid
// workgroups striding over them.  The sync pass is per image (MODE 0 for them too).
template <int LB, int PHASE, int RT, int MODE, int NTS = kSyncThreads, int NSPEC = kEntThreads>
__device__ __forceinline__ void ent_feed(ImgDesc* descs, const EntTables* tables, uint8_t* scratch, int32_t* routes,
                                         int cap) {
  if (MODE == 3) {  // (image, group) tasks (k_plan's group_tasks list); a capped grid strides over them
    const int nt = routes[kRtEnt11G];
    const int32_t* tasks = group_tasks(routes, cap);
    for (int k = blockIdx.x; k < nt; k += gridDim.x) {
      const int task = tasks[k];
      ent_phase<LB, PHASE, NTS, NSPEC>(task >> kGroupShift, task & ((1 << kGroupShift) - 1), descs, tables, scratch);
      __syncthreads();  // LDS reuse by the next task
    }
    return;
  }
  const int cnt = routes[RT];
  const int32_t* list = route_list(routes, cap, RT);
  if (MODE == 0) {  // one entry per workgroup at the full grid; a cold route's small grid strides (route_grid)
    for (int li = blockIdx.x; li < cnt; li += gridDim.x) {
      ent_phase<LB, PHASE, NTS, NSPEC>(list[li], 0, descs, tables, scratch);
      __syncthreads();  // LDS reuse by the next entry
    }
    return;
  }
  for (int li = blockIdx.x; li < cnt; li += gridDim.x) {
    const int img = list[li];
    const int G = PHASE == 1 ? 1 : descs[img].ent_groups;
    if (MODE == 2) {
      if ((int)blockIdx.y < G) ent_phase<LB, PHASE, NTS, NSPEC>(img, blockIdx.y, descs, tables, scratch);
    } else {
      for (int grp = 0; grp < G; grp++) {
        ent_phase<LB, PHASE, NTS, NSPEC>(img, grp, descs, tables, scratch);
        __syncthreads();  // LDS reuse by the next group
      }
    }
    __syncthreads();  // LDS reuse by the next image
  }
}

// k_entspec: subsequence layout + speculative pass (warm-up, records); k_entsync: sync rounds +
// segmented scan, decode tables built only when some entry disagrees with its predecessor's exit.
template <int LB, int RT, int MODE, int NSPEC = kEntThreads>
__global__ void __launch_bounds__(NSPEC) __attribute__((amdgpu_waves_per_eu(LB == 11 ? SDSJ_SPEC_WAVES : 5)))
k_entspec(ImgDesc* __restrict__ descs, const EntTables* __restrict__ tables, uint8_t* __restrict__ scratch,
          int32_t* __restrict__ routes, int cap) {
  ent_feed<LB, 0, RT, MODE, kSyncThreads, NSPEC>(descs, tables, scratch, routes, cap);
}

// Subsequences per lane of the speculative pass (one warm-up for the lane's run of them): the main
// route (one workgroup per image, kEntThreads / SDSJ_SPEC_SUBS threads) and the multi-group route.
#ifndef SDSJ_SPEC_SUBS
#define SDSJ_SPEC_SUBS 2
#endif
#ifndef SDSJ_SPEC_SUBS_G
#define SDSJ_SPEC_SUBS_G 1
#endif
constexpr int kSpecThreads = kEntThreads / SDSJ_SPEC_SUBS;
constexpr int kSpecThreadsG = kEntThreads / SDSJ_SPEC_SUBS_G;

// (multi-group images have several times the sync tasks: a 4-wave workgroup runs them)
template <int LB, int RT, int MODE, int NTS>
__global__ void __launch_bounds__(NTS) k_entsync(ImgDesc* __restrict__ descs, const EntTables* __restrict__ tables,
                                                 uint8_t* __restrict__ scratch, int32_t* __restrict__ routes, int cap) {
  ent_feed<LB, 1, RT, MODE, NTS>(descs, tables, scratch, routes, cap);
}

template <int LB, int RT, int MODE>
__global__ void __launch_bounds__(kEntThreads) k_entwrite(ImgDesc* __restrict__ descs, const EntTables* __restrict__ tables,
                                                          uint8_t* __restrict__ scratch, int32_t* __restrict__ routes,
                                                          int cap) {
  ent_feed<LB, 2, RT, MODE>(descs, tables, scratch, routes, cap);
}

// ------------------------------------------------------------------------------------------
// Latency mode, multi-hypothesis speculative pass (ImgDesc::mh: one image per call, no restart
// intervals).  A lane's speculative decode locks on to the true MCU phase only after ~1k bits (its
// Huffman codes self-synchronise within ~100 bits, the block phase much later), hence kLatWarm bits
// of warm-up per subsequence -- 80 % of a lane's serial chain.  Here each subsequence j is decoded by
// bpm lanes, lane h assuming MCU block h at its warm-up's first bit, from only kMhWarm bits before the
// subsequence: the lane whose assumption was right has re-aligned its codes and its coefficient index
// by the subsequence's start (at the first end of block), so its entry is the true one.  k_mh_select
// then picks per subsequence the phase whose entry equals the chosen predecessor's exit (a scan of
// phase maps), and k_entsync re-decodes the rare subsequences where none did.
// ------------------------------------------------------------------------------------------
struct MhRes {  // one (subsequence, phase) lane's speculative result (scratch at off_rec, unused by mh images)
  uint32_t entry_p, exit_p;
  uint16_t entry_bz, exit_bz;
  int32_t nblk;
  int32_t dc[kMaxComp];
  int32_t pad;
};
static_assert(sizeof(MhRes) * kMhMaxPhases <= sizeof(SyncRec) * kRec, "MhRes fit a subsequence's record scratch");

// The mh image's subsequences (one segment): [b0 + j SB, min(b0 + (j + 1) SB, b1)).
struct MhLayout {
  uint32_t b0, b1, sb;
  int nsub;
};
__device__ __forceinline__ MhLayout mh_layout(const ImgDesc* d, const SegView& sv) {
  MhLayout m;
  m.b0 = (uint32_t)sv.lo[0] * 8u;
  m.b1 = (uint32_t)sv.hi[0] * 8u;
  if (m.b1 < m.b0) m.b1 = m.b0;
  m.sb = (uint32_t)d->sub_bits;
  const int cnt = m.b1 > m.b0 ? (int)((m.b1 - m.b0 + m.sb - 1) / m.sb) : 1;
  m.nsub = cnt < d->nsub_cap ? cnt : d->nsub_cap;
  return m;
}

template <int RT>
__global__ void __launch_bounds__(kEntThreads) __attribute__((amdgpu_waves_per_eu(SDSJ_SPEC_WAVES)))
k_entspec_mh(ImgDesc* __restrict__ descs, const EntTables* __restrict__ tables, uint8_t* __restrict__ scratch,
             int32_t* __restrict__ routes, int cap) {
  if ((int)blockIdx.x >= routes[RT]) return;
  const int img = route_list(routes, cap, RT)[blockIdx.x];
  ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK || !d->mh) return;
  __shared__ LdsSpec<11, kEntThreads> L;
  if (!variant_owns<11>(load_tables(L.T, &tables[d->etab]))) return;
  const BlkCtx K = make_ctx(L.T, d->bpm);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(scratch + d->off_ustream);
  const SegView sv = seg_view(scratch + d->off_seg, d->nseg);
  MhRes* res = reinterpret_cast<MhRes*>(scratch + d->off_rec);
  const MhLayout m = mh_layout(d, sv);
  const int H = d->bpm;
  for (int i = blockIdx.y * kEntThreads + threadIdx.x; i < m.nsub * H; i += gridDim.y * kEntThreads) {
    const int j = i / H, h = i - j * H;
    MhRes r{};
    if (j > 0 || h == 0) {  // (the first subsequence starts exactly: block 0)
      SubState S;
      S.start_bit = m.b0 + (uint32_t)j * m.sb;
      const uint32_t e = S.start_bit + m.sb;
      S.end_bit = e < m.b1 ? e : m.b1;
      S.first = j == 0;
      S.seg = 0;
      S.lim_bit = m.b1;
      spec_pass<11>(L.T, K, src, S, nullptr, m.b0, (uint32_t)kMhWarm, false, 0u, 0, h, false);
      r.entry_p = S.entry_p;
      r.entry_bz = S.entry_bz;
      r.exit_p = S.spec_exit_p;
      r.exit_bz = S.spec_exit_bz;
      r.nblk = S.spec_nblk;
      for (int c = 0; c < kMaxComp; c++) r.dc[c] = S.spec_dc[c];
    }
    res[i] = r;
  }
}

// Per image (one workgroup): f_j(x) = the phase of subsequence j whose entry equals the exit of phase x
// of subsequence j - 1 (0 when none does: k_entsync re-decodes it); F_j = f_j o ... o f_1 from phase 0
// of subsequence 0 (an inclusive scan of maps: 4 bits per phase), j's phase = F_j(0).  Writes the
// chosen results into the SubStates as the speculative pass would (no records).  The lanes' entries
// and exits are staged in LDS by chunks of kMhStage (subsequence, phase) pairs.
constexpr int kMhStage = 3072;
__device__ __forceinline__ uint64_t mh_compose(uint64_t later, uint64_t earlier, int H) {
  uint64_t r = 0;
  for (int x = 0; x < H; x++) r |= ((later >> (4 * ((earlier >> (4 * x)) & 15))) & 15) << (4 * x);
  return r;
}
__device__ __forceinline__ uint64_t mh_key(uint32_t p, uint16_t bz) { return ((uint64_t)p << 16) | bz; }

template <int RT>
__global__ void __launch_bounds__(kEntThreads) k_mh_select(ImgDesc* __restrict__ descs, uint8_t* __restrict__ scratch,
                                                           int32_t* __restrict__ routes, int cap) {
  if ((int)blockIdx.x >= routes[RT]) return;
  const int img = route_list(routes, cap, RT)[blockIdx.x];
  ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK || !d->mh) return;
  __shared__ uint64_t ent[kMhStage], ext[kMhStage], F[kMhStage];
  __shared__ uint8_t pick[kMhStage];
  __shared__ uint64_t carry, prev_ext[kMhMaxPhases];
  const int t = threadIdx.x;
  const SegView sv = seg_view(scratch + d->off_seg, d->nseg);
  const MhRes* res = reinterpret_cast<const MhRes*>(scratch + d->off_rec);
  SubState* sub = reinterpret_cast<SubState*>(scratch + d->off_sub);
  const MhLayout m = mh_layout(d, sv);
  const int H = d->bpm, cs = kMhStage / H;
  if (t == 0) carry = 0;  // F_{-1}: every phase -> 0 (subsequence 0 is entered exactly)
  for (int c0 = 0; c0 < m.nsub; c0 += cs) {
    const int nc = m.nsub - c0 < cs ? m.nsub - c0 : cs;
    for (int i = t; i < nc * H; i += kEntThreads) {
      const MhRes& r = res[c0 * H + i];
      ent[i] = mh_key(r.entry_p, r.entry_bz);
      ext[i] = mh_key(r.exit_p, r.exit_bz);
    }
    __syncthreads();
    for (int i = t; i < nc * H; i += kEntThreads) {  // pair (k, x): the phase of k entered from phase x of k - 1
      const int k = i / H, x = i - k * H, j = c0 + k;
      int pk = 0;
      if (j > 0) {
        const uint64_t pe = k > 0 ? ext[(k - 1) * H + x] : prev_ext[x];
        for (int h = H - 1; h >= 0; h--) pk = ent[k * H + h] == pe ? h : pk;
      }
      pick[i] = (uint8_t)pk;
    }
    __syncthreads();
    for (int k = t; k < nc; k += kEntThreads) {
      uint64_t f = 0;
      for (int x = 0; x < H; x++) f |= (uint64_t)pick[k * H + x] << (4 * x);
      F[k] = f;
    }
    __syncthreads();
    for (int off = 1; off < nc; off <<= 1) {  // inclusive scan: F[k] = F[k] o F[k - off]
      uint64_t v[kMhStage / kEntThreads];
      for (int k = t, n = 0; k < nc; k += kEntThreads, n++) v[n] = k >= off ? mh_compose(F[k], F[k - off], H) : F[k];
      __syncthreads();
      for (int k = t, n = 0; k < nc; k += kEntThreads, n++) F[k] = v[n];
      __syncthreads();
    }
    const uint64_t cin = carry;
    for (int k = t; k < nc; k += kEntThreads) {
      const int j = c0 + k;
      const int h = j == 0 ? 0 : (int)(mh_compose(F[k], cin, H) & 15);  // F_j(0)
      const MhRes& r = res[j * H + h];
      SubState& S = sub[j];
      S.start_bit = m.b0 + (uint32_t)j * m.sb;
      const uint32_t e = S.start_bit + m.sb;
      S.end_bit = e < m.b1 ? e : m.b1;
      S.first = j == 0;
      S.seg = 0;
      S.lim_bit = m.b1;
      S.entry_p = r.entry_p;
      S.entry_bz = r.entry_bz;
      S.spec_exit_p = S.cur_exit_p = r.exit_p;
      S.spec_exit_bz = S.cur_exit_bz = r.exit_bz;
      S.spec_nblk = S.cur_nblk = r.nblk;
      for (int c = 0; c < kMaxComp; c++) S.spec_dc[c] = S.cur_dc[c] = r.dc[c];
      S.nrec = 0;
    }
    __syncthreads();
    if (t == 0) carry = mh_compose(F[nc - 1], cin, H);
    if (t < H) prev_ext[t] = ext[(nc - 1) * H + t];
    __syncthreads();
  }
  if (t == 0) d->nsub = m.nsub;
}

size_t enttab_bytes() { return sizeof(EntTables); }

constexpr int kTaskGrid = 4096;  // MODE 3 grid cap (>= the workgroups the chip holds at once)
static int task_grid(int n) { return n * kMaxEntGroups < kTaskGrid ? n * kMaxEntGroups : kTaskGrid; }

hipError_t launch_entspec(int n, ImgDesc* descs, const ImgTables* specs, void* etab, uint8_t* scratch, int32_t* routes,
                          int cap, hipStream_t s, uint64_t rm, bool small, uint64_t hint) {
  const int g = n;  // one workgroup per image on the main route
  EntTables* tables = static_cast<EntTables*>(etab);
  const int gs = g < 256 ? g : 256;
  if (route_on(rm, kRtEnt11) || route_on(rm, kRtEnt11M) || route_on(rm, kRtEnt10))
    hipLaunchKernelGGL(k_enttab, dim3(n), dim3(kEntThreads), 0, s, descs, specs, tables);
  if (route_on(rm, kRtEnt11))
    hipLaunchKernelGGL((k_entspec<11, kRtEnt11, 0, kSpecThreads>), dim3(route_grid(hint, kRtEnt11, g)), dim3(kSpecThreads), 0,
                       s, descs, tables, scratch, routes, cap);
  if (route_on(rm, kRtEnt11M))
    hipLaunchKernelGGL((k_entspec<11, kRtEnt11M, 3, kSpecThreadsG>), dim3(route_grid(hint, kRtEnt11M, task_grid(n))),
                       dim3(kSpecThreadsG), 0, s, descs, tables, scratch, routes, cap);
  if (route_on(rm, kRtEnt10))
    hipLaunchKernelGGL((k_entspec<10, kRtEnt10, 1>), dim3(route_grid(hint, kRtEnt10, gs)), dim3(kEntThreads), 0, s, descs,
                       tables, scratch, routes, cap);
  if (SDSJ_MH && small) {  // latency-mode images (ImgDesc::mh; the kernels above skip them)
    constexpr int kMhGridY = 64;
    if (route_on(rm, kRtEnt11)) {
      hipLaunchKernelGGL(k_entspec_mh<kRtEnt11>, dim3(n, kMhGridY), dim3(kEntThreads), 0, s, descs, tables, scratch, routes, cap);
      hipLaunchKernelGGL(k_mh_select<kRtEnt11>, dim3(n), dim3(kEntThreads), 0, s, descs, scratch, routes, cap);
    }
    if (route_on(rm, kRtEnt11M)) {
      hipLaunchKernelGGL(k_entspec_mh<kRtEnt11M>, dim3(n, kMhGridY), dim3(kEntThreads), 0, s, descs, tables, scratch, routes, cap);
      hipLaunchKernelGGL(k_mh_select<kRtEnt11M>, dim3(n), dim3(kEntThreads), 0, s, descs, scratch, routes, cap);
    }
  }
  return hipGetLastError();
}

hipError_t launch_entsync(int n, ImgDesc* descs, void* etab, uint8_t* scratch, int32_t* routes, int cap, hipStream_t s,
                          uint64_t rm, uint64_t hint) {
  const int g = n;
  EntTables* tables = static_cast<EntTables*>(etab);
  const int gs = g < 256 ? g : 256;
  if (route_on(rm, kRtEnt11))
    hipLaunchKernelGGL((k_entsync<11, kRtEnt11, 0, kSyncThreads>), dim3(route_grid(hint, kRtEnt11, g)), dim3(kSyncThreads), 0,
                       s, descs, tables, scratch, routes, cap);
  if (route_on(rm, kRtEnt11M))
    hipLaunchKernelGGL((k_entsync<11, kRtEnt11M, 0, kEntThreads>), dim3(route_grid(hint, kRtEnt11M, g)), dim3(kEntThreads), 0,
                       s, descs, tables, scratch, routes, cap);
  if (route_on(rm, kRtEnt10))
    hipLaunchKernelGGL((k_entsync<10, kRtEnt10, 1, kSyncThreads>), dim3(route_grid(hint, kRtEnt10, gs)), dim3(kSyncThreads), 0,
                       s, descs, tables, scratch, routes, cap);
  return hipGetLastError();
}

hipError_t launch_entwrite(int n, ImgDesc* descs, const void* etab, uint8_t* scratch, int32_t* routes, int cap,
                           hipStream_t s, uint64_t rm, uint64_t hint) {
  const int g = n;  // one workgroup per image on the main route
  const EntTables* tables = static_cast<const EntTables*>(etab);
  const int gs = g < 256 ? g : 256;
  if (route_on(rm, kRtEnt11))
    hipLaunchKernelGGL((k_entwrite<11, kRtEnt11, 0>), dim3(route_grid(hint, kRtEnt11, g)), dim3(kEntThreads), 0, s, descs,
                       tables, scratch, routes, cap);
  if (route_on(rm, kRtEnt11M))
    hipLaunchKernelGGL((k_entwrite<11, kRtEnt11M, 3>), dim3(route_grid(hint, kRtEnt11M, task_grid(n))), dim3(kEntThreads), 0,
                       s, descs, tables, scratch, routes, cap);
  if (route_on(rm, kRtEnt10))
    hipLaunchKernelGGL((k_entwrite<10, kRtEnt10, 1>), dim3(route_grid(hint, kRtEnt10, gs)), dim3(kEntThreads), 0, s, descs,
                       tables, scratch, routes, cap);
  return hipGetLastError();
}

}  // namespace sdsj
