// sdsj_progressive.hip -- progressive JPEG (SOF2, Huffman) for the MI355X path.
//
// Restates libjpeg-turbo's progressive decoder as Pillow runs it: jdphuff.c decode_mcu_DC_first /
// _AC_first / _DC_refine / _AC_refine with EOB runs and start_pass_phuff_decoder's progression
// checks, jdinput.c per-scan MCU geometry and latch_quant_tables, jdmarker.c read_markers between
// scans (DHT / DQT / DRI may change from one scan to the next) up to EOI, and the bit reader /
// restart / resynchronisation rules the baseline path shares (jdhuff.c jpeg_fill_bit_buffer,
// read_restart_marker + jpeg_resync_to_restart).  Each image's scans depend on one another, so one
// wave walks an image's whole file (its decoder state wave-uniform, in scalar registers) and its
// lanes split the work that is parallel within a block: the AC refinement scans coefficient by
// coefficient, the DC refinement scan block by block (k_prog).  The coefficients land in the same
// MCU-ordered array the baseline entropy kernels write, and k_idct / the resample kernels take it
// from there.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sdsj_common.h"
#include "sdsj_kernels.h"

namespace sdsj {

namespace {

// Bit reader over the stuffed stream (jdhuff.c jpeg_fill_bit_buffer semantics): FF00 -> FF, FF fill
// bytes skipped; a marker stops the data (zeros are fed from there); the input ending first is eof.
struct PBits {
  const uint8_t* d;
  int n, pos;  // (32-bit: the scans' data is far below 2 GB; fewer scalar registers)
  uint64_t buf;
  int nbits, hit_marker, marker, pad_bits, insufficient, eof;
  uintptr_t wbase;  // 16-byte window of the stream held in registers (one load per 16 bytes)
  uint4 w;
};

// The aligned 16 bytes around p (address a).  Addressed from p itself, not from the integer a: a
// pointer rebuilt from an integer is a flat pointer, whose loads the compiler must treat as
// per-lane values -- the whole bit reader then runs on vector registers under exec masks.  From
// the global pointer the window, and everything decoded from it, is wave-uniform.
__device__ __forceinline__ uint4 pwindow(const uint8_t* p, uintptr_t a) {
  return *reinterpret_cast<const uint4*>(p - (a & 15));
}

// Byte i of the stream (0 <= i < n) through the window: the aligned 16 bytes around it come in as
// one load (the blob allocation holds the whole granule).
__device__ __forceinline__ int pbyte(PBits& b, int i) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(b.d + i), base = a & ~(uintptr_t)15;
  if (base != b.wbase) {
    b.wbase = base;
    b.w = pwindow(b.d + i, a);
  }
  // (the window is picked from computed values, not from field loads: a select between loads of
  // b.w's fields becomes a select between their addresses, and the bit reader state then stays in
  // scratch memory instead of registers)
  const uint32_t o = (uint32_t)(a - base);
  const uint64_t lo = ((uint64_t)b.w.y << 32) | b.w.x, hi = ((uint64_t)b.w.w << 32) | b.w.z;
  return (int)((((o & 8) ? hi : lo) >> (8 * (o & 7))) & 0xFF);
}

__device__ __forceinline__ void pfill(PBits& b) {
  while (b.nbits <= 56) {
    // fast path: 4 bytes inside the window with no 0xFF among them go in at once
    if (b.nbits <= 32 && !b.hit_marker && b.pos + 4 <= b.n) {
      const uintptr_t a = reinterpret_cast<uintptr_t>(b.d + b.pos), base = a & ~(uintptr_t)15;
      const uint32_t o = (uint32_t)(a - base);
      if (o <= 12) {
        if (base != b.wbase) {
          b.wbase = base;
          b.w = pwindow(b.d + b.pos, a);
        }
        // bytes o .. o + 3 of the 16-byte window (a 128-bit shift; see pbyte)
        const uint64_t lo = ((uint64_t)b.w.y << 32) | b.w.x, hi = ((uint64_t)b.w.w << 32) | b.w.z;
        const uint32_t sh = 8 * (o & 7);
        const uint64_t q = (o & 8) ? hi >> sh : (sh ? (lo >> sh) | (hi << (64 - sh)) : lo);
        const uint32_t x = (uint32_t)q, t = ~x;
        if (((t - 0x01010101u) & ~t & 0x80808080u) == 0) {
          b.buf |= (uint64_t)__builtin_bswap32(x) << (32 - b.nbits);
          b.nbits += 32;
          b.pos += 4;
          continue;
        }
      }
    }
    int c;
    if (b.hit_marker || b.pos >= b.n) {
      if (!b.hit_marker) b.eof = 1;
      c = 0;
      b.pad_bits += 8;
    } else {
      c = pbyte(b, b.pos++);
      if (c == 0xFF) {
        int c2;
        do {
          c2 = b.pos < b.n ? pbyte(b, b.pos++) : -1;
        } while (c2 == 0xFF);
        if (c2 == 0) {
          c = 0xFF;
        } else if (c2 < 0) {
          b.pos = b.n;
          continue;
        } else {
          b.hit_marker = 1;
          b.marker = c2;
          b.pos -= 2;  // the marker stays for process_restart / read_markers
          continue;
        }
      }
    }
    b.buf |= (uint64_t)c << (56 - b.nbits);
    b.nbits += 8;
  }
}

// n (1..32) bits the caller knows are in the buffer (phuff left >= 32 after its symbol's start)
__device__ __forceinline__ int pgetbits_nc(PBits& b, int n) {
  const int v = (int)(b.buf >> (64 - n));
  b.buf <<= n;
  b.nbits -= n;
  if (b.nbits < b.pad_bits) b.insufficient = 1;
  return v;
}

__device__ __forceinline__ int pgetbits(PBits& b, int n) {
  if (n == 0) return 0;
  if (b.nbits < n) pfill(b);
  const int v = (int)(b.buf >> (64 - n));
  b.buf <<= n;
  b.nbits -= n;
  if (b.nbits < b.pad_bits) b.insufficient = 1;  // consumed inserted zeros (JWRN_HIT_MARKER)
  return v;
}

// The lookahead tables of the scan being decoded, in LDS (one slot per lane = per image); the
// canonical bounds and symbols that codes of more than 9 bits need stay in ProgTables (global
// memory: such codes are rare, and 4.3 KB of LDS per image instead of 7.4 KB lets more images run
// per CU).
struct PLds {
  uint16_t look[4][1 << 9];  // per scan position: (length << 8) | symbol of the codes of <= 9 bits, 0 = longer
  int32_t qh[4], qv[4], qbo[4], qdsl[4], ldc[4];  // interleaved DC scans: per scan position h, v, block
                                                  // offset in the MCU, DC table slot, DC predictor
  int32_t ins_m;  // the MCU in which the scan ran out of data (-1: none); in LDS, off the MCU loop's registers
};

// jdhuff.c jpeg_huff_decode: codes of <= 9 bits come from the scan position's lookahead table in one
// LDS read; longer (and bad) codes take the first l whose l-bit prefix is <= maxcode[l] (all 16
// compares issue together on 17 peeked bits); no match = bad code: 17 bits, symbol 0.  Bits are
// consumed only after the length is known, so insufficient_data follows the consumed count as with
// a bit-serial decode.
// The buffer holds >= 32 bits when the symbol starts, so its extra bits (<= 15, or 1 + a correction
// bit) need no second check.
__device__ __forceinline__ int phuff(PBits& b, const PLds& L, const ProgTables* __restrict__ T, int slot, int q) {
  if (b.nbits < 32) pfill(b);
  const uint32_t e = L.look[q][(uint32_t)(b.buf >> 55)];
  if (e) {
    const int l = (int)(e >> 8);
    b.buf <<= l;
    b.nbits -= l;
    if (b.nbits < b.pad_bits) b.insufficient = 1;
    return (int)(e & 0xFF);
  }
  const uint32_t peek = (uint32_t)(b.buf >> 47);
  int l = 17;
#pragma unroll
  for (int k = 16; k >= 10; k--) l = (int32_t)(peek >> (17 - k)) <= T->maxcode[slot][k] ? k : l;
  b.buf <<= l;
  b.nbits -= l;
  if (b.nbits < b.pad_bits) b.insufficient = 1;
  if (l > 16) return 0;
  return T->vals[slot][((int32_t)(peek >> (17 - l)) + T->valoff[slot][l]) & 0xFF];
}

__device__ __forceinline__ int pextend(int x, int s) { return x < (1 << (s - 1)) ? x + (int)((~0u << s) + 1) : x; }

// jdmarker.c next_marker from the byte cursor: pos ends on the marker's last FF; -1 at the end
__device__ __forceinline__ int pnext_marker(PBits& b) {
  for (;;) {
    while (b.pos < b.n && pbyte(b, b.pos) != 0xFF) b.pos++;
    if (b.pos >= b.n) return -1;
    int p = b.pos + 1;
    while (p < b.n && pbyte(b, p) == 0xFF) p++;
    if (p >= b.n) return -1;
    const int m = pbyte(b, p);
    if (m != 0) {
      b.pos = p - 1;
      return m;
    }
    b.pos = p + 1;
  }
}

__device__ __forceinline__ void pconsume_marker(PBits& b) {
  b.pos += 2;
  b.hit_marker = 0;
  b.marker = 0;
}

// read_restart_marker + jpeg_resync_to_restart (actions 1 / 2 / 3); -1 when the input ends first
__device__ __forceinline__ int pread_restart(PBits& b, int desired) {
  if (!b.hit_marker) {
    const int m = pnext_marker(b);
    if (m < 0) return -1;
    b.hit_marker = 1;
    b.marker = m;
  }
  if (b.marker == 0xD0 + desired) {
    pconsume_marker(b);
    return 0;
  }
  for (;;) {
    const int m = b.marker;
    int action;
    if (m < 0xC0) action = 2;
    else if (m < 0xD0 || m > 0xD7) action = 3;
    else if (m == 0xD0 + ((desired + 1) & 7) || m == 0xD0 + ((desired + 2) & 7)) action = 3;
    else if (m == 0xD0 + ((desired - 1) & 7) || m == 0xD0 + ((desired - 2) & 7)) action = 2;
    else action = 1;
    if (action == 1) {
      pconsume_marker(b);
      return 0;
    }
    if (action == 3) return 0;
    pconsume_marker(b);
    const int m2 = pnext_marker(b);
    if (m2 < 0) return -1;
    b.hit_marker = 1;
    b.marker = m2;
  }
}

__device__ __forceinline__ int pprocess_restart(PBits& b, int* next_num) {
  b.buf = 0;
  b.nbits = 0;
  b.pad_bits = 0;
  if (pread_restart(b, *next_num)) return -1;
  *next_num = (*next_num + 1) & 7;
  if (!b.hit_marker) b.insufficient = 0;
  return 0;
}

__device__ __forceinline__ int rd16(const uint8_t* p) { return (p[0] << 8) | p[1]; }

// jdhuff.c jpeg_make_d_derived_tbl for slot (0..3 DC, 4..7 AC) and scan position q: canonical
// bounds plus the 9-bit lookahead table (entry x: the code of length l <= 9 that is x's l-bit
// prefix, found like jpeg_huff_decode's search; the lanes fill 8 entries each); false when the code
// assignment overflows (JERR_BAD_HUFF_TABLE), or a DC table holds a symbol > 15
__device__ __forceinline__ bool pderive(ProgTables* P, PLds& L, int slot, int q, int lane) {
  if (!P->defined[slot]) return false;
  int code = 0, p = 0;
  int mc[10], vo[10];
#pragma unroll
  for (int l = 1; l <= 16; l++) {
    const int cnt = P->bits[slot][l];
    const int m = cnt ? code + cnt - 1 : -1, o = cnt ? p - code : 0;
    P->maxcode[slot][l] = m;
    P->valoff[slot][l] = o;
    if (l <= 9) {
      mc[l] = m;
      vo[l] = o;
    }
    p += cnt;
    code += cnt;
    if (cnt && code >= (1 << l)) return false;  // (the all-ones code is reserved)
    code <<= 1;
  }
  if (p > 256) return false;
  if (slot < 4)
    for (int i = 0; i < p; i++)
      if (P->vals[slot][i] > 15) return false;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int x = lane + 64 * k;
    int ls = 0, vi = 0;  // (selects, no branches: one symbol load per entry)
#pragma unroll
    for (int l = 9; l >= 1; l--) {
      const int c = x >> (9 - l);
      const bool hit = c <= mc[l];
      ls = hit ? l : ls;
      vi = hit ? c + vo[l] : vi;
    }
    const int sym = P->vals[slot][vi & 0xFF];
    L.look[q][x] = (uint16_t)(ls ? (ls << 8) | sym : 0);
  }
  return true;
}

// get_dht / get_dqt bodies
__device__ __forceinline__ int pread_dht(ProgTables* P, const uint8_t* s, int sl) {
  int k = 0;
  while (k < sl) {
    if (k + 17 > sl) return SDSJ_CORRUPT;
    const int tc = s[k] >> 4, th = s[k] & 15;
    if (tc > 1 || th > 3) return SDSJ_CORRUPT;
    const int slot = tc * 4 + th;
    int cnt = 0;
    P->bits[slot][0] = 0;
    for (int l = 1; l <= 16; l++) {
      P->bits[slot][l] = s[k + l];
      cnt += s[k + l];
    }
    if (cnt > 256 || k + 17 + cnt > sl) return SDSJ_CORRUPT;
    for (int i = 0; i < 256; i++) P->vals[slot][i] = i < cnt ? s[k + 17 + i] : 0;
    P->defined[slot] = 1;
    k += 17 + cnt;
  }
  return SDSJ_OK;
}

__device__ __forceinline__ int pread_dqt(ProgTables* P, const uint8_t* s, int sl) {
  int k = 0;
  while (k < sl) {
    const int pq = s[k] >> 4, tq = s[k] & 15;
    if (tq > 3 || pq > 1) return SDSJ_CORRUPT;
    const int need = 1 + 64 * (pq ? 2 : 1);
    if (k + need > sl) return SDSJ_CORRUPT;
    for (int q = 0; q < 64; q++)
      P->qt[tq][natural_order(q)] = (uint16_t)(pq ? rd16(s + k + 1 + 2 * q) : s[k + 1 + q]);
    P->qt_defined[tq] = 1;
    k += need;
  }
  return SDSJ_OK;
}

// Blocks are kept in zigzag order (the order k_idct reads): zigzag index k is natural_order(k), and
// natural_order's guard entries past 63 are all 63.
__device__ __forceinline__ int zig(int k) { return k < 63 ? k : 63; }

// n (1..32) bits as an unsigned word (the correction bits of up to 32 coefficients at once)
__device__ __forceinline__ uint32_t pgetbits32(PBits& b, int n) {
  if (b.nbits < n) pfill(b);  // (pfill leaves >= 57 bits)
  const uint32_t v = (uint32_t)(b.buf >> (64 - n));
  b.buf <<= n;
  b.nbits -= n;
  if (b.nbits < b.pad_bits) b.insufficient = 1;
  return v;
}

// One block of a DC scan or an AC first scan (jdphuff.c decode_mcu_DC_first / _DC_refine / _AC_first).
__device__ __forceinline__ void pblock(PBits& b, const PLds& P, const ProgTables* __restrict__ T, int dslot, int aslot, int lq, int16_t* blk, int ss, int se,
                       int ah, int al, int* last_dc, int* eobrun) {
  if (ss == 0) {
    if (ah == 0) {  // decode_mcu_DC_first
      int s = phuff(b, P, T, dslot, lq);
      if (s) s = pextend(pgetbits_nc(b, s), s);
      s += *last_dc;
      *last_dc = s;
      blk[0] = (int16_t)((unsigned)s << al);
    } else if (pgetbits(b, 1)) {  // decode_mcu_DC_refine
      blk[0] = (int16_t)(blk[0] | (1 << al));
    }
    return;
  }
  // decode_mcu_AC_first
  if (*eobrun > 0) {
    (*eobrun)--;
    return;
  }
  for (int k = ss; k <= se; k++) {
    const int sym = phuff(b, P, T, aslot, lq);
    const int r = sym >> 4, s = sym & 15;
    if (s) {
      k += r;
      const int x = pgetbits_nc(b, s);
      blk[zig(k)] = (int16_t)((unsigned)pextend(x, s) << al);
    } else if (r == 15) {
      k += 15;
    } else {
      *eobrun = 1 << r;
      if (r) *eobrun += pgetbits_nc(b, r);
      (*eobrun)--;
      break;
    }
  }
}

// One block of an AC refinement scan (jdphuff.c decode_mcu_AC_refine), lane-parallel: the wave walks
// the block's symbols together (every lane decodes the same bits), and lane k holds the block's
// zigzag coefficient k in a register.  A ballot gives the mask of non-zero coefficients; the stop of
// a run of r zeros is the (r + 1)-th zero bit at or after k, and the non-zero coefficients passed on
// the way each take one correction bit -- read in chunks of up to 32, the i-th lowest position of a
// chunk taking its i-th bit from the top, each lane applying its own.
// A ballot as a wave-uniform value (readfirstlane on each half: the compiler then knows the mask,
// and everything the decode derives from it, is the same in every lane)
__device__ __forceinline__ uint64_t uballot(bool x) {
  const uint64_t m = __builtin_amdgcn_ballot_w64(x);
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(m >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)m);
}

__device__ __forceinline__ int prefine(PBits& b, const PLds& P, const ProgTables* __restrict__ T, int aslot, int v,
                                       int lane, int ss, int se, int al, int* eobrun) {
  const int p1 = 1 << al, m1 = -(1 << al);
  uint64_t nz = uballot(v != 0);
  const uint64_t band = se >= 63 ? ~0ull : ((1ull << (se + 1)) - 1);  // positions <= se
  const uint64_t lower = (1ull << lane) - 1;                           // positions below this lane's
  auto below = [](int z) { return z >= 64 ? ~0ull : ((1ull << z) - 1); };
  // correction bits for the non-zero coefficients flagged in span (jdphuff.c: a 1 adds p1 away
  // from zero unless that bit is already set)
  auto correct = [&](uint64_t span) {
    while (span) {
      // (min() here resolves to the double overload; an integer select measured 12 % slower overall
      // -- code generation, profiles/r03e_prog_lanes_ab.txt -- so it stays)
      const int cnt = min(__popcll(span), 32);
      const uint32_t bits = pgetbits32(b, cnt);
      const int rank = __popcll(span & lower);
      const bool mine = ((span >> lane) & 1) != 0 && rank < cnt;
      if (mine && ((bits >> (cnt - 1 - rank)) & 1) && (v & p1) == 0) v = v >= 0 ? v + p1 : v - p1;
      span &= ~uballot(mine);
    }
  };
  int k = ss;
  if (*eobrun == 0) {
    for (; k <= se; k++) {
      const int sym = phuff(b, P, T, aslot, 0);
      const int r = sym >> 4;
      int s = sym & 15;
      if (s) {
        s = pgetbits_nc(b, 1) ? p1 : m1;  // (s != 1: JWRN_HUFF_BAD_CODE, decoding goes on)
      } else if (r != 15) {
        *eobrun = 1 << r;
        if (r) *eobrun += pgetbits_nc(b, r);
        break;
      }
      // skip r zero coefficients (correcting the non-zero ones passed), stop on the next zero: the
      // zero lane of rank r among the zero lanes in [k, se] (v != 0 exactly where nz has a bit)
      int z;
      {
        const bool zl = v == 0 && lane >= k && lane <= se;
        const uint64_t zeros = uballot(zl);
        z = __popcll(zeros) <= r ? se + 1 : __ffsll((unsigned long long)uballot(zl && __popcll(zeros & lower) == r)) - 1;
      }
      correct(nz & below(z) & (~0ull << k));
      k = z;
      if (s) {
        if (lane == zig(k)) v = s;
        nz |= 1ull << zig(k);
      }
    }
  }
  if (*eobrun > 0) {
    if (k <= se) correct(nz & band & (~0ull << k));
    (*eobrun)--;
  }
  return v;
}

// Every scan of image d, then the markers up to EOI.  Returns an SDSJ status.
__device__ __forceinline__ int decode_progressive(ImgDesc* d, ImgTables* t, const uint8_t* raw, int n, int16_t* coef,
                                  ProgTables* P, PLds& L, int lane) {
  // table state as k_parse left it (the DHT / DQT segments before the first SOS)
  for (int q = 0; q < 4; q++) {
    P->qt_defined[q] = t->qt_defined[q];
    for (int i = 0; i < 64; i++) P->qt[q][i] = t->qt[q][i];
    for (int k = 0; k < 2; k++) {
      const HuffSpec& h = k ? t->ac_spec[q] : t->dc_spec[q];
      const int slot = k * 4 + q;
      P->defined[slot] = h.defined;
      for (int l = 0; l <= 16; l++) P->bits[slot][l] = h.bits[l];
      for (int i = 0; i < 256; i++) P->vals[slot][i] = h.vals[i];
    }
  }
  for (int c = 0; c < kMaxComp; c++) P->latched[c] = 0;
  d->t_spec = d->t_sync = d->t_scan = d->t_write = 0;
#ifdef SDSJ_PROG_STATS
  d->sym_spec = d->sym_sync = d->sym_write = d->it_write = 0;
#endif
  // block smoothing state (jdphuff.c start_pass_phuff_decoder coef_bits / prev_coef_bits)
  d->smooth = 0;
  for (int c = 0; c < kMaxComp; c++)
    for (int k = 0; k < 10; k++) d->sm_bits[0][c][k] = d->sm_bits[1][c][k] = -1;
  int nscans = 0, good = 1 << 30;
  int restart_interval = d->restart_interval;
  // first block of components 1 and 2 within an MCU
  const int boff1 = d->ncomp > 1 ? d->comp[0].h * d->comp[0].v : 0;
  const int boff2 = d->ncomp > 2 ? boff1 + d->comp[1].h * d->comp[1].v : 0;
  int pos = (int)d->sos_pos;
  for (;;) {
    if (pos + 2 > n) return SDSJ_CORRUPT;
    const int len = rd16(raw + pos), sl = len - 2;
    if (len < 2 || pos + len > n) return SDSJ_CORRUPT;
    const uint8_t* s = raw + pos + 2;
    if (sl < 1) return SDSJ_CORRUPT;
    const int ns = s[0];
    if (ns < 1 || ns > 4 || sl != 2 * ns + 4) return SDSJ_CORRUPT;  // get_sos: JERR_BAD_LENGTH
    // (per-position arrays are indexed only from unrolled loops, so they stay in registers)
    int comps[4] = {0, 0, 0, 0}, td[4] = {0, 0, 0, 0}, ta[4] = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if (q >= ns) break;
      const int cid = s[1 + 2 * q];
      int c = 0;
      while (c < d->ncomp && d->comp_id[c] != cid) c++;
      if (c == d->ncomp) return SDSJ_CORRUPT;
      comps[q] = c;
      td[q] = s[2 + 2 * q] >> 4;  // checked only where the table is used (jpeg_make_d_derived_tbl)
      ta[q] = s[2 + 2 * q] & 15;
    }
    const int ss = s[1 + 2 * ns], se = s[2 + 2 * ns], ah = s[3 + 2 * ns] >> 4, al = s[3 + 2 * ns] & 15;
    bool bad = false;
    if (ss == 0) bad = se != 0;
    else bad = se < ss || se > 63 || ns != 1;
    if (ah != 0 && al != ah - 1) bad = true;
    if (al > 13) bad = true;
    if (bad) return SDSJ_CORRUPT;  // JERR_BAD_PROGRESSION
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if (q >= ns) break;
      const int c = comps[q], tq = d->comp[c].tq;
      if (!P->latched[c]) {  // latch_quant_tables: the component's table at its first scan
        if (!P->qt_defined[tq]) return SDSJ_CORRUPT;
        for (int i = 0; i < 64; i++) t->qt[c][i] = P->qt[tq][i];  // (k_idct reads slot c: see below)
        P->latched[c] = 1;
      }
      if (ss == 0 && ah == 0) {
        if (td[q] > 3 || !pderive(P, L, td[q], q, lane)) return SDSJ_CORRUPT;
      } else if (ss != 0) {
        if (ta[q] > 3 || !pderive(P, L, 4 + ta[q], q, lane)) return SDSJ_CORRUPT;
      }
      // coef_bits of the band (the smoothing reads coefficients 0..9), the previous values kept
      for (int k = ss < 1 ? ss : 1; k < 10; k++) d->sm_bits[1][c][k] = nscans > 0 ? d->sm_bits[0][c][k] : 0;
      for (int k = ss; k <= se && k < 10; k++) d->sm_bits[0][c][k] = (int8_t)al;
    }
    nscans++;
    good = 1 << 30;
    // the scan's geometry in registers (descriptor reads would repeat for every block: the
    // coefficient stores may alias them as far as the compiler knows)
    int sh[4] = {1, 1, 1, 1}, sv[4] = {1, 1, 1, 1}, sbw[4] = {0, 0, 0, 0}, sbo[4] = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if (q >= ns) break;
      sh[q] = d->comp[comps[q]].h;
      sv[q] = d->comp[comps[q]].v;
      sbw[q] = d->comp[comps[q]].bw;
      sbo[q] = comps[q] == 0 ? 0 : comps[q] == 1 ? boff1 : boff2;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      L.qh[q] = sh[q];
      L.qv[q] = sv[q];
      L.qbo[q] = sbo[q];
      L.qdsl[q] = td[q] & 3;
      L.ldc[q] = 0;
    }
    const int mcux = d->mcux, bpm = d->bpm, ncomp = d->ncomp;
    // jdinput.c per_scan_setup: a single-component scan walks that component's own block grid
    int nmcu, cwb = 0;
    if (ns == 1) {
      const CompDesc& cp = d->comp[comps[0]];
      cwb = (cp.dw + 7) / 8;
      nmcu = cwb * ((cp.dh + 7) / 8);
    } else {
      nmcu = mcux * d->mcuy;
    }
    PBits b;
    b.d = raw;
    b.n = n;
    b.pos = pos + len;
    b.buf = 0;
    b.nbits = b.hit_marker = b.marker = b.pad_bits = b.insufficient = b.eof = 0;
    b.wbase = 1;  // (no window yet: never 16-byte aligned)
    int ldc0 = 0, eobrun = 0;  // (a single-component scan's DC predictor; interleaved ones: L.ldc)
    int restarts_left = restart_interval, next_num = 0;
    // block cursor of a single-component scan, kept incrementally (no divisions per block): (bx, by)
    // in the component's grid, (mx, my) its MCU, (sx, sy) its place in the MCU
    int bx = 0, by = 0, mx = 0, my = 0, sx = 0, sy = 0;
    const int ch0 = sh[0], cv0 = sv[0], bw0 = sbw[0], bo0 = sbo[0];
    const int dsl0 = td[0] & 3, asl0 = 4 + (ta[0] & 3);
    auto gpos = [&]() -> int {
      return ncomp == 1 ? by * bw0 + bx : (my * mcux + mx) * bpm + bo0 + sy * ch0 + sx;
    };
    const bool refine = ss != 0 && ah != 0;
#ifdef SDSJ_PROG_STATS  // (tools/prog_stats.py: shader cycles and bytes per scan kind)
    const uint64_t st_t0 = __builtin_amdgcn_s_memtime();
    const int64_t st_p0 = b.pos;
#endif
    int gn = ns == 1 ? gpos() : 0;
    L.ins_m = -1;
    // refinement: lane k's coefficient k of the current block, and of the next one in flight
    int vcur = refine && nmcu > 0 ? coef[gn * 64 + lane] : 0;
    // DC refinement over all components in frame order without restart intervals: one bit per block
    // in decode order (block g of MCU-order storage), so 32 blocks take one read and a lane each
    bool dc_fast = ss == 0 && ah != 0 && ns == ncomp && ncomp > 1 && restart_interval == 0;
#pragma unroll
    for (int q = 0; q < 4; q++) dc_fast = dc_fast && (q >= ns || comps[q] == q);
    if (dc_fast) {
      const int nblk = nmcu * bpm;
      for (int j0 = 0; j0 < nblk && !b.insufficient; j0 += 32) {
        const int cnt = nblk - j0 < 32 ? nblk - j0 : 32;
        if (b.nbits < cnt) pfill(b);
        const int real = b.nbits - b.pad_bits;  // bits before the inserted zeros
        const uint32_t bits = pgetbits32(b, cnt);
        if (lane < cnt && ((bits >> (cnt - 1 - lane)) & 1)) {
          int16_t* p = coef + (j0 + lane) * 64;
          *p = (int16_t)(*p | (1 << al));
        }
        // the data ran out at block j0 + real: its MCU finished, the next ones are skipped
        if (b.insufficient && L.ins_m < 0) L.ins_m = (j0 + real) / bpm;
      }
    }
    for (int m = 0; m < (dc_fast ? 0 : nmcu); m++) {
      const int g1 = gn;
      if (ns == 1) {
        bx++;
        if (++sx == ch0) {
          sx = 0;
          mx++;
        }
        if (bx == cwb) {
          bx = sx = mx = 0;
          by++;
          if (++sy == cv0) {
            sy = 0;
            my++;
          }
        }
        gn = gpos();
      }
      if (restart_interval) {
        if (restarts_left == 0) {
          if (b.insufficient && L.ins_m < 0) L.ins_m = m - 1;
          if (pprocess_restart(b, &next_num)) return SDSJ_CORRUPT;
          ldc0 = L.ldc[0] = L.ldc[1] = L.ldc[2] = L.ldc[3] = 0;
          eobrun = 0;
          restarts_left = restart_interval;
        }
        restarts_left--;
      }
      // (L.ins_m: the MCU in which this scan ran out of data -- the one before the first MCU skipped
      // or restarted with insufficient data)
      if (refine) {
        const int vnext = m + 1 < nmcu ? coef[gn * 64 + lane] : 0;
        if (!b.insufficient) coef[g1 * 64 + lane] = (int16_t)prefine(b, L, P, asl0, vcur, lane, ss, se, al, &eobrun);
        else if (L.ins_m < 0) L.ins_m = m - 1;
        vcur = vnext;
        continue;
      }
      if (b.insufficient) {  // the MCU's coefficients stay as they are
        if (L.ins_m < 0) L.ins_m = m - 1;
        continue;
      }
      if (ns == 1) {
        if (ss != 0 && eobrun > 0) {
          // AC first scan inside an EOB run: this block and the next eobrun - 1 ones stay empty
          // (decode_mcu_AC_first only counts the run down), up to the scan's or the restart
          // interval's end -- skipped at once, the block cursor recomputed for the block after
          int skip = eobrun;
          if (skip > nmcu - m) skip = nmcu - m;
          if (restart_interval && skip > restarts_left + 1) skip = restarts_left + 1;
          eobrun -= skip;
          if (skip > 1) {
            if (restart_interval) restarts_left -= skip - 1;
            m += skip - 1;
            const int nb = m + 1;
            bx = nb % cwb;
            by = nb / cwb;
            mx = bx / ch0;
            sx = bx - mx * ch0;
            my = by / cv0;
            sy = by - my * cv0;
            gn = gpos();
          }
          continue;
        }
        pblock(b, L, P, dsl0, asl0, 0, coef + g1 * 64, ss, se, ah, al, &ldc0, &eobrun);
        continue;
      }
      for (int q = 0; q < ns; q++) {
        const int ch = L.qh[q], cv = L.qv[q];
        for (int v = 0; v < cv; v++)
          for (int h = 0; h < ch; h++) {
            // block (h, v) of component c in MCU m: ((by / cv) * mcux + bx / ch) * bpm + ... with
            // bx = (m % mcux) * ch + h, by = (m / mcux) * cv + v reduces to m * bpm + ...
            int g;
            if (ncomp == 1) {  // (a single-component frame lists its component more than once)
              const int gx = (m % mcux) * ch + h, gy = (m / mcux) * cv + v;
              g = gy * sbw[q] + gx;
            } else {
              g = m * bpm + L.qbo[q] + v * ch + h;
            }
            pblock(b, L, P, L.qdsl[q], 4, q, coef + g * 64, ss, se, ah, al, &L.ldc[q], &eobrun);
          }
      }
    }
#ifdef SDSJ_PROG_STATS
    {
      const int kind = ss == 0 ? (ah == 0 ? 0 : 2) : (ah == 0 ? 1 : 3);
      const int64_t dt = (int64_t)(__builtin_amdgcn_s_memtime() - st_t0), db = b.pos - st_p0;
      int64_t* tt = kind == 0 ? &d->t_spec : kind == 1 ? &d->t_sync : kind == 2 ? &d->t_scan : &d->t_write;
      int64_t* bb = kind == 0 ? &d->sym_spec : kind == 1 ? &d->sym_sync : kind == 2 ? &d->sym_write : &d->it_write;
      *tt += dt;
      *bb += db;
    }
#endif
    if (b.insufficient && L.ins_m < 0) L.ins_m = nmcu - 1;
    if (L.ins_m >= 0) {  // later iMCU rows keep the previous scan's smoothing parameters
      const int r = ns == 1 ? L.ins_m / cwb : L.ins_m / mcux;
      good = ns == 1 && ncomp > 1 ? r / cv0 : r;
    }
    if (b.eof) return SDSJ_CORRUPT;  // the input ended inside the scan (Pillow: truncated)
    if (!b.hit_marker && pnext_marker(b) < 0) return SDSJ_CORRUPT;
    // jdmarker.c read_markers until the next SOS or EOI
    for (;;) {
      if (b.pos + 1 >= n) return SDSJ_CORRUPT;
      const int m = pbyte(b, b.pos + 1);
      const int body = b.pos + 2;
      if (m == 0xD9) {
        // k_idct reads each component's latched table from slot c
        for (int c = 0; c < d->ncomp; c++) d->comp[c].tq = c;
        // jdcoefct.c smoothing_ok: every component's latched Q00..Q30 nonzero and its DC at least
        // partly known; useful when a coefficient 1..9 of some component is not exact
        bool ok = true, useful = false;
        for (int c = 0; c < d->ncomp; c++) {
          const uint16_t* qc = t->qt[c];
          ok = ok && qc[0] && qc[1] && qc[8] && qc[16] && qc[9] && qc[2] && qc[3] && qc[10] && qc[17] && qc[24] &&
               d->sm_bits[0][c][0] >= 0;
          for (int k = 1; k < 10; k++) {
            useful = useful || d->sm_bits[0][c][k] != 0;
            if (nscans <= 1) d->sm_bits[1][c][k] = -1;
          }
        }
        d->smooth = ok && useful;
        d->sm_good = good;
        return SDSJ_OK;
      }
      if ((m >= 0xD0 && m <= 0xD7) || m == 0x01) {
        b.pos = body;
      } else {
        const bool seg = (m >= 0xE0 && m <= 0xEF) || m == 0xFE || m == 0xDC || m == 0xCC || m == 0xDD ||
                         m == 0xC4 || m == 0xDB || m == 0xDA;
        if (!seg) return SDSJ_CORRUPT;  // a second SOI / SOF, or an unknown marker
        if (m == 0xDC || m == 0xCC) return SDSJ_UNSUPPORTED;
        if (body + 2 > n) return SDSJ_CORRUPT;
        const int l2 = rd16(raw + body);
        if (l2 < 2 || body + l2 > n) return SDSJ_CORRUPT;
        if (m == 0xDA) {
          pos = body;
          break;
        }
        int st = SDSJ_OK;
        if (m == 0xC4) st = pread_dht(P, raw + body + 2, l2 - 2);
        if (m == 0xDB) st = pread_dqt(P, raw + body + 2, l2 - 2);
        if (m == 0xDD) {
          if (l2 != 4) return SDSJ_CORRUPT;
          restart_interval = rd16(raw + body + 2);
        }
        if (st != SDSJ_OK) return st;
        b.pos = body + l2;
      }
      if (pnext_marker(b) < 0) return SDSJ_CORRUPT;
    }
  }
}

}  // namespace

// Zeroes the coefficient arrays of the progressive images (scans accumulate into them).
__global__ void __launch_bounds__(256) k_prog_zero(const ImgDesc* __restrict__ descs, uint8_t* __restrict__ scratch,
                                                   const int32_t* __restrict__ routes, int cap) {
  const int cnt = routes[kRtProg];
  for (int li = blockIdx.x; li < cnt; li += gridDim.x) {
    const ImgDesc* d = &descs[route_list(routes, cap, kRtProg)[li]];
    if (d->status != SDSJ_OK) continue;
    uint4* p = reinterpret_cast<uint4*>(scratch + d->off_coef);
    const int64_t n16 = d->total_blocks * 8;
    for (int64_t i = (int64_t)blockIdx.y * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.y * 256)
      p[i] = make_uint4(0, 0, 0, 0);
  }
}

// The DC plane of the progressive images to be smoothed (int16 per block, decode order) in their
// plane area, which k_idct writes only later: k_prog_smooth reads the neighbours' DC values from it
// while it rewrites blocks in place.  (Blocks stay in zigzag order: k_idct reads that order.)
__global__ void __launch_bounds__(256) k_prog_dcs(const ImgDesc* __restrict__ descs, uint8_t* __restrict__ scratch,
                                                  const int32_t* __restrict__ routes, int cap) {
  const int cnt = routes[kRtProg];
  for (int li = blockIdx.x; li < cnt; li += gridDim.x) {
    const ImgDesc* d = &descs[route_list(routes, cap, kRtProg)[li]];
    if (d->status != SDSJ_OK || !d->smooth) continue;
    const int16_t* coef = reinterpret_cast<const int16_t*>(scratch + d->off_coef);
    int16_t* dcs = reinterpret_cast<int16_t*>(scratch + d->off_planes);
    const int64_t nb = d->total_blocks;
    for (int64_t i = (int64_t)blockIdx.y * 256 + threadIdx.x; i < nb; i += (int64_t)gridDim.y * 256) dcs[i] = coef[i * 64];
  }
}

// pred = num / (Q << 8) rounded half away from zero, clamped below 2^Al when Al > 0
// (jdcoefct.c decompress_smooth_data)
__device__ __forceinline__ int smooth_pred(int64_t num, int64_t q, int al) {
  int pred = (int)(((q << 7) + (num >= 0 ? num : -num)) / (q << 8));
  if (al > 0 && pred >= (1 << al)) pred = (1 << al) - 1;
  return num >= 0 ? pred : -pred;
}

// Block smoothing of the progressive images whose coefficients 1..9 are not all exact after the
// last scan (ImgDesc::smooth, k_prog): jdcoefct.c decompress_smooth_data, one thread per block of the
// image in decode order.  Zero coefficients AC01 AC10 AC20 AC11 AC02 (and AC03 AC12 AC21 AC30 and
// the DC itself when the component has no AC data at all) get estimates from the DC values of the
// block's 5x5 neighbourhood, read from the DC plane k_prog_dcs copied into the (not yet written)
// plane area -- libjpeg likewise reads the neighbours unmodified while it smooths a copy of the block.
// Rows: jdcoefct.c's per-iMCU-row choice (the last iMCU row's real rows only); columns clamped to the
// component's width in blocks (tests/test_gpu_parity.py: bit-exact against the Pillow-pinned CPU restatement).
__device__ void prog_smooth_image(int img, const ImgDesc* __restrict__ descs, const ImgTables* __restrict__ tables,
                                  uint8_t* __restrict__ scratch);
__global__ void __launch_bounds__(256) k_prog_smooth(const ImgDesc* __restrict__ descs,
                                                     const ImgTables* __restrict__ tables,
                                                     uint8_t* __restrict__ scratch, const int32_t* __restrict__ routes,
                                                     int cap) {
  const int cnt = routes[kRtProg];
  for (int li = blockIdx.x; li < cnt; li += gridDim.x)
    prog_smooth_image(route_list(routes, cap, kRtProg)[li], descs, tables, scratch);
}

__device__ void prog_smooth_image(int img, const ImgDesc* __restrict__ descs, const ImgTables* __restrict__ tables,
                                  uint8_t* __restrict__ scratch) {
  const ImgDesc* d = &descs[img];
  if (d->status != SDSJ_OK || !d->smooth) return;
  int16_t* coef = reinterpret_cast<int16_t*>(scratch + d->off_coef);
  const int16_t* dcs = reinterpret_cast<const int16_t*>(scratch + d->off_planes);
  const int ncomp = d->ncomp, bpm = d->bpm, mcux = d->mcux;
  const int64_t nb = d->total_blocks;
  for (int64_t g = (int64_t)blockIdx.y * 256 + threadIdx.x; g < nb; g += (int64_t)gridDim.y * 256) {
    // block g -> component, block row / column (jdcoefct.c MCU order: components in turn, h x v each)
    int c = 0, by, bx;
    if (ncomp == 1) {
      by = (int)(g / mcux);
      bx = (int)(g - (int64_t)by * mcux);
    } else {
      const int m = (int)(g / bpm), b = (int)(g - (int64_t)m * bpm);
      c = d->blk_comp[b];
      const int my = m / mcux, mx = m - my * mcux;
      bx = mx * d->comp[c].h + d->blk_dx[b];
      by = my * d->comp[c].v + d->blk_dy[b];
    }
    const CompDesc& cd = d->comp[c];
    const int h = ncomp == 1 ? 1 : cd.h, v = ncomp == 1 ? 1 : cd.v;
    const int wib = (cd.dw + 7) >> 3, hib = (cd.dh + 7) >> 3;
    if (bx >= wib || by >= hib) continue;  // (padding blocks: never output)
    const int total = ncomp == 1 ? hib : d->mcuy, imcu = by / v, brow = by - imcu * v;
    int block_rows = v;
    if (imcu == total - 1) {
      block_rows = hib % v;
      if (block_rows == 0) block_rows = v;
    }
    const int ibr = imcu * block_rows + brow, ibrs = block_rows * total;
    int rows[5];
    rows[2] = by;
    rows[1] = ibr > 0 ? by - 1 : by;
    rows[0] = ibr > 1 ? by - 2 : rows[1];
    rows[3] = ibr < ibrs - 1 ? by + 1 : by;
    rows[4] = ibr < ibrs - 2 ? by + 2 : rows[3];
    int boff = 0;  // first MCU block of component c
    for (int q = 0; q < c; q++) boff += d->comp[q].h * d->comp[q].v;
    int DC[5][5];
    for (int i = 0; i < 5; i++)
      for (int jx = 0; jx < 5; jx++) {
        int x = bx + jx - 2;
        x = x < 0 ? 0 : (x > wib - 1 ? wib - 1 : x);
        const int y = rows[i];
        const int64_t gg = ncomp == 1 ? (int64_t)y * mcux + x
                                      : ((int64_t)(y / v) * mcux + x / h) * bpm + boff + (y % v) * h + (x % h);
        DC[i][jx] = dcs[gg];
      }
    const int8_t* cb = d->sm_bits[imcu > d->sm_good ? 1 : 0][c];
    bool change_dc = true;
    for (int k = 1; k < 10; k++) change_dc = change_dc && cb[k] == -1;
    const uint16_t* qt = tables[img].qt[c];  // (k_prog: the component's latched table sits in slot c)
    const int64_t Q00 = qt[0];
    int16_t* blk = coef + g * 64;
    // DCnn of jdcoefct.c: DC01 .. DC25 row by row (DC13 = this block)
#define SD(n) DC[((n) - 1) / 5][((n) - 1) % 5]
    // coefficient zz (zigzag = coef_bits index; the blocks are in zigzag order), quantiser at natural index nat
    auto est = [&](int nat, int zz, int64_t num) {
      const int al = cb[zz];
      if (al != 0 && blk[zz] == 0) blk[zz] = (int16_t)smooth_pred(Q00 * num, qt[nat], al);
    };
    est(1, 1,
        change_dc ? (-SD(1) - SD(2) + SD(4) + SD(5) - 3 * SD(6) + 13 * SD(7) - 13 * SD(9) + 3 * SD(10) - 3 * SD(11) +
                     38 * SD(12) - 38 * SD(14) + 3 * SD(15) - 3 * SD(16) + 13 * SD(17) - 13 * SD(19) + 3 * SD(20) -
                     SD(21) - SD(22) + SD(24) + SD(25))
                  : (-7 * SD(11) + 50 * SD(12) - 50 * SD(14) + 7 * SD(15)));
    est(8, 2,
        change_dc ? (-SD(1) - 3 * SD(2) - 3 * SD(3) - 3 * SD(4) - SD(5) - SD(6) + 13 * SD(7) + 38 * SD(8) +
                     13 * SD(9) - SD(10) + SD(16) - 13 * SD(17) - 38 * SD(18) - 13 * SD(19) + SD(20) + SD(21) +
                     3 * SD(22) + 3 * SD(23) + 3 * SD(24) + SD(25))
                  : (-7 * SD(3) + 50 * SD(8) - 50 * SD(18) + 7 * SD(23)));
    est(16, 3,
        change_dc ? (SD(3) + 2 * SD(7) + 7 * SD(8) + 2 * SD(9) - 5 * SD(12) - 14 * SD(13) - 5 * SD(14) + 2 * SD(17) +
                     7 * SD(18) + 2 * SD(19) + SD(23))
                  : (-SD(3) + 13 * SD(8) - 24 * SD(13) + 13 * SD(18) - SD(23)));
    est(9, 4,
        change_dc ? (-SD(1) + SD(5) + 9 * SD(7) - 9 * SD(9) - 9 * SD(17) + 9 * SD(19) + SD(21) - SD(25))
                  : (-SD(2) + SD(4) - SD(6) + 10 * SD(7) - 10 * SD(9) + SD(10) + SD(16) - 10 * SD(17) + 10 * SD(19) -
                     SD(20) + SD(22) - SD(24)));
    est(2, 5,
        change_dc ? (2 * SD(7) - 5 * SD(8) + 2 * SD(9) + SD(11) + 7 * SD(12) - 14 * SD(13) + 7 * SD(14) + SD(15) +
                     2 * SD(17) - 5 * SD(18) + 2 * SD(19))
                  : (-SD(11) + 13 * SD(12) - 24 * SD(13) + 13 * SD(14) - SD(15)));
    if (change_dc) {
      est(3, 6, SD(7) - SD(9) + 2 * SD(12) - 2 * SD(14) + SD(17) - SD(19));
      est(10, 7, SD(7) - 3 * SD(8) + SD(9) - SD(17) + 3 * SD(18) - SD(19));
      est(17, 8, SD(7) - SD(9) - 3 * SD(12) + 3 * SD(14) + SD(17) - SD(19));
      est(24, 9, SD(7) + 2 * SD(8) + SD(9) - SD(17) - 2 * SD(18) - SD(19));
      const int64_t num =
          Q00 * (-2 * SD(1) - 6 * SD(2) - 8 * SD(3) - 6 * SD(4) - 2 * SD(5) - 6 * SD(6) + 6 * SD(7) + 42 * SD(8) +
                 6 * SD(9) - 6 * SD(10) - 8 * SD(11) + 42 * SD(12) + 152 * SD(13) + 42 * SD(14) - 8 * SD(15) -
                 6 * SD(16) + 6 * SD(17) + 42 * SD(18) + 6 * SD(19) - 6 * SD(20) - 2 * SD(21) - 6 * SD(22) -
                 8 * SD(23) - 6 * SD(24) - 2 * SD(25));
      blk[0] = (int16_t)smooth_pred(num, Q00, 0);
    }
#undef SD
  }
}

// One wave per progressive image: the wave walks all the scans together (the header); the lanes split
// the AC refinement scans' blocks coefficient by coefficient (prefine).  The derived tables in LDS.
#ifndef SDSJ_PROG_WAVES
#define SDSJ_PROG_WAVES 5
#endif
constexpr int kProgThreads = 64;
constexpr int kProgHelperGrid = 1024;  // workgroup columns of k_prog_zero / k_prog_dcs / k_prog_smooth
__global__ void __launch_bounds__(kProgThreads) __attribute__((amdgpu_waves_per_eu(SDSJ_PROG_WAVES)))
k_prog(ImgDesc* __restrict__ descs, ImgTables* __restrict__ tables, const uint8_t* __restrict__ blob,
       const int64_t* __restrict__ offsets, const int32_t* __restrict__ lengths, uint8_t* __restrict__ scratch,
       const int32_t* __restrict__ routes, int cap) {
  __shared__ PLds lds;
  const int cnt = routes[kRtProg];
  const int32_t* lst = route_list(routes, cap, kRtProg);
  for (int li = blockIdx.x; li < cnt; li += gridDim.x) {  // (one entry per workgroup at the full grid)
    const int img = lst[li];
    ImgDesc* d = &descs[img];
    if (d->status == SDSJ_OK) {
      const int st = decode_progressive(d, &tables[img], blob + offsets[img], lengths[img],
                                        reinterpret_cast<int16_t*>(scratch + d->off_coef),
                                        reinterpret_cast<ProgTables*>(scratch + d->off_ptab), lds, threadIdx.x);
      if (st != SDSJ_OK && threadIdx.x == 0) d->status = st;
    }
    __syncthreads();  // LDS reuse by the next entry
  }
}

hipError_t launch_prog(int n, ImgDesc* descs, ImgTables* tables, const uint8_t* blob, const int64_t* offsets,
                       const int32_t* lengths, uint8_t* scratch, const int32_t* routes, int cap, hipStream_t s,
                       uint64_t rm, uint64_t hint) {
  if (!route_on(rm, kRtProg)) return hipSuccess;
  // (the helpers stride over the route list: a batch without progressive images launches few empty
  // workgroups -- at one per image their grids cost 115 us per 16,384 baseline images)
  const int gx = (int)route_grid(hint, kRtProg, n < kProgHelperGrid ? n : kProgHelperGrid);
  hipLaunchKernelGGL(k_prog_zero, dim3(gx, 16), dim3(256), 0, s, descs, scratch, routes, cap);
  hipLaunchKernelGGL(k_prog, dim3(route_grid(hint, kRtProg, n)), dim3(kProgThreads), 0, s, descs, tables, blob,
                     offsets, lengths, scratch, routes, cap);
  hipLaunchKernelGGL(k_prog_dcs, dim3(gx, 8), dim3(256), 0, s, descs, scratch, routes, cap);
  hipLaunchKernelGGL(k_prog_smooth, dim3(gx, 8), dim3(256), 0, s, descs, tables, scratch, routes, cap);
  return hipGetLastError();
}

}  // namespace sdsj
