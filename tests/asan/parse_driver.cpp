// Host AddressSanitizer / UBSan driver of the shared JPEG header parser (sds_amd/csrc/sdsj_common.h,
// the code sdsj_probe and the device k_parse run).  Reads records [u32 length][bytes] from the file
// in argv[1] and prints one line per record: status width height ncomp bpm total_blocks.
// Each input is copied into an exactly sized heap buffer, so any read past its end is reported.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../sds_amd/csrc/sdsj_common.h"

using namespace sdsj;

struct Rd {
  const uint8_t* p;
  int operator()(int64_t i) const { return p[i]; }
};

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<uint8_t> all;
  uint8_t tmp[1 << 16];
  size_t r;
  while ((r = fread(tmp, 1, sizeof(tmp), f)) > 0) all.insert(all.end(), tmp, tmp + r);
  fclose(f);
  size_t pos = 0;
  while (pos + 4 <= all.size()) {
    uint32_t n;
    memcpy(&n, &all[pos], 4);
    pos += 4;
    if (pos + n > all.size()) return 3;
    uint8_t* buf = static_cast<uint8_t*>(malloc(n ? n : 1));
    memcpy(buf, &all[pos], n);
    pos += n;
    ImgDesc* d = new ImgDesc();
    ImgTables* t = new ImgTables();
    Rd rd{buf};
    int st = parse_headers(rd, (int64_t)n, d, t, CopySink<Rd>{rd});
    if (st == SDSJ_OK) st = setup_geometry(d, t);
    for (int c = 0; st == SDSJ_OK && !d->progressive && c < d->ncomp; c++)
      if (!huff_table_ok(t->dc_spec[d->comp[c].td], true) || !huff_table_ok(t->ac_spec[d->comp[c].ta], false))
        st = SDSJ_CORRUPT;
    if (st == SDSJ_OK) {
      int x0, y0, cw, ch;
      crop_box(d->width, d->height, 256, 256, &x0, &y0, &cw, &ch);
      if (cw <= 0 || ch <= 0 || x0 < 0 || y0 < 0) st = 99;
      (void)resample_ksize(cw, 256, filter_support(SDSJ_FILTER_BILINEAR));
    }
    printf("%d %d %d %d %d %lld\n", st, d->width, d->height, d->ncomp, st == SDSJ_OK ? d->bpm : 0,
           st == SDSJ_OK ? (long long)d->total_blocks : 0LL);
    delete d;
    delete t;
    free(buf);
  }
  return 0;
}
