/* sdsj_oracle.h -- TEST INFRASTRUCTURE ONLY: CPU restatement used as the parity checker.
 * Status codes deliberately share values with include/sdsj.h so tests can compare them. */
#ifndef SDSJ_ORACLE_H
#define SDSJ_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifndef SDSJ_OK
#define SDSJ_OK 0
#define SDSJ_EINVAL (-1)
#define SDSJ_UNSUPPORTED (-2)
#define SDSJ_CORRUPT (-3)
#define SDSJ_ENOMEM (-4)
#endif

typedef struct {
    int32_t width, height, ncomp;
    int32_t h[3], v[3];
    int32_t restart_interval;
    int64_t entropy_offset;
} sdsj_oracle_info;

int sdsj_oracle_probe(const uint8_t *jpg, size_t n, sdsj_oracle_info *info);
int sdsj_oracle_decode(const uint8_t *jpg, size_t n, uint8_t *rgb, int cap_w, int cap_h);
int sdsj_oracle_coefficients(const uint8_t *jpg, size_t n, int c, int16_t *out, int64_t cap, int *bw, int *bh);
void sdsj_oracle_crop_box(int w, int h, int out_h, int out_w, int box[4]);
int sdsj_oracle_resize(const uint8_t *in, int w, int h, int out_w, int out_h, int filter, uint8_t *out);
int sdsj_oracle_pipeline(const uint8_t *jpg, size_t n, int out_h, int out_w, int crop_before_resize,
                         int filter, uint8_t *out);
#endif
