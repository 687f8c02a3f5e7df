// sdsj_kernels.h -- launchers of the gfx950 kernels in sdsj_kernels.hip (engine-internal).
#pragma once
#include <hip/hip_runtime.h>

#include "sdsj_common.h"

namespace sdsj {
// Route masks (bit r = route r may hold images): launchers skip the variant kernels of routes whose
// bit is clear.  The host paths know every image's routes from host planning (host_plan_need); the
// device-resident path passes kAllRoutes (its route lists exist only on the device).
constexpr uint64_t kAllRoutes = ~0ull;
SDSJ_HD inline bool route_on(uint64_t rm, int r) { return (rm >> r) & 1ull; }
// Route hints (hint: bit r = route r held images in a recent batch of this engine): a launched route
// outside the hint gets a small grid whose workgroups stride over its list -- exact for any count,
// only slower -- instead of one workgroup per possible entry.  The device path launches every route
// (its lists exist only on the device), and most of them are empty for a given dataset: thousands
// of empty workgroups per launch otherwise (sdsj_engine.hip run_chunk keeps the hint).
constexpr int kColdGrid = 64;
inline unsigned route_grid(uint64_t hint, int r, int64_t full) {
  return (unsigned)(route_on(hint, r) || full < kColdGrid ? full : kColdGrid);
}
// blob_bytes: the blob's size -- a sample whose [offset, offset + length) leaves it is reported EINVAL
hipError_t launch_parse(int n, const uint8_t* blob, int64_t blob_bytes, const int64_t* offsets, const int32_t* lengths,
                        const sdsj_op& op, int warm_bits, bool small, ImgDesc* descs, ImgTables* tables, hipStream_t s);
// base: scratch bytes a previous lane of the batch already took (device), or null
hipError_t launch_plan(int n, ImgDesc* descs, int64_t capacity, const int64_t* base, int64_t* total, int32_t* routes,
                       int cap, hipStream_t s);
hipError_t launch_unstuff(int n, const uint8_t* blob, const int64_t* offsets, ImgDesc* descs, uint8_t* scratch,
                          const int32_t* routes, int cap,
                          hipStream_t s, uint64_t rm = kAllRoutes, uint64_t hint = kAllRoutes);
hipError_t launch_scanmap(int n, const uint8_t* blob, const int64_t* offsets, ImgDesc* descs, uint8_t* scratch,
                          hipStream_t s);
// progressive images (route kRtProg): zero their coefficients, then one lane per image decodes all scans
hipError_t launch_prog(int n, ImgDesc* descs, ImgTables* tables, const uint8_t* blob, const int64_t* offsets,
                       const int32_t* lengths, uint8_t* scratch, const int32_t* routes, int cap, hipStream_t s,
                       uint64_t rm = kAllRoutes, uint64_t hint = kAllRoutes);
size_t enttab_bytes();  // per-image decode tables (k_enttab) held in HBM between the entropy kernels
// k_enttab (decode tables) + k_entspec (subsequence layout, warm-up, speculative decode)
// (small: a host-path latency-mode chunk, where ImgDesc::mh images take the multi-hypothesis pass)
hipError_t launch_entspec(int n, ImgDesc* descs, const ImgTables* specs, void* etab, uint8_t* scratch, int32_t* routes,
                          int cap, hipStream_t s, uint64_t rm = kAllRoutes, bool small = false,
                          uint64_t hint = kAllRoutes);
// k_entsync (sync rounds + segmented scan)
hipError_t launch_entsync(int n, ImgDesc* descs, void* etab, uint8_t* scratch, int32_t* routes, int cap, hipStream_t s,
                          uint64_t rm = kAllRoutes, uint64_t hint = kAllRoutes);
hipError_t launch_entwrite(int n, ImgDesc* descs, const void* etab, uint8_t* scratch, int32_t* routes, int cap,
                           hipStream_t s, uint64_t rm = kAllRoutes, uint64_t hint = kAllRoutes);
hipError_t launch_idct(int n, const ImgDesc* descs, const ImgTables* tables, uint8_t* scratch, hipStream_t s);
hipError_t launch_color(int n, const ImgDesc* descs, uint8_t* scratch, const int32_t* routes, int cap, hipStream_t s,
                        uint64_t rm = kAllRoutes);
hipError_t launch_coeffs(int n, ImgDesc* descs, const sdsj_op& op, uint8_t* scratch, hipStream_t s);
hipError_t launch_hpass(int n, const ImgDesc* descs, const sdsj_op& op, uint8_t* scratch, const int32_t* routes, int cap,
                        hipStream_t s, uint64_t rm = kAllRoutes);
hipError_t launch_vpass(int n, const ImgDesc* descs, const sdsj_op& op, const uint8_t* scratch, const uint8_t* flip,
                        void* out, const int32_t* routes, int cap, const float* lut, hipStream_t s,
                        uint64_t rm = kAllRoutes);
hipError_t launch_resample(int n, const ImgDesc* descs, const sdsj_op& op, const uint8_t* scratch, const uint8_t* flip,
                           void* out, int32_t* status, const int32_t* routes, int cap, const float* lut, hipStream_t s,
                           uint64_t rm = kAllRoutes, uint64_t hint = kAllRoutes);
hipError_t launch_resample420(int n, const ImgDesc* descs, const sdsj_op& op, int strip_h, const uint8_t* scratch,
                              const uint8_t* flip, void* out, const int32_t* routes, int cap, const float* lut,
                              hipStream_t s, uint64_t rm = kAllRoutes, uint64_t hint = kAllRoutes);
// lengths: the samples' encoded sizes (null: raw frames); counters: SDSJ_CTR_* accumulators (or null)
// (a negative length: the sample is reported as EINVAL -- an unreadable file of the host path)
hipError_t launch_finish(int n, ImgDesc* descs, const sdsj_op& op, void* out, int32_t* status, const float* lut,
                         const int32_t* lengths, unsigned long long* counters, hipStream_t s);
// host-side planning (same code as k_parse): returns the scratch bytes image `jpg` needs, or < 0
// *routes (optional): the routes the image takes (bits as in route masks; all of them when the host
// parse fails, so the device's own verdict is never starved of a kernel)
// small: the latency-mode plan of a chunk of at most kSmallBatch images (k_parse's `small`)
int64_t host_plan_need(const uint8_t* jpg, int64_t n, const sdsj_op& op, int* status, uint64_t* routes = nullptr,
                       bool small = false);
// host-side planning of one raw RGB frame (width x height) for the unfused passes; returns scratch bytes
int64_t host_plan_frame(ImgDesc* d, int width, int height, const sdsj_op& op);
}  // namespace sdsj
