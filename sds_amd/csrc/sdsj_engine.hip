// sdsj_engine.hip -- the C-ABI (include/sdsj.h): engine state, scratch management, batch driver.
//
// One engine per process and device (sds transforms are created lazily per DataLoader worker,
// presets.py:1-5).  The engine owns device scratch, per-image descriptor/table arrays, pinned
// staging for the host-bytes entry point and the 256-entry normalisation LUT.  Every batch is a
// fixed sequence of kernel launches on the caller's stream: no host synchronisation inside the
// device-resident entry point.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "sdsj_common.h"
#include "sdsj_kernels.h"

using namespace sdsj;

namespace {
constexpr int kStages = 13;
#ifndef SDSJ_MAX_LANES
#define SDSJ_MAX_LANES 4
#endif
constexpr int kMaxLanes = SDSJ_MAX_LANES;
const char* kStageNames[kStages] = {"parse", "plan",  "unstuff", "prog",  "entspec", "entsync", "entwrite",
                                    "idct",  "color", "coeffs",  "hpass", "vpass",   "resample"};
constexpr int kMarkAfterSpec = 5;  // mark index at the end of the entspec stage
}  // namespace

struct sdsj_engine {
  int device = 0;
  int max_batch = 4096;
  int64_t capacity = 0;
  bool grow = true;
  int warm_bits = -1;  // entropy warm-up override (SDSJ_WARM_BITS, experiments); < 0 = plan default
  uint8_t* scratch = nullptr;
  ImgDesc* descs = nullptr;
  ImgTables* tables = nullptr;
  int64_t* d_total = nullptr;
  void* d_etab = nullptr;       // per-image decode tables built by k_enttab
  int32_t* d_routes = nullptr;  // per-variant image lists built by k_plan (sdsj_common.h Route)
  // lanes 2.. of a chunk (run_chunk): route lists and scratch totals, streams and events
  int lanes = 4;     // SDSJ_LANES (experiments)
  int lane_mid = 2;  // lane k + 1 starts at lane k's mark lane_mid (>= 2: k_plan done; -1: its spec pass)
  int64_t* d_totals_x = nullptr;
  int32_t* d_routes_x = nullptr;
  hipStream_t aux[kMaxLanes - 1] = {};
  hipEvent_t ev_mid[kMaxLanes - 1] = {}, ev_join[kMaxLanes - 1] = {};
  // route hints of the device path (sdsj_kernels.h route_grid), one per op (the resample route -- taps,
  // layout -- follows the output size, filter, dtype and layout): each call copies its lanes' route counts
  // to pinned memory after k_plan; a later call folds a finished copy into the hint of the op it ran
  static constexpr int kHintSlots = 4;
  uint64_t hint_key[kHintSlots] = {};
  uint64_t hint[kHintSlots] = {};
  int hint_n = 0, hint_next = 0;
  int32_t* h_rcounts = nullptr;  // [kMaxLanes][kNumRoutes]
  hipEvent_t ev_rc[kMaxLanes] = {};
  bool rc_pending = false;
  int rc_lanes = 0;
  uint64_t rc_key = 0;  // the op of the outstanding readback
  // frames path: host-planned descriptors and route list, staged through pinned memory
  ImgDesc* h_fdescs = nullptr;
  int32_t* h_froutes = nullptr;
  float* d_lut = nullptr;
  unsigned long long* d_counters = nullptr;  // SDSJ_CTR_* (k_finish)
  // host-bytes path
  uint8_t* h_stage = nullptr;
  size_t h_stage_cap = 0;
  uint8_t* d_blob = nullptr;
  size_t d_blob_cap = 0;
  int64_t* h_offsets = nullptr;
  int32_t* h_lengths = nullptr;
  uint8_t* h_flip = nullptr;
  int64_t* d_offsets = nullptr;
  int32_t* d_lengths = nullptr;
  uint8_t* d_flip = nullptr;
  int32_t* d_status = nullptr;
  int32_t* h_status = nullptr;
  int io_cap = 0;
  // persistent staging threads of the host paths (parallel_for), created on first use
  std::unique_ptr<struct StagePool> pool;
  // asynchronous host path (sdsj_submit_*): per-slot pinned staging, device inputs and events
  struct Slot {
    uint8_t* h_stage = nullptr;
    uint8_t* d_blob = nullptr;
    size_t bytes_cap = 0;
    int64_t *h_offsets = nullptr, *d_offsets = nullptr;
    int32_t *h_lengths = nullptr, *d_lengths = nullptr;
    uint8_t *h_flip = nullptr, *d_flip = nullptr;
    int32_t *h_status = nullptr, *d_status = nullptr;
    int32_t* h_pre = nullptr;  // host-side per-sample status (unreadable files)
    int cap = 0, n = 0;
    bool pending = false;
    hipEvent_t ev_h2d = nullptr, ev_done = nullptr;
  } slots[SDSJ_SLOTS];
  hipStream_t copy_stream = nullptr;
  // timing: one event set per chunk launched since the last sdsj_engine_set_timing(e, 1)
  bool timing = false;
  std::vector<std::vector<hipEvent_t>> ev_sets;
  size_t ev_used = 0;
  std::string err;
};

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int fail(sdsj_engine* e, int code, const std::string& msg) {
  if (e) e->err = msg;
  return code;
}

int hip_fail(sdsj_engine* e, hipError_t st, const char* what) {
  return fail(e, SDSJ_EHIP, std::string(what) + ": " + hipGetErrorString(st));
}

#define SDSJ_HIP(e, call)                                  \
  do {                                                     \
    hipError_t _st = (call);                               \
    if (_st != hipSuccess) return hip_fail((e), _st, #call); \
  } while (0)

int ensure_io(sdsj_engine* e, int n) {
  if (n <= e->io_cap) return SDSJ_OK;
  int cap = std::max(n, 64);
  (void)hipFree(e->d_offsets);
  (void)hipFree(e->d_lengths);
  (void)hipFree(e->d_flip);
  (void)hipFree(e->d_status);
  (void)hipHostFree(e->h_offsets);
  (void)hipHostFree(e->h_lengths);
  (void)hipHostFree(e->h_flip);
  (void)hipHostFree(e->h_status);
  e->io_cap = 0;
  SDSJ_HIP(e, hipMalloc(&e->d_offsets, sizeof(int64_t) * cap));
  SDSJ_HIP(e, hipMalloc(&e->d_lengths, sizeof(int32_t) * cap));
  SDSJ_HIP(e, hipMalloc(&e->d_flip, cap));
  SDSJ_HIP(e, hipMalloc(&e->d_status, sizeof(int32_t) * cap));
  SDSJ_HIP(e, hipHostMalloc(&e->h_offsets, sizeof(int64_t) * cap));
  SDSJ_HIP(e, hipHostMalloc(&e->h_lengths, sizeof(int32_t) * cap));
  SDSJ_HIP(e, hipHostMalloc(&e->h_flip, cap));
  SDSJ_HIP(e, hipHostMalloc(&e->h_status, sizeof(int32_t) * cap));
  e->io_cap = cap;
  return SDSJ_OK;
}

int ensure_scratch(sdsj_engine* e, int64_t need) {
  if (need <= e->capacity && e->scratch) return SDSJ_OK;
  int64_t cap = std::max<int64_t>(need, e->capacity * 3 / 2);
  cap = std::max<int64_t>(cap, 64 << 20);
  (void)hipFree(e->scratch);
  e->scratch = nullptr;
  e->capacity = 0;
  SDSJ_HIP(e, hipMalloc(&e->scratch, cap));
  e->capacity = cap;
  return SDSJ_OK;
}

bool valid_op(const sdsj_op* op) {
  return op && op->out_h > 0 && op->out_w > 0 && op->out_h <= 65535 && op->out_w <= 65535 && op->filter >= 0 &&
         op->filter <= SDSJ_FILTER_NEAREST && (op->out_dtype == SDSJ_DTYPE_U8 || op->out_dtype == SDSJ_DTYPE_F32) &&
         (op->layout == SDSJ_LAYOUT_CHW || op->layout == SDSJ_LAYOUT_HWC);
}

int64_t out_bytes_per_image(const sdsj_op& op) {
  return (int64_t)op.out_h * op.out_w * 3 * (op.out_dtype == SDSJ_DTYPE_F32 ? 4 : 1);
}

// One lane of a chunk: a contiguous range of its images with their own route lists and scratch
// total.  `base`: the scratch bytes the previous lane took (device), or null for the first lane.
struct Lane {
  ImgDesc* descs;
  ImgTables* tables;
  void* etab;
  int32_t* routes;
  int64_t* total;
  const int64_t* base;
};

// Runs the kernel sequence for one lane (n <= max_batch images) of device-resident inputs.
// after_spec (optional) is recorded once the lane's speculative entropy pass is queued.
// hint: routes expected to hold images (full grids); rc_lane >= 0: copy this lane's route counts to the
// engine's pinned readback slot rc_lane after k_plan
int run_lane(sdsj_engine* e, const Lane& ln, int n, bool small, const uint8_t* d_blob, int64_t blob_bytes, const int64_t* d_offsets,
             const int32_t* d_lengths, const sdsj_op& op, const uint8_t* d_flip, void* d_out, int32_t* d_status,
             hipStream_t s, hipEvent_t after_spec, uint64_t rm, uint64_t hint = kAllRoutes, int rc_lane = -1) {
  std::vector<hipEvent_t>* evs = nullptr;
  if (e->timing) {
    if (e->ev_used == e->ev_sets.size()) {
      std::vector<hipEvent_t> set(kStages + 1);
      for (auto& ev : set) SDSJ_HIP(e, hipEventCreate(&ev));
      e->ev_sets.push_back(set);
    }
    evs = &e->ev_sets[e->ev_used++];
  }
  auto mark = [&](int k) {
    if (evs) (void)hipEventRecord((*evs)[k], s);
    if (after_spec && (e->lane_mid == k || (e->lane_mid < 0 && k == kMarkAfterSpec))) (void)hipEventRecord(after_spec, s);
  };
  mark(0);
  SDSJ_HIP(e, launch_parse(n, d_blob, blob_bytes, d_offsets, d_lengths, op, e->warm_bits, small, ln.descs, ln.tables, s));
  mark(1);
  const int cap = e->max_batch;
  SDSJ_HIP(e, launch_plan(n, ln.descs, e->capacity, ln.base, ln.total, ln.routes, cap, s));
  if (rc_lane >= 0) {
    SDSJ_HIP(e, hipMemcpyAsync(e->h_rcounts + rc_lane * kNumRoutes, ln.routes, sizeof(int32_t) * kNumRoutes,
                               hipMemcpyDeviceToHost, s));
    SDSJ_HIP(e, hipEventRecord(e->ev_rc[rc_lane], s));
  }
  mark(2);
  SDSJ_HIP(e, launch_unstuff(n, d_blob, d_offsets, ln.descs, e->scratch, ln.routes, cap, s, rm, hint));
  SDSJ_HIP(e, launch_scanmap(n, d_blob, d_offsets, ln.descs, e->scratch, s));
  mark(3);
  // (after mark 3: the next lane may start while this lane's progressive images decode)
  SDSJ_HIP(e, launch_prog(n, ln.descs, ln.tables, d_blob, d_offsets, d_lengths, e->scratch, ln.routes, cap, s, rm, hint));
  mark(4);
  SDSJ_HIP(e, launch_entspec(n, ln.descs, ln.tables, ln.etab, e->scratch, ln.routes, cap, s, rm, small, hint));
  mark(5);
  SDSJ_HIP(e, launch_entsync(n, ln.descs, ln.etab, e->scratch, ln.routes, cap, s, rm, hint));
  mark(6);
  SDSJ_HIP(e, launch_entwrite(n, ln.descs, ln.etab, e->scratch, ln.routes, cap, s, rm, hint));
  mark(7);
  SDSJ_HIP(e, launch_idct(n, ln.descs, ln.tables, e->scratch, s));
  mark(8);
  SDSJ_HIP(e, launch_color(n, ln.descs, e->scratch, ln.routes, cap, s, rm));
  mark(9);
  SDSJ_HIP(e, launch_coeffs(n, ln.descs, op, e->scratch, s));
  mark(10);
  SDSJ_HIP(e, launch_hpass(n, ln.descs, op, e->scratch, ln.routes, cap, s, rm));
  mark(11);
  SDSJ_HIP(e, launch_vpass(n, ln.descs, op, e->scratch, d_flip, d_out, ln.routes, cap, e->d_lut, s, rm));
  mark(12);
  SDSJ_HIP(e, launch_resample(n, ln.descs, op, e->scratch, d_flip, d_out, d_status, ln.routes, cap, e->d_lut, s, rm, hint));
  SDSJ_HIP(e, launch_finish(n, ln.descs, op, d_out, d_status, e->d_lut, d_lengths, e->d_counters, s));
  mark(13);
  return SDSJ_OK;
}

// Runs one chunk (n <= max_batch).  A chunk of at least L x kLaneMin images runs as L lanes
// (contiguous image ranges) on L streams, lane k + 1 starting once lane k has planned its scratch:
// the lanes' kernel sequences overlap, so the latency-bound kernels of one lane (the entropy sync
// pass, every kernel's tail) run beside the throughput-bound kernels of another.  The caller's
// stream waits for every lane at the end.  Scratch is taken by the lanes in image order (lane k + 1's
// k_plan starts from lane k's total), so per-image results and capacity failures are those of a
// single lane.
constexpr int kLaneMin = 128;

uint64_t op_key(const sdsj_op& op) {
  return (uint64_t)(uint32_t)op.out_h | (uint64_t)(uint32_t)op.out_w << 16 | (uint64_t)(op.crop_before_resize != 0) << 32 |
         (uint64_t)(op.filter & 0xff) << 33 | (uint64_t)(op.out_dtype & 0xf) << 41 | (uint64_t)(op.layout & 0xf) << 45 |
         1ull << 63;  // (never 0: an empty slot's key)
}

uint64_t hint_lookup(const sdsj_engine* e, uint64_t key) {
  for (int k = 0; k < e->hint_n; k++)
    if (e->hint_key[k] == key) return e->hint[k];
  return kAllRoutes;
}

void hint_store(sdsj_engine* e, uint64_t key, uint64_t h) {
  for (int k = 0; k < e->hint_n; k++)
    if (e->hint_key[k] == key) {
      e->hint[k] = h;
      return;
    }
  int k = e->hint_n < sdsj_engine::kHintSlots ? e->hint_n++ : (e->hint_next++ % sdsj_engine::kHintSlots);
  e->hint_key[k] = key;
  e->hint[k] = h;
}

// rm: the routes the chunk's images may take (host planning), or kAllRoutes; small: the chunk was
// host-planned in latency mode (host paths, n <= kSmallBatch)
int run_chunk(sdsj_engine* e, int n, const uint8_t* d_blob, int64_t blob_bytes, const int64_t* d_offsets, const int32_t* d_lengths,
              const sdsj_op& op, const uint8_t* d_flip, void* d_out, int32_t* d_status, hipStream_t s,
              uint64_t rm = kAllRoutes, bool small = false) {
  int nl = std::min(std::max(e->lanes, 1), kMaxLanes);
  while (nl > 1 && n < nl * kLaneMin) nl--;
  // route hint: the host paths know their routes exactly (rm); the device path uses the routes that held
  // images in the last batch of the same op whose counts have come back (all routes until one has, or
  // when the op changed: another output size selects other resample routes), and requests a new
  // readback when none is outstanding
  uint64_t hint = rm;
  bool readback = false;
  const uint64_t key = op_key(op);
  if (rm == kAllRoutes) {
    if (e->rc_pending) {
      bool done = true, lost = false;
      for (int k = 0; k < e->rc_lanes; k++) {
        const hipError_t q = hipEventQuery(e->ev_rc[k]);
        if (q == hipErrorNotReady) done = false;
        else if (q != hipSuccess) lost = true;
      }
      if (lost) {  // a failed query: drop this readback rather than wait on it forever
        (void)hipGetLastError();
        e->rc_pending = false;
      } else if (done) {
        uint64_t h = 0;
        for (int k = 0; k < e->rc_lanes; k++)
          for (int r = 0; r < kNumRoutes; r++)
            if (e->h_rcounts[k * kNumRoutes + r] > 0) h |= 1ull << r;
        if (h & (1ull << kRtEnt11M)) h |= 1ull << kRtEnt11G;
        hint_store(e, e->rc_key, h);
        e->rc_pending = false;
      }
    }
    hint = hint_lookup(e, key);
    readback = !e->rc_pending;
  }
  const Lane first{e->descs, e->tables, e->d_etab, e->d_routes, e->d_total, nullptr};
  auto readback_queued = [&](int lanes) {  // every lane recorded its ev_rc: the next call may fold them
    if (!readback) return;
    e->rc_pending = true;
    e->rc_lanes = lanes;
    e->rc_key = key;
  };
  if (nl == 1) {
    const int st = run_lane(e, first, n, small, d_blob, blob_bytes, d_offsets, d_lengths, op, d_flip, d_out, d_status, s,
                            nullptr, rm, hint, readback ? 0 : -1);
    if (st == SDSJ_OK) readback_queued(1);
    return st;
  }
  for (int k = 0; k + 1 < nl; k++)
    if (!e->aux[k]) {
      SDSJ_HIP(e, hipStreamCreateWithFlags(&e->aux[k], hipStreamNonBlocking));
      SDSJ_HIP(e, hipEventCreateWithFlags(&e->ev_mid[k], hipEventDisableTiming));
      SDSJ_HIP(e, hipEventCreateWithFlags(&e->ev_join[k], hipEventDisableTiming));
    }
  const int64_t ob = out_bytes_per_image(op);
  const size_t rsz = (size_t)route_ints(e->max_batch);
  for (int k = 0; k < nl; k++) {
    const int i0 = (int)((int64_t)n * k / nl), i1 = (int)((int64_t)n * (k + 1) / nl);
    const Lane ln = k == 0 ? first
                           : Lane{e->descs + i0, e->tables + i0,
                                  static_cast<uint8_t*>(e->d_etab) + (size_t)i0 * enttab_bytes(),
                                  e->d_routes_x + (k - 1) * rsz, e->d_totals_x + (k - 1),
                                  k == 1 ? e->d_total : e->d_totals_x + (k - 2)};
    hipStream_t ls = k == 0 ? s : e->aux[k - 1];
    if (k > 0) SDSJ_HIP(e, hipStreamWaitEvent(ls, e->ev_mid[k - 1], 0));
    int st = run_lane(e, ln, i1 - i0, small, d_blob, blob_bytes, d_offsets + i0, d_lengths + i0, op, d_flip ? d_flip + i0 : nullptr,
                      static_cast<uint8_t*>(d_out) + i0 * ob, d_status + i0, ls,
                      k + 1 < nl ? e->ev_mid[k] : nullptr, rm, hint, readback ? k : -1);
    if (st != SDSJ_OK) return st;
  }
  readback_queued(nl);
  for (int k = 0; k + 1 < nl; k++) {
    SDSJ_HIP(e, hipEventRecord(e->ev_join[k], e->aux[k]));
    SDSJ_HIP(e, hipStreamWaitEvent(s, e->ev_join[k], 0));
  }
  return SDSJ_OK;
}

// -- asynchronous host path (sdsj_submit_*) ---------------------------------------------------
using Slot = sdsj_engine::Slot;

// Host staging (copies / file reads into pinned memory, header planning) is split over threads:
// a single core's memcpy bandwidth would otherwise bound the pipelined host path.
int stage_threads() {
  static const int k = [] {
    const char* v = getenv("SDSJ_STAGE_THREADS");
    const int hw = (int)std::thread::hardware_concurrency();
    const int d = std::max(1, std::min(8, hw > 0 ? hw : 1));
    return v ? std::max(1, atoi(v)) : d;
  }();
  return k;
}

}  // namespace

// The engine's staging threads, kept across calls: starting and joining 7 threads per parallel_for cost
// as much as the parallel memcpy saved (submit 1.29 ms serial vs 1.44 ms with 8 fresh threads per
// 256-image batch at 16 DataLoader workers, profiles/r06_f1_stage_threads.jsonl).  One call at a time;
// worker k runs part k of the current call's range and the caller runs part 0.
struct StagePool {
  std::vector<std::thread> th;
  std::mutex call_m, m;
  std::condition_variable go, done;
  std::function<void(int, int)> fn;
  int n = 0, nt = 0, left = 0;
  uint64_t gen = 0;
  bool stop = false;
  explicit StagePool(int workers) {
    for (int k = 1; k <= workers; k++) th.emplace_back([this, k] { run(k); });
  }
  ~StagePool() {
    {
      std::lock_guard<std::mutex> l(m);
      stop = true;
    }
    go.notify_all();
    for (auto& t : th) t.join();
  }
  void run(int k) {
    uint64_t seen = 0;
    for (;;) {
      std::function<void(int, int)> f;
      int a = 0, b = 0;
      {
        std::unique_lock<std::mutex> l(m);
        go.wait(l, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
        if (k >= nt) continue;
        f = fn;
        a = (int)((int64_t)n * k / nt);
        b = (int)((int64_t)n * (k + 1) / nt);
      }
      f(a, b);
      std::lock_guard<std::mutex> l(m);
      if (--left == 0) done.notify_one();
    }
  }
  void parallel_for(int n_, int nt_, const std::function<void(int, int)>& body) {
    std::lock_guard<std::mutex> cl(call_m);
    {
      std::lock_guard<std::mutex> l(m);
      fn = body;
      n = n_;
      nt = nt_;
      left = nt_ - 1;
      gen++;
    }
    go.notify_all();
    body(0, (int)((int64_t)n_ / nt_));
    std::unique_lock<std::mutex> l(m);
    done.wait(l, [&] { return left == 0; });
  }
};

namespace {

template <class F>
void parallel_for(sdsj_engine* e, int n, F fn) {
  const int nt = std::min(stage_threads(), std::max(1, n / 16));
  if (nt <= 1) {
    fn(0, n);
    return;
  }
  if (!e->pool) e->pool.reset(new StagePool(stage_threads() - 1));
  e->pool->parallel_for(n, nt, fn);
}

void slot_free(Slot& sl) {
  (void)hipHostFree(sl.h_stage);
  (void)hipFree(sl.d_blob);
  (void)hipHostFree(sl.h_offsets);
  (void)hipFree(sl.d_offsets);
  (void)hipHostFree(sl.h_lengths);
  (void)hipFree(sl.d_lengths);
  (void)hipHostFree(sl.h_flip);
  (void)hipFree(sl.d_flip);
  (void)hipHostFree(sl.h_status);
  (void)hipFree(sl.d_status);
  free(sl.h_pre);
  if (sl.ev_h2d) (void)hipEventDestroy(sl.ev_h2d);
  if (sl.ev_done) (void)hipEventDestroy(sl.ev_done);
  sl = Slot();
}

// Waits for the slot's previous batch (its pinned and device buffers are then free) and sizes the
// buffers for n samples / `bytes` staged bytes.
int slot_reserve(sdsj_engine* e, Slot& sl, int n, size_t bytes) {
  if (sl.pending) {
    SDSJ_HIP(e, hipEventSynchronize(sl.ev_done));
    sl.pending = false;
  }
  if (!e->copy_stream) SDSJ_HIP(e, hipStreamCreateWithFlags(&e->copy_stream, hipStreamNonBlocking));
  if (!sl.ev_done) {
    SDSJ_HIP(e, hipEventCreateWithFlags(&sl.ev_h2d, hipEventDisableTiming));
    SDSJ_HIP(e, hipEventCreateWithFlags(&sl.ev_done, hipEventDisableTiming));
  }
  if (n > sl.cap) {
    const int cap = std::max(n, 64);
    (void)hipHostFree(sl.h_offsets), (void)hipFree(sl.d_offsets), (void)hipHostFree(sl.h_lengths);
    (void)hipFree(sl.d_lengths), (void)hipHostFree(sl.h_flip), (void)hipFree(sl.d_flip);
    (void)hipHostFree(sl.h_status), (void)hipFree(sl.d_status), free(sl.h_pre);
    sl.h_pre = nullptr;
    sl.cap = 0;
    SDSJ_HIP(e, hipHostMalloc(&sl.h_offsets, sizeof(int64_t) * cap));
    SDSJ_HIP(e, hipMalloc(&sl.d_offsets, sizeof(int64_t) * cap));
    SDSJ_HIP(e, hipHostMalloc(&sl.h_lengths, sizeof(int32_t) * cap));
    SDSJ_HIP(e, hipMalloc(&sl.d_lengths, sizeof(int32_t) * cap));
    SDSJ_HIP(e, hipHostMalloc(&sl.h_flip, cap));
    SDSJ_HIP(e, hipMalloc(&sl.d_flip, cap));
    SDSJ_HIP(e, hipHostMalloc(&sl.h_status, sizeof(int32_t) * cap));
    SDSJ_HIP(e, hipMalloc(&sl.d_status, sizeof(int32_t) * cap));
    sl.h_pre = static_cast<int32_t*>(malloc(sizeof(int32_t) * cap));
    if (!sl.h_pre) return fail(e, SDSJ_ENOMEM, "host allocation failed");
    sl.cap = cap;
  }
  if (bytes > sl.bytes_cap) {
    (void)hipHostFree(sl.h_stage);
    (void)hipFree(sl.d_blob);
    sl.h_stage = nullptr;
    sl.d_blob = nullptr;
    sl.bytes_cap = 0;
    const size_t cap = std::max<size_t>(bytes * 3 / 2, 1 << 20);
    SDSJ_HIP(e, hipHostMalloc(&sl.h_stage, cap));
    SDSJ_HIP(e, hipMalloc(&sl.d_blob, cap));
    sl.bytes_cap = cap;
  }
  return SDSJ_OK;
}

// The staged batch: scratch sized from host planning, H2D on the copy stream, the decode on `s`
// behind that copy, status D2H into pinned memory, completion event.
int slot_launch(sdsj_engine* e, Slot& sl, int n, size_t bytes, const sdsj_op& op, void* out, hipStream_t s) {
  std::vector<int64_t> needs(n, 0);
  const bool small = n <= kSmallBatch;
  std::atomic<uint64_t> rmask{0};  // the routes the batch takes (launchers skip the others)
  parallel_for(e, n, [&](int i0, int i1) {
    uint64_t rm = 0;
    for (int i = i0; i < i1; i++) {
      if (sl.h_pre[i] != SDSJ_OK) continue;
      int st = SDSJ_OK;
      uint64_t r = 0;
      const int64_t ni = host_plan_need(sl.h_stage + sl.h_offsets[i], sl.h_lengths[i], op, &st, &r, small);
      if (st == SDSJ_OK) needs[i] = align_up(ni, 256);
      rm |= r;
    }
    rmask.fetch_or(rm);
  });
  int64_t need = 0;
  for (int i = 0; i < n; i++) need += needs[i];
  if (need > e->capacity || !e->scratch) {
    if (e->scratch && !e->grow) return fail(e, SDSJ_ECAPACITY, "batch exceeds the configured scratch capacity");
    SDSJ_HIP(e, hipStreamSynchronize(s));
    const int st = ensure_scratch(e, need);
    if (st != SDSJ_OK) return st;
  }
  hipStream_t cs = e->copy_stream;
  SDSJ_HIP(e, hipMemcpyAsync(sl.d_blob, sl.h_stage, bytes, hipMemcpyHostToDevice, cs));
  SDSJ_HIP(e, hipMemcpyAsync(sl.d_offsets, sl.h_offsets, sizeof(int64_t) * n, hipMemcpyHostToDevice, cs));
  SDSJ_HIP(e, hipMemcpyAsync(sl.d_lengths, sl.h_lengths, sizeof(int32_t) * n, hipMemcpyHostToDevice, cs));
  SDSJ_HIP(e, hipMemcpyAsync(sl.d_flip, sl.h_flip, n, hipMemcpyHostToDevice, cs));
  SDSJ_HIP(e, hipEventRecord(sl.ev_h2d, cs));
  SDSJ_HIP(e, hipStreamWaitEvent(s, sl.ev_h2d, 0));
  const int rc = run_chunk(e, n, sl.d_blob, (int64_t)bytes, sl.d_offsets, sl.d_lengths, op, sl.d_flip, out, sl.d_status, s,
                           rmask.load(), small);
  if (rc != SDSJ_OK) return rc;
  SDSJ_HIP(e, hipMemcpyAsync(sl.h_status, sl.d_status, sizeof(int32_t) * n, hipMemcpyDeviceToHost, s));
  SDSJ_HIP(e, hipEventRecord(sl.ev_done, s));
  sl.n = n;
  sl.pending = true;
  return SDSJ_OK;
}

int64_t file_size(const char* path) {
  struct stat sb;
  if (!path || stat(path, &sb) != 0 || !S_ISREG(sb.st_mode)) return -1;
  return (int64_t)sb.st_size;
}

// Reads exactly `size` bytes of `path` into dst; false on any error or a short file.
bool read_file(const char* path, uint8_t* dst, int64_t size) {
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  int64_t got = 0;
  while (got < size) {
    const ssize_t r = read(fd, dst + got, (size_t)std::min<int64_t>(size - got, 1 << 30));
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) break;
    got += r;
  }
  close(fd);
  return got == size;
}

}  // namespace

extern "C" {

int sdsj_abi_version(void) { return SDSJ_ABI_VERSION; }

int sdsj_submit_batch(sdsj_engine* e, int slot, int n, const uint8_t* const* jpg, const size_t* len, const sdsj_op* op,
                      const uint8_t* flip, void* out, void* hip_stream) {
  if (!e) return SDSJ_EINVAL;
  if (slot < 0 || slot >= SDSJ_SLOTS || n < 0 || n > e->max_batch || (n > 0 && (!jpg || !len || !out)) ||
      !valid_op(op))
    return fail(e, SDSJ_EINVAL, "invalid argument");
  DeviceGuard g(e->device);
  Slot& sl = e->slots[slot];
  size_t bytes = 0;
  for (int i = 0; i < n; i++) {
    if (len[i] > (size_t)INT32_MAX) return fail(e, SDSJ_EINVAL, "sample larger than 2 GiB");
    bytes += align_up((int64_t)len[i], 16);
  }
  int rc = slot_reserve(e, sl, std::max(n, 1), std::max<size_t>(bytes, 16));
  if (rc != SDSJ_OK) return rc;
  int64_t off = 0;
  for (int i = 0; i < n; i++) {
    sl.h_offsets[i] = off;
    sl.h_lengths[i] = (int32_t)len[i];
    sl.h_flip[i] = flip ? flip[i] : 0;
    sl.h_pre[i] = SDSJ_OK;
    off += align_up((int64_t)len[i], 16);
  }
  parallel_for(e, n, [&](int i0, int i1) {
    for (int i = i0; i < i1; i++) memcpy(sl.h_stage + sl.h_offsets[i], jpg[i], len[i]);
  });
  if (n == 0) {
    sl.n = 0;
    sl.pending = true;
    return hipEventRecord(sl.ev_done, reinterpret_cast<hipStream_t>(hip_stream)) == hipSuccess ? SDSJ_OK : SDSJ_EHIP;
  }
  return slot_launch(e, sl, n, (size_t)off, *op, out, reinterpret_cast<hipStream_t>(hip_stream));
}

int sdsj_submit_files(sdsj_engine* e, int slot, int n, const char* const* paths, const sdsj_op* op,
                      const uint8_t* flip, void* out, void* hip_stream) {
  if (!e) return SDSJ_EINVAL;
  if (slot < 0 || slot >= SDSJ_SLOTS || n < 0 || n > e->max_batch || (n > 0 && (!paths || !out)) || !valid_op(op))
    return fail(e, SDSJ_EINVAL, "invalid argument");
  DeviceGuard g(e->device);
  Slot& sl = e->slots[slot];
  std::vector<int64_t> sizes(n);
  parallel_for(e, n, [&](int i0, int i1) {
    for (int i = i0; i < i1; i++) {
      sizes[i] = file_size(paths[i]);
      if (sizes[i] > INT32_MAX) sizes[i] = -1;
    }
  });
  size_t bytes = 0;
  for (int i = 0; i < n; i++)
    if (sizes[i] > 0) bytes += align_up(sizes[i], 16);
  int rc = slot_reserve(e, sl, std::max(n, 1), std::max<size_t>(bytes, 16));
  if (rc != SDSJ_OK) return rc;
  int64_t off = 0;
  for (int i = 0; i < n; i++) {
    sl.h_offsets[i] = off;
    sl.h_flip[i] = flip ? flip[i] : 0;
    if (sizes[i] > 0) off += align_up(sizes[i], 16);
  }
  parallel_for(e, n, [&](int i0, int i1) {
    for (int i = i0; i < i1; i++) {
      const bool ok = sizes[i] >= 0 && read_file(paths[i], sl.h_stage + sl.h_offsets[i], sizes[i]);
      sl.h_lengths[i] = ok ? (int32_t)sizes[i] : -1;  // (k_finish reports a negative length as EINVAL, counted "other")
      sl.h_pre[i] = ok ? SDSJ_OK : SDSJ_EINVAL;
    }
  });
  if (n == 0) {
    sl.n = 0;
    sl.pending = true;
    return hipEventRecord(sl.ev_done, reinterpret_cast<hipStream_t>(hip_stream)) == hipSuccess ? SDSJ_OK : SDSJ_EHIP;
  }
  return slot_launch(e, sl, n, (size_t)std::max<int64_t>(off, 16), *op, out, reinterpret_cast<hipStream_t>(hip_stream));
}

int sdsj_wait_batch(sdsj_engine* e, int slot, int32_t* status) {
  if (!e) return SDSJ_EINVAL;
  if (slot < 0 || slot >= SDSJ_SLOTS || !e->slots[slot].pending) return fail(e, SDSJ_EINVAL, "no batch in flight on slot");
  DeviceGuard g(e->device);
  Slot& sl = e->slots[slot];
  SDSJ_HIP(e, hipEventSynchronize(sl.ev_done));
  sl.pending = false;
  if (status)  // (an unreadable file went to the device with length -1: k_finish reports it EINVAL)
    for (int i = 0; i < sl.n; i++) status[i] = sl.h_pre[i] != SDSJ_OK ? sl.h_pre[i] : sl.h_status[i];
  return SDSJ_OK;
}

int sdsj_probe(const uint8_t* jpg, size_t n, sdsj_info* out) {
  if (!jpg || !out) return SDSJ_EINVAL;
  memset(out, 0, sizeof(*out));
  ImgDesc d;
  static thread_local ImgTables t;
  struct R {
    const uint8_t* p;
    int operator()(int64_t i) const { return p[i]; }
  } rd{jpg};
  int st = parse_headers(rd, (int64_t)n, &d, &t, CopySink<R>{rd});
  out->width = d.width;
  out->height = d.height;
  out->ncomp = d.ncomp;
  if (st == SDSJ_OK) st = setup_geometry(&d, &t);
  for (int c = 0; st == SDSJ_OK && !d.progressive && c < d.ncomp; c++)  // (progressive: checked per scan)
    if (!huff_table_ok(t.dc_spec[d.comp[c].td], true) || !huff_table_ok(t.ac_spec[d.comp[c].ta], false))
      st = SDSJ_CORRUPT;
  for (int c = 0; c < d.ncomp && c < 3; c++) {
    out->h_samp[c] = d.comp[c].h;
    out->v_samp[c] = d.comp[c].v;
  }
  out->restart_interval = d.restart_interval;
  out->entropy_offset = st == SDSJ_OK ? d.entropy_off : 0;
  out->supported = st == SDSJ_OK;
  return st;
}

int sdsj_plan_need(const uint8_t* jpg, size_t n, const sdsj_op* op, int64_t* need) {
  if (!jpg || !need || !valid_op(op)) return SDSJ_EINVAL;
  int st = SDSJ_OK;
  const int64_t b = host_plan_need(jpg, (int64_t)n, *op, &st);
  *need = st == SDSJ_OK ? align_up(b, 256) : 0;
  return st;
}

int sdsj_engine_create(int hip_device, const sdsj_cfg* cfg, sdsj_engine** out) {
  if (!out) return SDSJ_EINVAL;
  *out = nullptr;
  if (cfg && cfg->abi_version != SDSJ_ABI_VERSION) return SDSJ_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || hip_device < 0 || hip_device >= ndev) return SDSJ_EHIP;
  sdsj_engine* e = new (std::nothrow) sdsj_engine();
  if (!e) return SDSJ_ENOMEM;
  e->device = hip_device;
  if (const char* w = getenv("SDSJ_WARM_BITS")) e->warm_bits = atoi(w);
  if (cfg && cfg->max_batch > 0) e->max_batch = cfg->max_batch;
  DeviceGuard g(hip_device);
  int st = SDSJ_OK;
  auto cleanup = [&](int code) {
    sdsj_engine_destroy(e);
    return code;
  };
  if (hipMalloc(&e->descs, sizeof(ImgDesc) * e->max_batch) != hipSuccess) return cleanup(SDSJ_ENOMEM);
  if (hipMalloc(&e->tables, sizeof(ImgTables) * e->max_batch) != hipSuccess) return cleanup(SDSJ_ENOMEM);
  if (const char* l = getenv("SDSJ_LANES")) e->lanes = atoi(l);
  if (const char* l = getenv("SDSJ_LANE_MID")) e->lane_mid = atoi(l);
  if (e->lane_mid >= 0 && e->lane_mid < 2) e->lane_mid = 2;  // a lane's k_plan reads the previous lane's total
  if (hipMalloc(&e->d_total, sizeof(int64_t)) != hipSuccess) return cleanup(SDSJ_ENOMEM);
  if (hipMalloc(&e->d_totals_x, sizeof(int64_t) * (kMaxLanes - 1)) != hipSuccess) return cleanup(SDSJ_ENOMEM);
  if (hipMalloc(&e->d_routes_x, sizeof(int32_t) * (kMaxLanes - 1) * (size_t)route_ints(e->max_batch)) !=
      hipSuccess)
    return cleanup(SDSJ_ENOMEM);
  if (hipMalloc(&e->d_etab, enttab_bytes() * e->max_batch) != hipSuccess) return cleanup(SDSJ_ENOMEM);
  if (hipMalloc(&e->d_routes, sizeof(int32_t) * (size_t)route_ints(e->max_batch)) != hipSuccess)
    return cleanup(SDSJ_ENOMEM);
  if (hipMalloc(&e->d_lut, sizeof(float) * 256) != hipSuccess) return cleanup(SDSJ_ENOMEM);
  if (hipHostMalloc(&e->h_rcounts, sizeof(int32_t) * kMaxLanes * kNumRoutes) != hipSuccess) return cleanup(SDSJ_ENOMEM);
  for (int k = 0; k < kMaxLanes; k++)
    if (hipEventCreateWithFlags(&e->ev_rc[k], hipEventDisableTiming) != hipSuccess) return cleanup(SDSJ_EHIP);
  if (hipMalloc(&e->d_counters, sizeof(unsigned long long) * SDSJ_NUM_COUNTERS) != hipSuccess) return cleanup(SDSJ_ENOMEM);
  if (hipMemset(e->d_counters, 0, sizeof(unsigned long long) * SDSJ_NUM_COUNTERS) != hipSuccess) return cleanup(SDSJ_EHIP);
  {
    // presets.py:161 `x.float() / 127.5 - 1.0` in float32 (IEEE division then subtraction)
    float lut[256];
    volatile float div = 127.5f, one = 1.0f;
    for (int v = 0; v < 256; v++) {
      float q = (float)v / div;
      lut[v] = q - one;
    }
    if (hipMemcpy(e->d_lut, lut, sizeof(lut), hipMemcpyHostToDevice) != hipSuccess) return cleanup(SDSJ_EHIP);
  }
  if (cfg && cfg->scratch_bytes > 0) {
    e->grow = false;
    st = ensure_scratch(e, cfg->scratch_bytes);
    if (st != SDSJ_OK) return cleanup(st);
  }
  *out = e;
  return SDSJ_OK;
}

int sdsj_engine_destroy(sdsj_engine* e) {
  if (!e) return SDSJ_EINVAL;
  DeviceGuard g(e->device);
  (void)hipDeviceSynchronize();
  (void)hipFree(e->scratch);
  (void)hipFree(e->descs);
  (void)hipFree(e->tables);
  (void)hipFree(e->d_total);
  (void)hipFree(e->d_routes);
  (void)hipFree(e->d_etab);
  (void)hipFree(e->d_totals_x);
  (void)hipFree(e->d_routes_x);
  for (auto& sl : e->slots) slot_free(sl);
  if (e->copy_stream) (void)hipStreamDestroy(e->copy_stream);
  for (int k = 0; k + 1 < kMaxLanes; k++) {
    if (e->aux[k]) (void)hipStreamDestroy(e->aux[k]);
    if (e->ev_mid[k]) (void)hipEventDestroy(e->ev_mid[k]);
    if (e->ev_join[k]) (void)hipEventDestroy(e->ev_join[k]);
  }
  for (int k = 0; k < kMaxLanes; k++)
    if (e->ev_rc[k]) (void)hipEventDestroy(e->ev_rc[k]);
  (void)hipHostFree(e->h_rcounts);
  (void)hipHostFree(e->h_fdescs);
  (void)hipHostFree(e->h_froutes);
  (void)hipFree(e->d_lut);
  (void)hipFree(e->d_counters);
  (void)hipFree(e->d_blob);
  (void)hipFree(e->d_offsets);
  (void)hipFree(e->d_lengths);
  (void)hipFree(e->d_flip);
  (void)hipFree(e->d_status);
  (void)hipHostFree(e->h_stage);
  (void)hipHostFree(e->h_offsets);
  (void)hipHostFree(e->h_lengths);
  (void)hipHostFree(e->h_flip);
  (void)hipHostFree(e->h_status);
  for (auto& set : e->ev_sets)
    for (auto ev : set) (void)hipEventDestroy(ev);
  delete e;
  return SDSJ_OK;
}

int sdsj_decode_resize_batch_device(sdsj_engine* e, int n, const uint8_t* d_blob, size_t blob_bytes,
                                    const int64_t* d_offsets, const int32_t* d_lengths, const sdsj_op* op,
                                    const uint8_t* d_flip, void* d_out, int32_t* d_status, void* hip_stream) {
  if (!e) return SDSJ_EINVAL;
  if (n < 0 || (n > 0 && (!d_blob || !d_offsets || !d_lengths || !d_out || !d_status)) || !valid_op(op))
    return fail(e, SDSJ_EINVAL, "invalid argument");
  if (n == 0) return SDSJ_OK;
  DeviceGuard g(e->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(hip_stream);
  if (!e->scratch) {
    int st = ensure_scratch(e, (int64_t)2 << 30);
    if (st != SDSJ_OK) return st;
  }
  const int64_t ob = out_bytes_per_image(*op);
  for (int c0 = 0; c0 < n; c0 += e->max_batch) {
    int m = std::min(e->max_batch, n - c0);
    int st = run_chunk(e, m, d_blob, (int64_t)blob_bytes, d_offsets + c0, d_lengths + c0, *op, d_flip ? d_flip + c0 : nullptr,
                       reinterpret_cast<uint8_t*>(d_out) + c0 * ob, d_status + c0, s);
    if (st != SDSJ_OK) return st;
  }
  return SDSJ_OK;
}

int sdsj_decode_resize_batch(sdsj_engine* e, int n, const uint8_t* const* jpg, const size_t* len, const sdsj_op* op,
                             const uint8_t* flip, void* out, int32_t* status, void* hip_stream) {
  if (!e) return SDSJ_EINVAL;
  if (n < 0 || (n > 0 && (!jpg || !len || !out || !status)) || !valid_op(op))
    return fail(e, SDSJ_EINVAL, "invalid argument");
  if (n == 0) return SDSJ_OK;
  DeviceGuard g(e->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(hip_stream);
  const int64_t ob = out_bytes_per_image(*op);
  int rc = ensure_io(e, std::min(n, e->max_batch));
  if (rc != SDSJ_OK) return rc;
  for (int c0 = 0; c0 < n; c0 += e->max_batch) {
    int m = std::min(e->max_batch, n - c0);
    const bool small = m <= kSmallBatch;
    // host planning: exact scratch need of this chunk (same code as k_parse / k_plan)
    int64_t need = 0, bytes = 0;
    uint64_t rm = 0;  // the routes the chunk takes (launchers skip the others)
    for (int i = 0; i < m; i++) {
      int st = SDSJ_OK;
      if (len[c0 + i] > (size_t)INT32_MAX) return fail(e, SDSJ_EINVAL, "sample larger than 2 GiB");
      uint64_t r = 0;
      int64_t ni = host_plan_need(jpg[c0 + i], (int64_t)len[c0 + i], *op, &st, &r, small);
      if (st == SDSJ_OK) need += align_up(ni, 256);
      rm |= r;
      bytes += align_up((int64_t)len[c0 + i], 16);
    }
    if (need > e->capacity) {
      if (!e->grow) return fail(e, SDSJ_ECAPACITY, "batch exceeds the configured scratch capacity");
      SDSJ_HIP(e, hipStreamSynchronize(s));
      rc = ensure_scratch(e, need);
      if (rc != SDSJ_OK) return rc;
    }
    // one staging region, one H2D copy: the samples, then their offsets, lengths and flip flags
    const int64_t meta = align_up(bytes, 16);
    const int64_t staged = meta + align_up((int64_t)m * 8, 16) + align_up((int64_t)m * 4, 16) + align_up(m, 16);
    if ((size_t)staged > e->h_stage_cap) {
      SDSJ_HIP(e, hipStreamSynchronize(s));
      (void)hipHostFree(e->h_stage);
      (void)hipFree(e->d_blob);
      e->h_stage = nullptr;
      e->d_blob = nullptr;
      e->h_stage_cap = e->d_blob_cap = 0;
      size_t cap = std::max<size_t>((size_t)staged * 3 / 2, 1 << 20);
      SDSJ_HIP(e, hipHostMalloc(&e->h_stage, cap));
      SDSJ_HIP(e, hipMalloc(&e->d_blob, cap));
      e->h_stage_cap = e->d_blob_cap = cap;
    }
    // the staging buffers are reused: wait for the previous chunk's H2D to finish
    SDSJ_HIP(e, hipStreamSynchronize(s));
    const int64_t o_off = meta, o_len = o_off + align_up((int64_t)m * 8, 16), o_flip = o_len + align_up((int64_t)m * 4, 16);
    int64_t* h_off = reinterpret_cast<int64_t*>(e->h_stage + o_off);
    int32_t* h_len = reinterpret_cast<int32_t*>(e->h_stage + o_len);
    uint8_t* h_fl = e->h_stage + o_flip;
    int64_t off = 0;
    for (int i = 0; i < m; i++) {
      memcpy(e->h_stage + off, jpg[c0 + i], len[c0 + i]);
      h_off[i] = off;
      h_len[i] = (int32_t)len[c0 + i];
      h_fl[i] = flip ? flip[c0 + i] : 0;
      off += align_up((int64_t)len[c0 + i], 16);
    }
    SDSJ_HIP(e, hipMemcpyAsync(e->d_blob, e->h_stage, (size_t)staged, hipMemcpyHostToDevice, s));
    rc = run_chunk(e, m, e->d_blob, off, reinterpret_cast<const int64_t*>(e->d_blob + o_off),
                   reinterpret_cast<const int32_t*>(e->d_blob + o_len), *op, e->d_blob + o_flip,
                   reinterpret_cast<uint8_t*>(out) + c0 * ob, e->d_status, s, rm, small);
    if (rc != SDSJ_OK) return rc;
    SDSJ_HIP(e, hipMemcpyAsync(e->h_status, e->d_status, sizeof(int32_t) * m, hipMemcpyDeviceToHost, s));
    SDSJ_HIP(e, hipStreamSynchronize(s));
    memcpy(status + c0, e->h_status, sizeof(int32_t) * m);
  }
  return SDSJ_OK;
}

int sdsj_resize_frames_device(sdsj_engine* e, int n, const uint8_t* d_frames, int32_t width, int32_t height,
                              int64_t frame_stride, const sdsj_op* op, const uint8_t* d_flip, void* d_out,
                              int32_t* d_status, void* hip_stream) {
  if (!e) return SDSJ_EINVAL;
  if (n < 0 || (n > 0 && (!d_frames || !d_out || !d_status)) || !valid_op(op) || width <= 0 || height <= 0 ||
      width > 65535 || height > 65535 || frame_stride < (int64_t)width * height * 3)
    return fail(e, SDSJ_EINVAL, "invalid argument");
  if (n == 0) return SDSJ_OK;
  DeviceGuard g(e->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(hip_stream);
  ImgDesc base;
  const int64_t need = align_up(host_plan_frame(&base, width, height, *op), 256);
  const int cap = e->max_batch;
  if (!e->h_fdescs) {
    SDSJ_HIP(e, hipHostMalloc(&e->h_fdescs, sizeof(ImgDesc) * cap));
    SDSJ_HIP(e, hipHostMalloc(&e->h_froutes, sizeof(int32_t) * (kRouteSlots + cap)));
  }
  const int64_t ob = out_bytes_per_image(*op);
  for (int c0 = 0; c0 < n; c0 += cap) {
    const int m = std::min(cap, n - c0);
    if (!e->scratch || need * m > e->capacity) {
      if (e->scratch && !e->grow) return fail(e, SDSJ_ECAPACITY, "frames exceed the configured scratch capacity");
      SDSJ_HIP(e, hipStreamSynchronize(s));
      int rc = ensure_scratch(e, std::max<int64_t>(need * m, (int64_t)256 << 20));
      if (rc != SDSJ_OK) return rc;
    }
    SDSJ_HIP(e, hipStreamSynchronize(s));  // the pinned staging is reused chunk to chunk
    for (int k = 0; k < m; k++) {
      ImgDesc& d = e->h_fdescs[k];
      d = base;
      const int64_t o = need * k;
      d.off_ustream += o;
      d.off_seg += o;
      d.off_tiles += o;
      d.off_sub += o;
      d.off_rec += o;
      d.off_ptab += o;
      d.off_coef += o;
      d.off_planes += o;
      d.off_tmp += o;
      d.off_kh += o;
      d.off_kv += o;
      // the passes read the frame's crop rows in place: scratch + off_rgb = the crop's first pixel
      const uint8_t* px = d_frames + (int64_t)(c0 + k) * frame_stride + ((int64_t)d.src_y0 * width + d.src_x0) * 3;
      d.off_rgb = (int64_t)(px - e->scratch);
      d.rgb_pitch = width;
    }
    for (int r = 0; r < kRouteSlots; r++) e->h_froutes[r] = 0;
    e->h_froutes[kRtUnfused] = m;
    for (int k = 0; k < m; k++) e->h_froutes[kRouteSlots + kRtUnfused * cap + k] = k;
    SDSJ_HIP(e, hipMemcpyAsync(e->descs, e->h_fdescs, sizeof(ImgDesc) * m, hipMemcpyHostToDevice, s));
    SDSJ_HIP(e, hipMemcpyAsync(e->d_routes, e->h_froutes, sizeof(int32_t) * (kRouteSlots + m), hipMemcpyHostToDevice, s));
    void* out = reinterpret_cast<uint8_t*>(d_out) + c0 * ob;
    const uint8_t* flip = d_flip ? d_flip + c0 : nullptr;
    SDSJ_HIP(e, launch_coeffs(m, e->descs, *op, e->scratch, s));
    SDSJ_HIP(e, launch_hpass(m, e->descs, *op, e->scratch, e->d_routes, cap, s));
    SDSJ_HIP(e, launch_vpass(m, e->descs, *op, e->scratch, flip, out, e->d_routes, cap, e->d_lut, s));
    SDSJ_HIP(e, launch_finish(m, e->descs, *op, out, d_status + c0, e->d_lut, nullptr, e->d_counters, s));
  }
  return SDSJ_OK;
}

int sdsj_engine_set_timing(sdsj_engine* e, int enable) {
  if (!e) return SDSJ_EINVAL;
  e->timing = enable != 0;
  e->ev_used = 0;  // restart accumulation
  return SDSJ_OK;
}

int sdsj_engine_stage_times(const sdsj_engine* e, float* ms, int cap, int* n_stages) {
  if (!e || !n_stages || (cap > 0 && !ms)) return SDSJ_EINVAL;
  *n_stages = kStages;
  for (int k = 0; k < cap && k < kStages; k++) ms[k] = 0.f;
  if (!e->timing || e->ev_used == 0) return SDSJ_OK;
  DeviceGuard g(e->device);
  for (size_t c = 0; c < e->ev_used; c++)  // lanes run on two streams: wait for every set
    if (hipEventSynchronize(e->ev_sets[c][kStages]) != hipSuccess) return SDSJ_EHIP;
  for (size_t c = 0; c < e->ev_used; c++) {
    for (int k = 0; k < cap && k < kStages; k++) {
      float v = 0.f;
      if (hipEventElapsedTime(&v, e->ev_sets[c][k], e->ev_sets[c][k + 1]) != hipSuccess) return SDSJ_EHIP;
      ms[k] += v;
    }
  }
  return SDSJ_OK;
}

const char* sdsj_last_error(const sdsj_engine* e) {
  if (!e) return "null engine";
  return e->err.c_str();
}

int sdsj_engine_debug_buffers(const sdsj_engine* e, void** scratch, void** descs, int64_t* desc_bytes,
                              int64_t* scratch_bytes) {
  if (!e || !scratch || !descs || !desc_bytes || !scratch_bytes) return SDSJ_EINVAL;
  *scratch = e->scratch;
  *descs = e->descs;
  *desc_bytes = (int64_t)sizeof(ImgDesc);
  *scratch_bytes = e->capacity;
  return SDSJ_OK;
}

const char* sdsj_stage_name(int k) { return k >= 0 && k < kStages ? kStageNames[k] : ""; }

int sdsj_engine_counters(sdsj_engine* e, uint64_t* out, int cap, int reset) {
  if (!e || (cap > 0 && !out)) return SDSJ_EINVAL;
  DeviceGuard g(e->device);
  unsigned long long h[SDSJ_NUM_COUNTERS];
  SDSJ_HIP(e, hipDeviceSynchronize());
  SDSJ_HIP(e, hipMemcpy(h, e->d_counters, sizeof(h), hipMemcpyDeviceToHost));
  for (int k = 0; k < cap && k < SDSJ_NUM_COUNTERS; k++) out[k] = (uint64_t)h[k];
  if (reset) {
    SDSJ_HIP(e, hipMemset(e->d_counters, 0, sizeof(h)));
  }
  return SDSJ_OK;
}

const char* sdsj_counter_name(int k) {
  static const char* names[SDSJ_NUM_COUNTERS] = {"images",    "ok",        "unsupported", "corrupt", "capacity",
                                                 "other",     "bytes_in",  "bytes_out",   "frames",  "progressive"};
  return k >= 0 && k < SDSJ_NUM_COUNTERS ? names[k] : "";
}

int sdsj_engine_set_lanes(sdsj_engine* e, int lanes) {
  if (!e || lanes < 1 || lanes > kMaxLanes) return SDSJ_EINVAL;
  e->lanes = lanes;
  return SDSJ_OK;
}

int sdsj_engine_reserve(sdsj_engine* e, int64_t bytes) {
  if (!e || bytes < 0) return SDSJ_EINVAL;
  DeviceGuard g(e->device);
  if (bytes <= e->capacity && e->scratch) return SDSJ_OK;
  SDSJ_HIP(e, hipDeviceSynchronize());
  return ensure_scratch(e, bytes);
}

}  // extern "C"
