/*
 * sdsj.h -- C-ABI of the MI355X-native JPEG decode + crop/resize/flip/normalise path.
 *
 * The reference (snap-research/sds) has no native boundary: its image hot path is the Python
 * transform list built by create_standard_image_pipeline (sds/transforms/presets.py:716-744),
 * whose arithmetic runs in Pillow/libjpeg-turbo.  Each entry point below replaces one piece of
 * that list; the Python drop-in (sds_amd/presets.py) binds them with ctypes, exactly as a
 * maintainer would add a ctypes stub to sds (INTEGRATION.md shows that binding):
 *
 *   sdsj_probe                      <- PIL.Image.open() header parse inside
 *                                      load_image_from_bytes (functional.py:94-100)
 *   sdsj_decode_resize_batch        <- DecodeImageTransform (presets.py:39-45) +
 *                                      ResizeImageTransform (presets.py:47-58 -> functional.py:38-86,
 *                                      crop functional.py:118-147) +
 *                                      ConvertImageToByteTensorTransform (presets.py:68-74 ->
 *                                      functional.py:102-110) + optional
 *                                      NormalizeFramesTransform (presets.py:154-162) and the
 *                                      user hflip (README.md:99-108), inputs in host memory
 *   sdsj_decode_resize_batch_device <- the same, inputs already resident in device memory
 *                                      (the device-resident benchmark, configs 2-4)
 *   sdsj_engine_create/destroy      <- (no reference counterpart: per-process GPU state that the
 *                                      transform creates lazily, presets.py:1-5 pickling rule)
 *
 * Conventions: plain C types only; every function returns an int status (0 = SDSJ_OK, < 0 an
 * error) and never throws; pointers are borrowed for the duration of the call.  All device work
 * is enqueued on the caller's HIP stream (hipStream_t passed as void*).
 */
#ifndef SDSJ_H
#define SDSJ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDSJ_ABI_VERSION 2 /* 2: blob_bytes on the device entry point */

/* status codes (per call and per sample) */
#define SDSJ_OK 0
#define SDSJ_EINVAL (-1)      /* bad argument */
#define SDSJ_UNSUPPORTED (-2) /* valid JPEG the MI355X path does not decode (arithmetic, 12-bit, CMYK, ...) */
#define SDSJ_CORRUPT (-3)     /* malformed / truncated stream (PIL raises OSError) */
#define SDSJ_ENOMEM (-4)      /* allocation failed */
#define SDSJ_EHIP (-5)        /* HIP runtime error (see sdsj_last_error) */
#define SDSJ_ECAPACITY (-6)   /* sample did not fit the engine's scratch; resubmit in a smaller batch */

/* resampling filters (Pillow Image.Resampling numbering is not used; see sds_amd/presets.py) */
#define SDSJ_FILTER_BOX 0
#define SDSJ_FILTER_BILINEAR 1
#define SDSJ_FILTER_HAMMING 2
#define SDSJ_FILTER_BICUBIC 3
#define SDSJ_FILTER_LANCZOS 4
#define SDSJ_FILTER_NEAREST 5 /* Pillow NEAREST (ImagingScaleAffine), torchvision 'nearest' / 'nearest-exact' on PIL */

#define SDSJ_DTYPE_U8 0  /* uint8 samples, as ConvertImageToByteTensorTransform */
#define SDSJ_DTYPE_F32 1 /* float32 x/127.5-1, as NormalizeFramesTransform */

#define SDSJ_LAYOUT_CHW 0 /* [3][H][W] contiguous */
#define SDSJ_LAYOUT_HWC 1 /* [H][W][3] contiguous (the reference's storage order, functional.py:104-108) */

typedef struct sdsj_info {
    int32_t width, height; /* image size (PIL Image.size order: width, height) */
    int32_t ncomp;         /* 1 (grayscale) or 3 (YCbCr) */
    int32_t h_samp[3], v_samp[3];
    int32_t restart_interval;
    int32_t supported; /* 1 if the MI355X path decodes it */
    int64_t entropy_offset;
} sdsj_info;

typedef struct sdsj_cfg {
    int32_t abi_version;     /* must be SDSJ_ABI_VERSION */
    int32_t max_batch;       /* images per internal launch (0 = default 4096) */
    int64_t scratch_bytes;   /* device scratch capacity; 0 = grow on demand (host API) / 2 GiB */
} sdsj_cfg;

typedef struct sdsj_op {
    int32_t out_h, out_w;        /* target resolution, the reference's (h, w) tuple (functional.py:76) */
    int32_t crop_before_resize;  /* functional.py:45 (default 1): centre crop to out_w/out_h first */
    int32_t filter;              /* SDSJ_FILTER_*; the reference default is bilinear (functional.py:48) */
    int32_t out_dtype;           /* SDSJ_DTYPE_* */
    int32_t layout;              /* SDSJ_LAYOUT_* */
} sdsj_op;

typedef struct sdsj_engine sdsj_engine;

int sdsj_abi_version(void);

/* Host-side header parse of one JPEG (no GPU needed). */
int sdsj_probe(const uint8_t* jpg, size_t n, sdsj_info* out);

/* Device scratch one JPEG needs for `op` (host planning, no GPU): *need = bytes (256-aligned share of
 * the engine's scratch).  Returns the header status (SDSJ_OK, SDSJ_UNSUPPORTED, SDSJ_CORRUPT); a
 * batch on the device-resident entry point needs the sum over its samples (sdsj_engine_reserve). */
int sdsj_plan_need(const uint8_t* jpg, size_t n, const sdsj_op* op, int64_t* need);

/* Creates an engine bound to HIP device `hip_device`.  Scratch memory is owned by the engine. */
int sdsj_engine_create(int hip_device, const sdsj_cfg* cfg, sdsj_engine** out);
int sdsj_engine_destroy(sdsj_engine* eng);

/* Decode + crop + resize (+flip, +normalise) of n JPEGs held in HOST memory.
 *   jpg[i], len[i]  : encoded bytes of sample i (borrowed)
 *   flip            : host array of n bytes (1 = horizontal flip) or NULL
 *   out             : device pointer to n * out_h * out_w * 3 elements of op->out_dtype, laid
 *                     out per op->layout, sample-major; allocated by the caller (torch).  Pinned
 *                     host memory (hipHostMalloc / torch pin_memory) is device-accessible and works
 *                     too: the kernels then store the pixels over PCIe (no separate D2H copy)
 *   status          : host array of n ints, per-sample SDSJ_* code (filled before return)
 * Synchronises `hip_stream` before returning (status is host memory). */
int sdsj_decode_resize_batch(sdsj_engine* eng, int n, const uint8_t* const* jpg, const size_t* len,
                             const sdsj_op* op, const uint8_t* flip, void* out, int32_t* status,
                             void* hip_stream);

/* Same with inputs already in DEVICE memory: sample i is d_blob[d_offsets[i] .. + d_lengths[i]) of the
 * blob_bytes-byte buffer d_blob; a sample whose range is negative or leaves the buffer reports
 * SDSJ_EINVAL (checked on the device before anything reads it).  d_flip (n bytes) may be NULL;
 * d_status is a device array of n ints.  Fully asynchronous on `hip_stream` (no host
 * synchronisation, capturable into a hipGraph for a fixed n). */
int sdsj_decode_resize_batch_device(sdsj_engine* eng, int n, const uint8_t* d_blob, size_t blob_bytes,
                                    const int64_t* d_offsets, const int32_t* d_lengths, const sdsj_op* op,
                                    const uint8_t* d_flip, void* d_out, int32_t* d_status, void* hip_stream);

/* Asynchronous host path with double-buffered pinned staging (downloader /
 * host cache -> pinned staging -> H2D -> decode, overlapped; config 5).  Up to SDSJ_SLOTS batches are
 * in flight.  A submit stages its batch into the slot's pinned buffer -- while the GPU still decodes
 * the previous batch --, copies it H2D on an engine-owned copy stream and enqueues the decode on
 * `hip_stream` behind that copy, then returns.  sdsj_wait_batch blocks until the slot's batch is done
 * and fills its per-sample status.  `out` (device, as in sdsj_decode_resize_batch) must stay untouched
 * until then.  n <= the engine's max_batch.  Submitting to a slot still in flight waits for it first
 * (its statuses are then dropped).
 *   sdsj_submit_batch : encoded bytes in host memory, borrowed for the call only
 *                       (same samples as sdsj_decode_resize_batch)
 *   sdsj_submit_files : n file paths read straight into the slot's pinned buffer -- what
 *                       LoadFromDiskTransform (presets.py:613-626) does with the local cache that
 *                       run_downloading_task (downloader.py:117-131) fills.  A file that cannot be
 *                       read is reported per sample as SDSJ_EINVAL. */
#define SDSJ_SLOTS 2
int sdsj_submit_batch(sdsj_engine* eng, int slot, int n, const uint8_t* const* jpg, const size_t* len,
                      const sdsj_op* op, const uint8_t* flip, void* out, void* hip_stream);
int sdsj_submit_files(sdsj_engine* eng, int slot, int n, const char* const* paths, const sdsj_op* op,
                      const uint8_t* flip, void* out, void* hip_stream);
int sdsj_wait_batch(sdsj_engine* eng, int slot, int32_t* status);

/* Crop + resize (+flip, +normalise) of n raw RGB frames already in DEVICE memory -- the video path
 * (sds/transforms/presets.py:121-135 ResizeVideoTransform + ConvertVideoToByteTensorTransform ->
 * functional.py:42-86 lean_resize_frames on the frames PyAV decoded).  Frame i is uint8 HWC
 * [height][width][3] at d_frames + i * frame_stride (frame_stride >= width * height * 3).  Same
 * op, flip, output and status conventions as sdsj_decode_resize_batch_device.  Synchronises
 * `hip_stream` between chunks of max_batch frames (host-planned descriptors are staged). */
int sdsj_resize_frames_device(sdsj_engine* eng, int n, const uint8_t* d_frames, int32_t width, int32_t height,
                              int64_t frame_stride, const sdsj_op* op, const uint8_t* d_flip, void* d_out,
                              int32_t* d_status, void* hip_stream);

/* Per-process counters (SURVEY.md §5 metrics; sds itself only logs through loguru, sds/__init__.py:5-17).
 * Accumulated on the device by every batch an engine decodes, over all entry points: samples by
 * status, encoded bytes in, output bytes out.  sdsj_engine_counters waits for the work queued so far
 * and copies up to `cap` counters (index = SDSJ_CTR_*); `reset` != 0 zeroes them afterwards. */
#define SDSJ_CTR_IMAGES 0      /* JPEG samples submitted */
#define SDSJ_CTR_OK 1          /* samples (images or frames) decoded / resized */
#define SDSJ_CTR_UNSUPPORTED 2 /* valid images this path does not decode (PNG, WebP, arithmetic, 12-bit, CMYK...) */
#define SDSJ_CTR_CORRUPT 3     /* malformed / truncated streams */
#define SDSJ_CTR_CAPACITY 4    /* samples that did not fit the scratch */
#define SDSJ_CTR_OTHER 5       /* other per-sample errors (unreadable files) */
#define SDSJ_CTR_BYTES_IN 6    /* encoded bytes of the JPEG samples */
#define SDSJ_CTR_BYTES_OUT 7   /* output tensor bytes written (failed samples included: zeros) */
#define SDSJ_CTR_FRAMES 8      /* raw frames resized (sdsj_resize_frames_device) */
#define SDSJ_CTR_PROGRESSIVE 9 /* progressive JPEGs decoded */
#define SDSJ_NUM_COUNTERS 10
int sdsj_engine_counters(sdsj_engine* eng, uint64_t* out, int cap, int reset);
const char* sdsj_counter_name(int k);

/* Kernel lanes: a batch of >= 256 x L images runs as L contiguous lanes on L streams whose kernel
 * sequences overlap (default 4, at most 4).  1 = one dispatch of every kernel per batch, the setting
 * under which a kernel's launch duration is measured alone (bench.py roofline). */
int sdsj_engine_set_lanes(sdsj_engine* eng, int lanes);

/* Grows the engine's device scratch to at least `bytes` (waits for the device first).  The device-resident
 * entry point never grows scratch by itself (it does not synchronise): its capacity is the engine's
 * cfg->scratch_bytes, or 2 GiB at the first call; samples beyond it report SDSJ_ECAPACITY. */
int sdsj_engine_reserve(sdsj_engine* eng, int64_t bytes);

/* Stage timing: sdsj_engine_set_timing(e, 1) starts (and restarts) accumulation; every chunk launched
 * afterwards records HIP events around each kernel on the caller's stream.  sdsj_engine_stage_times
 * waits for the last recorded chunk and returns, per stage, the summed device milliseconds. */
int sdsj_engine_set_timing(sdsj_engine* eng, int enable);
int sdsj_engine_stage_times(const sdsj_engine* eng, float* ms, int cap, int* n_stages);

const char* sdsj_last_error(const sdsj_engine* eng);

/* Node-local decode service (SURVEY.md §8(f) f1 for the reference's own loader shape: sds runs the
 * transform list per sample inside forked DataLoader workers, sds/dataset.py:535-561, with
 * DataLoader(num_workers=2, pin_memory=True), examples/iter_image_dataset.py:72-80 /
 * sds/dataloader.py:191-193 -- workers that cannot initialise HIP after their parent did).  One
 * process per GPU owns `engines` engines (each its own stream and scratch, one batch in flight each);
 * the per-sample transform in every worker sends its encoded bytes through a shared-memory region and
 * a SOCK_SEQPACKET request, and the service coalesces the requests of all workers into batched engine
 * calls and writes host outputs (the reference's tensor type) back into the worker's region.
 *
 * Wire protocol (little-endian, fixed-size packets on an AF_UNIX SOCK_SEQPACKET connection):
 *   client -> service  sdsj_svc_req.  kind MAP carries the client's region (memfd) as SCM_RIGHTS, in_len =
 *                      its size; the service maps it and replies.  kind DECODE: the JPEG is region[0,
 *                      in_len), the output (op->out_h * out_w * 3 elements of op->out_dtype, op->layout) is
 *                      written to region[out_off, ...).  kind FRAME: region[0, in_len) is a uint8 HWC RGB
 *                      frame of width x height (a sample decoded by PIL), cropped / resized as DECODE does.
 *   service -> client  sdsj_svc_rep {seq, status}: status = the sample's SDSJ_* code (the output is in the
 *                      region when SDSJ_OK). */
#define SDSJ_SVC_MAGIC 0x4A534453u /* "SDSJ" */
#define SDSJ_SVC_MAP 1
#define SDSJ_SVC_DECODE 2
#define SDSJ_SVC_FRAME 3
typedef struct sdsj_svc_req {
    uint32_t magic, kind;
    uint64_t seq;
    int64_t in_len, out_off;
    int32_t width, height; /* FRAME only */
    sdsj_op op;
    int32_t flip;
    int32_t reserved;
} sdsj_svc_req; /* 72 bytes */
typedef struct sdsj_svc_rep {
    uint64_t seq;
    int32_t status, reserved;
} sdsj_svc_rep; /* 16 bytes */

typedef struct sdsj_service_cfg {
    int32_t abi_version; /* SDSJ_ABI_VERSION */
    int32_t device;      /* HIP device */
    int32_t engines;     /* batches in flight at once (0 = 8) */
    int32_t max_batch;   /* requests per batch (0 = 64) */
    int32_t listen_fd;   /* a bound, listening AF_UNIX SOCK_SEQPACKET socket */
    int32_t parent_pid;  /* the service returns when this process is gone (0 = never) */
} sdsj_service_cfg;

/* Serves requests until SIGTERM / SIGINT or the parent's exit; returns SDSJ_OK, or an error code with a
 * message on stderr.  Runs in the calling thread (the service process's main thread). */
int sdsj_service_serve(const sdsj_service_cfg* cfg);

/* Diagnostics for tests: device pointers of the engine's scratch and per-image descriptor array of the
 * most recent chunk, and the byte size of one descriptor (layout: sds_amd/csrc/sdsj_common.h ImgDesc). */
int sdsj_engine_debug_buffers(const sdsj_engine* eng, void** scratch, void** descs, int64_t* desc_bytes,
                              int64_t* scratch_bytes);

/* Name of stage k of sdsj_engine_stage_times ("parse", "unstuff", "entropy", ...). */
const char* sdsj_stage_name(int k);

#ifdef __cplusplus
}
#endif
#endif /* SDSJ_H */
