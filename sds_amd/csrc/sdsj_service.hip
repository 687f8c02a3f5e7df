// sdsj_service.hip -- the node-local decode service (include/sdsj.h sdsj_service_serve).
//
// sds applies its transform list per sample inside forked DataLoader workers (sds/dataset.py:535-561;
// examples/iter_image_dataset.py:72-80 with num_workers=2, pin_memory=True), each worker holding one
// sample at a time.  A worker forked after its parent initialised HIP cannot use the GPU itself, and one
// image per engine call cannot fill the chip.  This service is the one process per GPU that decodes for
// all of them: the worker-side transform (sds_amd/service.py) puts the encoded bytes into its shared
// region and sends a request; the service gathers the requests of every worker into batches, runs up to
// `engines` batches at once (one engine, stream and scratch each; a batch is whatever arrived while the
// previous ones ran), and copies each output into its worker's region before replying.
//
// Threads: the caller's thread reads requests (epoll over the listening socket and the clients) into
// one queue; one thread per engine takes a batch from it, runs it on the engine's one stream (host
// planning and H2D, kernels, status, then the D2H of the outputs) and answers its requests.  One stream
// per engine matters: with the pipelined host path's second (copy) stream per engine, 8 streams shared
// HIP's 4 hardware queues and the engines' batches ran one after another (16 clients: 3.8k images/s,
// 10.0k with one stream each; profiles/r04_service.txt).  A single thread polling every engine's event
// measured no overlap either.
#include <hip/hip_runtime.h>

#include <errno.h>
#include <poll.h>
#include <pthread.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "sdsj.h"

namespace {

static_assert(sizeof(sdsj_svc_req) == 72, "wire format");
static_assert(sizeof(sdsj_svc_rep) == 16, "wire format");

volatile sig_atomic_t g_stop = 0;
void on_signal(int) { g_stop = 1; }

int64_t out_bytes(const sdsj_op& op) {
  return (int64_t)op.out_h * op.out_w * 3 * (op.out_dtype == SDSJ_DTYPE_F32 ? 4 : 1);
}

bool same_op(const sdsj_op& a, const sdsj_op& b) { return memcmp(&a, &b, sizeof(sdsj_op)) == 0; }

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void log_err(const char* what, const char* detail) { fprintf(stderr, "sdsj_service: %s: %s\n", what, detail); }

// A worker's connection and its shared region.  The region stays mapped while requests of the client
// are queued or in a batch (inflight), even after the client went away (closed).
struct Client {
  int fd = -1;
  uint8_t* base = nullptr;  // MAP_SHARED memfd
  size_t size = 0;
  std::atomic<int> inflight{0};
  std::atomic<bool> closed{false};
  std::mutex mu;  // base / size / unmap

  // max_wait_ms bounds the wait for a full socket buffer: a client that stops reading its replies while
  // still connected is dropped (closed) after that long in total instead of blocking the caller -- an
  // engine thread (kReplyWaitMs), or the epoll thread that serves every client (kEpollReplyWaitMs).
  static constexpr int kReplyWaitMs = 10000, kEpollReplyWaitMs = 20;
  void reply(uint64_t seq, int status, int max_wait_ms = kReplyWaitMs) {
    if (closed.load()) return;
    sdsj_svc_rep rep{seq, status, 0};
    const double deadline = now_us() + 1e3 * max_wait_ms;
    for (;;) {  // (SOCK_SEQPACKET: a packet is sent whole; concurrent senders do not interleave)
      const ssize_t w = send(fd, &rep, sizeof(rep), MSG_NOSIGNAL);
      if (w == (ssize_t)sizeof(rep)) return;
      if (w < 0 && errno == EINTR) continue;
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {  // socket buffer full: wait until writable
        const int left_ms = (int)((deadline - now_us()) / 1e3);
        pollfd p{fd, POLLOUT, 0};
        if (left_ms > 0 && poll(&p, 1, std::min(left_ms, 1000)) >= 0 && !(p.revents & (POLLERR | POLLHUP | POLLNVAL)))
          continue;
      }
      closed.store(true);  // the worker went away (EPIPE, ECONNRESET, ...) or stopped reading: later requests are dropped
      return;
    }
  }
  bool region_ok(int64_t off, int64_t len) const {
    return base && off >= 0 && len >= 0 && (uint64_t)off + (uint64_t)len <= size;
  }
  // The last reference of a client that went away unmaps its region and closes its socket (not
  // earlier: a lane thread may still reply on it, and a closed descriptor number can be reused).
  void finalize_locked() {
    if (!closed.load() || inflight.load() != 0) return;
    if (base) munmap(base, size);
    base = nullptr;
    if (fd >= 0) close(fd);
    fd = -1;
  }
  void release() {
    if (--inflight == 0 && closed.load()) {
      std::lock_guard<std::mutex> g(mu);
      finalize_locked();
    }
  }
};

struct Req {
  std::shared_ptr<Client> c;
  sdsj_svc_req r;
};

class Service {
 public:
  explicit Service(const sdsj_service_cfg& cfg) : cfg_(cfg) {}

  int run() {
    trace_ = getenv("SDSJ_SERVICE_TRACE") != nullptr;
    // SDSJ_SERVICE_SPIN=1: the engine threads spin in their stream waits (HIP's default policy) instead
    // of sleeping on them; sleeping leaves the waited-on GPU time's CPU to the DataLoader workers
    const char* spin = getenv("SDSJ_SERVICE_SPIN");
    if (!(spin && spin[0] == '1')) (void)hipSetDeviceFlags(hipDeviceScheduleBlockingSync);
    if (hipSetDevice(cfg_.device) != hipSuccess) return fail("hipSetDevice", SDSJ_EHIP);
    const int nl = cfg_.engines > 0 ? cfg_.engines : 8;
    max_batch_ = cfg_.max_batch > 0 ? cfg_.max_batch : 64;
    lanes_.resize(nl);
    for (auto& l : lanes_) {
      sdsj_cfg ec{SDSJ_ABI_VERSION, max_batch_, 0};
      if (sdsj_engine_create(cfg_.device, &ec, &l.e) != SDSJ_OK) return fail("sdsj_engine_create", SDSJ_EHIP);
      if (hipStreamCreateWithFlags(&l.s, hipStreamNonBlocking) != hipSuccess) return fail("stream", SDSJ_EHIP);
      if (hipEventCreateWithFlags(&l.done, hipEventDisableTiming) != hipSuccess) return fail("event", SDSJ_EHIP);
      l.status.resize(max_batch_);
    }
    ep_ = epoll_create1(EPOLL_CLOEXEC);
    if (ep_ < 0) return fail("epoll_create1", SDSJ_EINVAL);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = cfg_.listen_fd;
    if (epoll_ctl(ep_, EPOLL_CTL_ADD, cfg_.listen_fd, &ev) != 0) return fail("epoll_ctl(listen)", SDSJ_EINVAL);
    // engine threads with SIGTERM / SIGINT blocked: the signals reach this thread's epoll_wait
    sigset_t block, old;
    sigemptyset(&block);
    sigaddset(&block, SIGTERM);
    sigaddset(&block, SIGINT);
    pthread_sigmask(SIG_BLOCK, &block, &old);
    for (int k = 0; k < nl; k++) threads_.emplace_back([this, k] { lane_loop(lanes_[k]); });
    pthread_sigmask(SIG_SETMASK, &old, nullptr);
    int rc = SDSJ_OK;
    while (!g_stop) {
      if (cfg_.parent_pid > 0 && getppid() != cfg_.parent_pid) break;
      epoll_event evs[64];
      const int n = epoll_wait(ep_, evs, 64, 500);
      if (n < 0 && errno != EINTR) {
        rc = SDSJ_EINVAL;
        log_err("epoll_wait", strerror(errno));
        break;
      }
      for (int i = 0; i < n; i++) {
        if (evs[i].data.fd == cfg_.listen_fd) accept_clients();
        else read_client(evs[i].data.fd);
      }
    }
    {
      std::lock_guard<std::mutex> g(qmu_);
      stopping_ = true;
    }
    qcv_.notify_all();
    for (auto& t : threads_) t.join();  // each finishes (and answers) the batch it holds
    shutdown();
    return rc;
  }

 private:
  struct Lane {  // one engine, its stream, and the batch it runs
    sdsj_engine* e = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t done = nullptr;
    uint8_t* d_out = nullptr;
    uint8_t* h_out = nullptr;  // pinned
    size_t out_cap = 0;
    std::vector<Req> batch;
    std::vector<int32_t> status;
    // frame path buffers (grow only)
    uint8_t *fr_in = nullptr, *fr_out = nullptr, *fr_small = nullptr;
    size_t fr_in_cap = 0, fr_out_cap = 0;
  };

  int fail(const char* what, int code) {
    log_err(what, strerror(errno));
    shutdown();
    return code;
  }

  void shutdown() {
    for (auto& kv : clients_) drop(*kv.second);
    clients_.clear();
    for (auto& l : lanes_) {
      if (l.e) sdsj_engine_destroy(l.e);
      if (l.s) (void)hipStreamDestroy(l.s);
      if (l.done) (void)hipEventDestroy(l.done);
      (void)hipFree(l.d_out);
      (void)hipHostFree(l.h_out);
      (void)hipFree(l.fr_in), (void)hipFree(l.fr_out), (void)hipFree(l.fr_small);
      l = Lane();
    }
    if (ep_ >= 0) close(ep_);
    ep_ = -1;
  }

  void drop(Client& c) {
    std::lock_guard<std::mutex> g(c.mu);
    if (c.fd >= 0) (void)epoll_ctl(ep_, EPOLL_CTL_DEL, c.fd, nullptr);
    c.closed.store(true);
    c.finalize_locked();
  }

  void accept_clients() {
    for (;;) {
      const int fd = accept4(cfg_.listen_fd, nullptr, nullptr, SOCK_CLOEXEC | SOCK_NONBLOCK);
      if (fd < 0) return;
      auto c = std::make_shared<Client>();
      c->fd = fd;
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.fd = fd;
      if (epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev) != 0) {
        close(fd);
        continue;
      }
      clients_[fd] = c;
    }
  }

  void read_client(int fd) {
    auto it = clients_.find(fd);
    if (it == clients_.end()) return;
    std::shared_ptr<Client> c = it->second;
    int queued = 0;
    for (;;) {
      sdsj_svc_req r;
      char cbuf[CMSG_SPACE(sizeof(int))];
      iovec iov{&r, sizeof(r)};
      msghdr mh{};
      mh.msg_iov = &iov;
      mh.msg_iovlen = 1;
      mh.msg_control = cbuf;
      mh.msg_controllen = sizeof(cbuf);
      const ssize_t got = recvmsg(fd, &mh, MSG_CMSG_CLOEXEC);
      if (got < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
      if (got < 0 && errno == EINTR) continue;
      int passed = -1;
      for (cmsghdr* cm = CMSG_FIRSTHDR(&mh); cm; cm = CMSG_NXTHDR(&mh, cm))
        if (cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_RIGHTS) memcpy(&passed, CMSG_DATA(cm), sizeof(int));
      if (got != (ssize_t)sizeof(r) || r.magic != SDSJ_SVC_MAGIC) {  // closed, or not our protocol
        if (passed >= 0) close(passed);
        clients_.erase(fd);
        drop(*c);
        break;
      }
      if (r.kind == SDSJ_SVC_MAP) {
        int st = SDSJ_EINVAL;
        if (passed >= 0 && r.in_len > 0 && c->inflight.load() == 0) {  // (a client maps between requests)
          std::lock_guard<std::mutex> g(c->mu);
          if (c->base) munmap(c->base, c->size);
          c->base = nullptr;
          void* p = mmap(nullptr, (size_t)r.in_len, PROT_READ | PROT_WRITE, MAP_SHARED, passed, 0);
          if (p != MAP_FAILED) {
            c->base = static_cast<uint8_t*>(p);
            c->size = (size_t)r.in_len;
            st = SDSJ_OK;
          }
        }
        if (passed >= 0) close(passed);
        c->reply(r.seq, st, Client::kEpollReplyWaitMs);
      } else if (r.kind == SDSJ_SVC_DECODE || r.kind == SDSJ_SVC_FRAME) {
        const bool frame = r.kind == SDSJ_SVC_FRAME;
        const int64_t in = frame ? (int64_t)r.width * r.height * 3 : r.in_len;
        if (!c->region_ok(0, in) || !c->region_ok(r.out_off, out_bytes(r.op)) || r.op.out_h <= 0 || r.op.out_w <= 0 ||
            (frame && (r.width <= 0 || r.height <= 0 || r.in_len < in))) {
          c->reply(r.seq, SDSJ_EINVAL, Client::kEpollReplyWaitMs);
          continue;
        }
        c->inflight++;
        std::lock_guard<std::mutex> g(qmu_);
        pending_.push_back(Req{c, r});
        queued++;
      } else {
        c->reply(r.seq, SDSJ_EINVAL, Client::kEpollReplyWaitMs);
      }
    }
    // one request wakes one idle engine thread (waking them all cost each request a herd of wake-ups
    // that found the queue drained); several may need several
    if (queued == 1) qcv_.notify_one();
    else if (queued > 1) qcv_.notify_all();
  }

  // Engine thread: the oldest pending request and every pending request with its op (up to max_batch)
  // form a batch; a FRAME request goes alone through the frame path.
  void lane_loop(Lane& l) {
    (void)hipSetDevice(cfg_.device);
    for (;;) {
      bool frame = false;
      {
        std::unique_lock<std::mutex> g(qmu_);
        qcv_.wait(g, [this] { return stopping_ || !pending_.empty(); });
        if (pending_.empty()) return;  // stopping, nothing left
        l.batch.clear();
        if (pending_.front().r.kind == SDSJ_SVC_FRAME) {
          l.batch.push_back(pending_.front());
          pending_.pop_front();
          frame = true;
        } else {
          const sdsj_op op = pending_.front().r.op;
          for (auto it = pending_.begin(); it != pending_.end() && (int)l.batch.size() < max_batch_;) {
            if (it->r.kind == SDSJ_SVC_DECODE && same_op(it->r.op, op)) {
              l.batch.push_back(*it);
              it = pending_.erase(it);
            } else {
              ++it;
            }
          }
        }
      }
      if (frame) {
        Req& q = l.batch[0];
        q.c->reply(q.r.seq, run_frame(l, *q.c, q.r));
        q.c->release();
      } else {
        run_batch(l);
      }
      l.batch.clear();
    }
  }

  void run_batch(Lane& l) {
    const double t0 = trace_ ? now_us() : 0;
    const int n = (int)l.batch.size();
    const sdsj_op op = l.batch[0].r.op;
    const int64_t ob = out_bytes(op);
    const size_t need = (size_t)ob * n;
    int rc = SDSJ_OK;
    if (need > l.out_cap) {
      (void)hipFree(l.d_out);
      (void)hipHostFree(l.h_out);
      l.d_out = l.h_out = nullptr;
      l.out_cap = 0;
      const size_t cap = std::max(need, (size_t)ob * max_batch_ / 4);
      if (hipMalloc(&l.d_out, cap) != hipSuccess || hipHostMalloc(&l.h_out, cap) != hipSuccess) rc = SDSJ_ENOMEM;
      else l.out_cap = cap;
    }
    std::vector<const uint8_t*> ptrs(n);
    std::vector<size_t> lens(n);
    std::vector<uint8_t> flips(n);
    for (int i = 0; i < n; i++) {
      ptrs[i] = l.batch[i].c->base;
      lens[i] = (size_t)l.batch[i].r.in_len;
      flips[i] = l.batch[i].r.flip ? 1 : 0;
    }
    // everything on the lane's one stream (H2D, kernels, status), so the lanes' streams are the only
    // ones the service queues work on: one hardware queue each
    if (rc == SDSJ_OK)
      rc = sdsj_decode_resize_batch(l.e, n, ptrs.data(), lens.data(), &op, flips.data(), l.d_out, l.status.data(), l.s);
    const double t1 = trace_ ? now_us() : 0;
    if (rc == SDSJ_OK && hipMemcpyAsync(l.h_out, l.d_out, need, hipMemcpyDeviceToHost, l.s) != hipSuccess) rc = SDSJ_EHIP;
    if (rc == SDSJ_OK && hipStreamSynchronize(l.s) != hipSuccess) rc = SDSJ_EHIP;
    if (rc != SDSJ_OK) {
      log_err("batch", sdsj_last_error(l.e));
      (void)hipStreamSynchronize(l.s);
      std::fill(l.status.begin(), l.status.begin() + n, rc);
    }
    for (int i = 0; i < n; i++) {
      Req& q = l.batch[i];
      if (!q.c->closed.load() && l.status[i] == SDSJ_OK) memcpy(q.c->base + q.r.out_off, l.h_out + (size_t)i * ob, ob);
      q.c->reply(q.r.seq, l.status[i]);
      q.c->release();
    }
    if (trace_)
      fprintf(stderr, "sdsj_service: lane %d n %d submit %.1f us, wait %.1f us\n", (int)(&l - lanes_.data()), n, t1 - t0,
              now_us() - t1);
  }

  // A frame PIL decoded in the worker (samples the JPEG kernels do not take): H2D, the frame path's
  // crop / resize (sdsj_resize_frames_device), D2H -- on this lane's engine.
  int run_frame(Lane& l, Client& c, const sdsj_svc_req& r) {
    const int64_t fb = (int64_t)r.width * r.height * 3;
    const int64_t ob = out_bytes(r.op);
    if ((size_t)fb > l.fr_in_cap || (size_t)ob > l.fr_out_cap || !l.fr_small) {
      (void)hipFree(l.fr_in), (void)hipFree(l.fr_out), (void)hipFree(l.fr_small);
      l.fr_in = l.fr_out = l.fr_small = nullptr;
      l.fr_in_cap = l.fr_out_cap = 0;
      if (hipMalloc(&l.fr_in, fb) != hipSuccess || hipMalloc(&l.fr_out, ob) != hipSuccess || hipMalloc(&l.fr_small, 16) != hipSuccess)
        return SDSJ_ENOMEM;
      l.fr_in_cap = (size_t)fb;
      l.fr_out_cap = (size_t)ob;
    }
    // fr_small: [0, 4) the frame's status, [4] its flip flag
    uint8_t small[8] = {0, 0, 0, 0, (uint8_t)(r.flip ? 1 : 0), 0, 0, 0};
    if (hipMemcpyAsync(l.fr_in, c.base, fb, hipMemcpyHostToDevice, l.s) != hipSuccess ||
        hipMemcpyAsync(l.fr_small, small, sizeof(small), hipMemcpyHostToDevice, l.s) != hipSuccess ||
        hipStreamSynchronize(l.s) != hipSuccess)
      return SDSJ_EHIP;
    int st = sdsj_resize_frames_device(l.e, 1, l.fr_in, r.width, r.height, fb, &r.op, l.fr_small + 4, l.fr_out,
                                       reinterpret_cast<int32_t*>(l.fr_small), l.s);
    if (st != SDSJ_OK) return st;
    if (hipMemcpyAsync(small, l.fr_small, sizeof(small), hipMemcpyDeviceToHost, l.s) != hipSuccess ||
        hipMemcpyAsync(c.base + r.out_off, l.fr_out, ob, hipMemcpyDeviceToHost, l.s) != hipSuccess ||
        hipStreamSynchronize(l.s) != hipSuccess)
      return SDSJ_EHIP;
    int32_t fst;
    memcpy(&fst, small, sizeof(fst));
    return fst;
  }

  sdsj_service_cfg cfg_;
  int max_batch_ = 64;
  bool trace_ = false;
  int ep_ = -1;
  std::vector<Lane> lanes_;
  std::vector<std::thread> threads_;
  std::map<int, std::shared_ptr<Client>> clients_;  // (the epoll thread's)
  std::mutex qmu_;
  std::condition_variable qcv_;
  std::deque<Req> pending_;
  bool stopping_ = false;
};

}  // namespace

extern "C" int sdsj_service_serve(const sdsj_service_cfg* cfg) {
  if (!cfg || cfg->abi_version != SDSJ_ABI_VERSION || cfg->listen_fd < 0) return SDSJ_EINVAL;
  struct sigaction sa {};
  sa.sa_handler = on_signal;
  sigemptyset(&sa.sa_mask);
  (void)sigaction(SIGTERM, &sa, nullptr);
  (void)sigaction(SIGINT, &sa, nullptr);
  g_stop = 0;
  Service svc(*cfg);
  return svc.run();
}
