// sdsj_service.hip -- the node-local decode service (include/sdsj.h sdsj_service_serve).
//
// sds applies its transform list per sample inside forked DataLoader workers (sds/dataset.py:535-561;
// examples/iter_image_dataset.py:72-80 with num_workers=2, pin_memory=True), each worker holding one
// sample at a time.  A worker forked after its parent initialised HIP cannot use the GPU itself, and one
// image per engine call cannot fill the chip.  This service is the one process per GPU that decodes for
// all of them: the worker-side transform (sds_amd/service.py) puts the encoded bytes into its shared
// region and sends a request; the loop here gathers the requests of every worker into batches, runs up
// to `engines` batches at once (one engine, stream and scratch each; a batch is whatever arrived while
// the previous ones ran), and copies each output into its worker's region before replying.
//
// One thread: epoll over the listening socket and the clients, completion by polling the engines'
// events (a finished batch is answered at once; an idle loop blocks in epoll).
#include <hip/hip_runtime.h>

#include <errno.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <deque>
#include <map>
#include <memory>
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

struct Client {
  int fd = -1;
  uint8_t* base = nullptr;  // the worker's region (MAP_SHARED memfd)
  size_t size = 0;
  int inflight = 0;  // requests queued or in a batch (the region stays mapped until they are done)
  bool closed = false;
};

struct Req {
  std::shared_ptr<Client> c;
  sdsj_svc_req r;
};

struct Lane {  // one engine, its stream, and the batch it runs
  sdsj_engine* e = nullptr;
  hipStream_t s = nullptr;
  hipEvent_t done = nullptr;
  uint8_t* d_out = nullptr;
  uint8_t* h_out = nullptr;  // pinned
  size_t out_cap = 0;
  std::vector<Req> batch;
  std::vector<int32_t> status;
  int64_t ob = 0;
  bool busy = false;
};

void log_err(const char* what, const char* detail) { fprintf(stderr, "sdsj_service: %s: %s\n", what, detail); }

void reply(Client& c, uint64_t seq, int status) {
  if (c.closed) return;
  sdsj_svc_rep rep{seq, status, 0};
  for (;;) {
    const ssize_t w = send(c.fd, &rep, sizeof(rep), MSG_NOSIGNAL);
    if (w == (ssize_t)sizeof(rep)) return;
    if (w < 0 && errno == EINTR) continue;
    c.closed = true;  // the worker went away: its later requests are dropped
    return;
  }
}

bool region_ok(const Client& c, int64_t off, int64_t len) {
  return c.base && off >= 0 && len >= 0 && (uint64_t)off + (uint64_t)len <= c.size;
}

class Service {
 public:
  explicit Service(const sdsj_service_cfg& cfg) : cfg_(cfg) {}

  int run() {
    if (hipSetDevice(cfg_.device) != hipSuccess) return fail("hipSetDevice", SDSJ_EHIP);
    const int nl = cfg_.engines > 0 ? cfg_.engines : 4;
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
    int rc = SDSJ_OK;
    while (!g_stop) {
      if (cfg_.parent_pid > 0 && getppid() != cfg_.parent_pid) break;
      const bool busy = std::any_of(lanes_.begin(), lanes_.end(), [](const Lane& l) { return l.busy; });
      epoll_event evs[64];
      const int n = epoll_wait(ep_, evs, 64, busy || !pending_.empty() ? 0 : 500);
      if (n < 0 && errno != EINTR) {
        rc = fail("epoll_wait", SDSJ_EINVAL);
        break;
      }
      for (int i = 0; i < n; i++) {
        if (evs[i].data.fd == cfg_.listen_fd) accept_clients();
        else read_client(evs[i].data.fd);
      }
      for (auto& l : lanes_)
        if (l.busy && hipEventQuery(l.done) == hipSuccess) complete(l);
      for (auto& l : lanes_) {
        if (pending_.empty()) break;
        if (!l.busy && (rc = submit(l)) != SDSJ_OK) break;
      }
      if (rc != SDSJ_OK) break;
      if (busy && n == 0) sched_yield();
    }
    for (auto& l : lanes_) {  // drain before the engines go
      if (l.busy) {
        (void)hipEventSynchronize(l.done);
        complete(l);
      }
    }
    shutdown();
    return rc;
  }

 private:
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
      l = Lane();
    }
    (void)hipFree(fr_in_), (void)hipFree(fr_out_), (void)hipFree(fr_small_);
    fr_in_ = fr_out_ = fr_small_ = nullptr;
    if (ep_ >= 0) close(ep_);
    ep_ = -1;
  }

  void drop(Client& c) {
    if (c.fd >= 0) {
      (void)epoll_ctl(ep_, EPOLL_CTL_DEL, c.fd, nullptr);
      close(c.fd);
    }
    c.fd = -1;
    c.closed = true;
    if (c.inflight == 0 && c.base) {
      munmap(c.base, c.size);
      c.base = nullptr;
    }
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
      if (got < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return;
      if (got < 0 && errno == EINTR) continue;
      int passed = -1;
      for (cmsghdr* cm = CMSG_FIRSTHDR(&mh); cm; cm = CMSG_NXTHDR(&mh, cm))
        if (cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_RIGHTS) memcpy(&passed, CMSG_DATA(cm), sizeof(int));
      if (got != (ssize_t)sizeof(r) || r.magic != SDSJ_SVC_MAGIC) {  // closed, or not our protocol
        if (passed >= 0) close(passed);
        clients_.erase(fd);
        drop(*c);
        return;
      }
      if (r.kind == SDSJ_SVC_MAP) {
        int st = SDSJ_EINVAL;
        if (passed >= 0 && r.in_len > 0 && c->inflight == 0) {
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
        reply(*c, r.seq, st);
      } else if (r.kind == SDSJ_SVC_DECODE) {
        if (!region_ok(*c, 0, r.in_len) || !region_ok(*c, r.out_off, out_bytes(r.op)) || r.op.out_h <= 0 || r.op.out_w <= 0) {
          reply(*c, r.seq, SDSJ_EINVAL);
          continue;
        }
        c->inflight++;
        pending_.push_back(Req{c, r});
      } else if (r.kind == SDSJ_SVC_FRAME) {
        reply(*c, r.seq, frame(*c, r));
      } else {
        reply(*c, r.seq, SDSJ_EINVAL);
      }
    }
  }

  // One batch from the oldest pending request's op: every pending request with that op, up to max_batch.
  int submit(Lane& l) {
    const sdsj_op op = pending_.front().r.op;
    l.batch.clear();
    for (auto it = pending_.begin(); it != pending_.end() && (int)l.batch.size() < max_batch_;) {
      if (same_op(it->r.op, op)) {
        l.batch.push_back(*it);
        it = pending_.erase(it);
      } else {
        ++it;
      }
    }
    const int n = (int)l.batch.size();
    l.ob = out_bytes(op);
    const size_t need = (size_t)l.ob * n;
    if (need > l.out_cap) {
      (void)hipFree(l.d_out);
      (void)hipHostFree(l.h_out);
      l.d_out = l.h_out = nullptr;
      l.out_cap = 0;
      const size_t cap = std::max(need, (size_t)l.ob * max_batch_ / 4);
      if (hipMalloc(&l.d_out, cap) != hipSuccess || hipHostMalloc(&l.h_out, cap) != hipSuccess) {
        finish_failed(l, SDSJ_ENOMEM);
        return SDSJ_OK;
      }
      l.out_cap = cap;
    }
    std::vector<const uint8_t*> ptrs(n);
    std::vector<size_t> lens(n);
    std::vector<uint8_t> flips(n);
    for (int i = 0; i < n; i++) {
      ptrs[i] = l.batch[i].c->base;
      lens[i] = (size_t)l.batch[i].r.in_len;
      flips[i] = l.batch[i].r.flip ? 1 : 0;
    }
    int rc = sdsj_submit_batch(l.e, 0, n, ptrs.data(), lens.data(), &op, flips.data(), l.d_out, l.s);
    if (rc == SDSJ_OK && hipMemcpyAsync(l.h_out, l.d_out, need, hipMemcpyDeviceToHost, l.s) != hipSuccess) rc = SDSJ_EHIP;
    if (rc == SDSJ_OK && hipEventRecord(l.done, l.s) != hipSuccess) rc = SDSJ_EHIP;
    if (rc != SDSJ_OK) {
      log_err("submit", sdsj_last_error(l.e));
      (void)hipStreamSynchronize(l.s);
      finish_failed(l, rc);
      return SDSJ_OK;
    }
    l.busy = true;
    return SDSJ_OK;
  }

  void finish_failed(Lane& l, int status) {
    for (auto& q : l.batch) {
      reply(*q.c, q.r.seq, status);
      release(q.c);
    }
    l.batch.clear();
  }

  void release(const std::shared_ptr<Client>& c) {
    if (--c->inflight == 0 && c->closed && c->base) {
      munmap(c->base, c->size);
      c->base = nullptr;
    }
  }

  void complete(Lane& l) {
    l.busy = false;
    const int n = (int)l.batch.size();
    if (sdsj_wait_batch(l.e, 0, l.status.data()) != SDSJ_OK)
      std::fill(l.status.begin(), l.status.begin() + n, SDSJ_EHIP);
    for (int i = 0; i < n; i++) {
      Req& q = l.batch[i];
      if (!q.c->closed && l.status[i] == SDSJ_OK) memcpy(q.c->base + q.r.out_off, l.h_out + (size_t)i * l.ob, l.ob);
      reply(*q.c, q.r.seq, l.status[i]);
      release(q.c);
    }
    l.batch.clear();
  }

  // A frame PIL decoded in the worker (samples the JPEG kernels do not take): H2D, the frame path's
  // crop / resize (sdsj_resize_frames_device), D2H -- synchronous on the first lane's engine once it is
  // idle (rare: other formats and damaged streams).
  int frame(Client& c, const sdsj_svc_req& r) {
    const int64_t fb = (int64_t)r.width * r.height * 3;
    if (r.width <= 0 || r.height <= 0 || r.in_len < fb || !region_ok(c, 0, fb) || !region_ok(c, r.out_off, out_bytes(r.op)))
      return SDSJ_EINVAL;
    Lane& l = lanes_[0];
    if (l.busy) {
      (void)hipEventSynchronize(l.done);
      complete(l);
    }
    const int64_t ob = out_bytes(r.op);
    if ((size_t)fb > fr_in_cap_ || (size_t)ob > fr_out_cap_ || !fr_small_) {
      (void)hipFree(fr_in_), (void)hipFree(fr_out_), (void)hipFree(fr_small_);
      fr_in_ = fr_out_ = fr_small_ = nullptr;
      fr_in_cap_ = fr_out_cap_ = 0;
      if (hipMalloc(&fr_in_, fb) != hipSuccess || hipMalloc(&fr_out_, ob) != hipSuccess || hipMalloc(&fr_small_, 16) != hipSuccess)
        return SDSJ_ENOMEM;
      fr_in_cap_ = (size_t)fb;
      fr_out_cap_ = (size_t)ob;
    }
    // fr_small_: [0, 4) the frame's status, [4] its flip flag
    uint8_t small[8] = {0, 0, 0, 0, (uint8_t)(r.flip ? 1 : 0), 0, 0, 0};
    if (hipMemcpyAsync(fr_in_, c.base, fb, hipMemcpyHostToDevice, l.s) != hipSuccess ||
        hipMemcpyAsync(fr_small_, small, sizeof(small), hipMemcpyHostToDevice, l.s) != hipSuccess ||
        hipStreamSynchronize(l.s) != hipSuccess)
      return SDSJ_EHIP;
    int st = sdsj_resize_frames_device(l.e, 1, fr_in_, r.width, r.height, fb, &r.op, fr_small_ + 4, fr_out_,
                                       reinterpret_cast<int32_t*>(fr_small_), l.s);
    if (st != SDSJ_OK) return st;
    if (hipMemcpyAsync(small, fr_small_, sizeof(small), hipMemcpyDeviceToHost, l.s) != hipSuccess ||
        hipMemcpyAsync(c.base + r.out_off, fr_out_, ob, hipMemcpyDeviceToHost, l.s) != hipSuccess ||
        hipStreamSynchronize(l.s) != hipSuccess)
      return SDSJ_EHIP;
    int32_t fst;
    memcpy(&fst, small, sizeof(fst));
    return fst;
  }

  sdsj_service_cfg cfg_;
  int max_batch_ = 64;
  int ep_ = -1;
  std::vector<Lane> lanes_;
  std::map<int, std::shared_ptr<Client>> clients_;
  std::deque<Req> pending_;
  uint8_t *fr_in_ = nullptr, *fr_out_ = nullptr, *fr_small_ = nullptr;  // frame path buffers (grow only)
  size_t fr_in_cap_ = 0, fr_out_cap_ = 0;
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
