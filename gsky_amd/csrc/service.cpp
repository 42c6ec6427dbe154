// service.cpp -- per-node GPU warp service: client side (forwarding from
// warp_operation_fast) and the daemon loop (gskyhip_service_run, gskyhipd).
// See service.h for the design.
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/uio.h>
#include <sys/un.h>
#include <unistd.h>

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <new>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gskyhip.h"
#include "gsky_device.h"
#include "service.h"

namespace gsky {
namespace {

// ---------------------------------------------------------------- framing
struct Out {
  std::vector<char> b;
  template <typename T> void put(const T &v) {
    const char *p = (const char *)&v;
    b.insert(b.end(), p, p + sizeof(T));
  }
  void put_bytes(const void *p, size_t n) {
    put<uint64_t>(n);
    b.insert(b.end(), (const char *)p, (const char *)p + n);
  }
  void put_str(const std::string &s) { put_bytes(s.data(), s.size()); }
};

struct In {
  const char *p, *e;
  bool ok = true;
  template <typename T> T get() {
    T v{};
    if (e - p < (ptrdiff_t)sizeof(T)) { ok = false; return v; }
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string get_str() {
    const uint64_t n = get<uint64_t>();
    if (!ok || (uint64_t)(e - p) < n) { ok = false; return std::string(); }
    std::string s(p, p + n);
    p += n;
    return s;
  }
  const char *get_bytes(uint64_t &n) {
    n = get<uint64_t>();
    if (!ok || (uint64_t)(e - p) < n) { ok = false; return nullptr; }
    const char *q = p;
    p += n;
    return q;
  }
};

bool write_all(int fd, const void *buf, size_t n) {
  const char *p = (const char *)buf;
  while (n > 0) {
    const ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);   // a dead peer must not SIGPIPE the daemon
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

// sendmsg over an iovec list until every byte is out (no copy into one buffer)
bool write_allv(int fd, iovec *iov, int cnt) {
  while (cnt > 0) {
    msghdr m;
    std::memset(&m, 0, sizeof(m));
    m.msg_iov = iov;
    m.msg_iovlen = (size_t)cnt;
    ssize_t k = ::sendmsg(fd, &m, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    while (cnt > 0 && (size_t)k >= iov->iov_len) { k -= (ssize_t)iov->iov_len; iov++; cnt--; }
    if (cnt > 0) { iov->iov_base = (char *)iov->iov_base + k; iov->iov_len -= (size_t)k; }
  }
  return true;
}

bool read_all(int fd, void *buf, size_t n) {
  char *p = (char *)buf;
  while (n > 0) {
    const ssize_t k = ::recv(fd, p, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

bool send_msg(int fd, uint32_t op, const std::vector<char> &payload) {
  char hdr[16];
  const uint64_t n = payload.size();
  std::memcpy(hdr, &kSvcMagic, 4);
  std::memcpy(hdr + 4, &op, 4);
  std::memcpy(hdr + 8, &n, 8);
  return write_all(fd, hdr, 16) && (n == 0 || write_all(fd, payload.data(), n));
}

// Largest payload a message of `op` may carry: a registration holds granule
// data (up to 64 GiB), a warp request a few strings and numbers, the rest
// nothing -- so one bad header cannot make the daemon allocate gigabytes.
uint64_t max_payload(uint32_t op) {
  switch (op) {
    case SVC_REGISTER: return 1ull << 36;
    case SVC_WARP: case SVC_WARP_SHM: return 1ull << 20;
    default: return 64;
  }
}

bool recv_msg(int fd, uint32_t &op, std::vector<char> &payload, bool reply = false) {
  char hdr[16];
  if (!read_all(fd, hdr, 16)) return false;
  uint32_t magic;
  uint64_t n;
  std::memcpy(&magic, hdr, 4);
  std::memcpy(&op, hdr + 4, 4);
  std::memcpy(&n, hdr + 8, 8);
  if (magic != kSvcMagic || n > (reply ? (1ull << 36) : max_payload(op))) return false;
  try {
    payload.resize(n);
  } catch (const std::bad_alloc &) {
    return false;
  }
  return n == 0 || read_all(fd, payload.data(), n);
}

int connect_to(const char *sock) {
  const int fd = ::socket(AF_UNIX, SOCK_STREAM, 0);
  if (fd < 0) return -1;
  sockaddr_un a;
  std::memset(&a, 0, sizeof(a));
  a.sun_family = AF_UNIX;
  std::strncpy(a.sun_path, sock, sizeof(a.sun_path) - 1);
  if (::connect(fd, (sockaddr *)&a, sizeof(a)) != 0) {
    ::close(fd);
    return -1;
  }
  return fd;
}

// one request / reply exchange on a fresh connection
bool exchange(const char *sock, uint32_t op, const std::vector<char> &req, std::vector<char> &rep) {
  const int fd = connect_to(sock);
  if (fd < 0) return false;
  uint32_t rop = 0;
  const bool ok = send_msg(fd, op, req) && recv_msg(fd, rop, rep, true) && rop == op;
  ::close(fd);
  return ok;
}

void put_req(Out &o, const WarpReq &q) {
  o.put_str(q.path);
  o.put(q.band);
  o.put(q.has_src_srs); o.put(q.has_src_gt); o.put(q.geoloc); o.put(q.has_dst_srs);
  o.put_str(q.src_srs);
  o.put_str(q.dst_srs);
  for (double v : q.src_gt) o.put(v);
  for (double v : q.dst_gt) o.put(v);
  o.put(q.width); o.put(q.height); o.put(q.srs_cf);
  o.put((int32_t)q.geoloc_opts.size());
  for (const std::string &g : q.geoloc_opts) o.put_str(g);
}

bool get_req(In &in, WarpReq &q) {
  q.path = in.get_str();
  q.band = in.get<int32_t>();
  q.has_src_srs = in.get<int32_t>(); q.has_src_gt = in.get<int32_t>();
  q.geoloc = in.get<int32_t>(); q.has_dst_srs = in.get<int32_t>();
  q.src_srs = in.get_str();
  q.dst_srs = in.get_str();
  for (double &v : q.src_gt) v = in.get<double>();
  for (double &v : q.dst_gt) v = in.get<double>();
  q.width = in.get<int32_t>(); q.height = in.get<int32_t>(); q.srs_cf = in.get<int32_t>();
  const int32_t ng = in.get<int32_t>();
  if (ng < 0 || ng > 64) return false;
  for (int32_t k = 0; k < ng && in.ok; k++) q.geoloc_opts.push_back(in.get_str());
  return in.ok;
}

// A warp reply: the fixed fields, the window length, then the window bytes --
// sent with one sendmsg from the batch's result (no copy into a message
// buffer) and received straight into the caller's memory.
constexpr size_t kRespFixed = 4 + 16 + 8 + 4 + 4 + 48 + 8;

void put_resp_fixed(Out &o, const WarpResp &r, uint64_t n_data) {
  o.put(r.rc);
  for (int32_t v : r.bbox) o.put(v);
  o.put(r.nodata); o.put(r.dtype); o.put(r.bytes_read);
  for (double v : r.src_gt) o.put(v);
  o.put<uint64_t>(n_data);
}

bool send_resp(int fd, const WarpResp &r) {
  Out o;
  put_resp_fixed(o, r, r.data.size());
  char hdr[16];
  const uint32_t op = SVC_WARP;
  const uint64_t n = o.b.size() + r.data.size();
  std::memcpy(hdr, &kSvcMagic, 4);
  std::memcpy(hdr + 4, &op, 4);
  std::memcpy(hdr + 8, &n, 8);
  iovec iov[3] = {{hdr, 16}, {o.b.data(), o.b.size()}, {(void *)r.data.data(), r.data.size()}};
  return write_allv(fd, iov, r.data.empty() ? 2 : 3);
}

bool get_resp_fixed(In &in, WarpResp &r, uint64_t &n_data) {
  r.rc = in.get<int32_t>();
  for (int32_t &v : r.bbox) v = in.get<int32_t>();
  r.nodata = in.get<double>(); r.dtype = in.get<int32_t>(); r.bytes_read = in.get<int32_t>();
  for (double &v : r.src_gt) v = in.get<double>();
  n_data = in.get<uint64_t>();
  return in.ok;
}

// ---------------------------------------------------------------- reply arenas
// A worker's reply arena: a sealed memfd the worker created and passed with
// its request (SCM_RIGHTS), mapped here and registered with HIP, so the warp
// kernel writes the window straight into memory the worker reads -- no
// read-back copy, no socket copy.  Freed when the connection has moved to a
// bigger arena (or closed) and no batch in flight writes to it.
struct Arena {
  char *host = nullptr;
  size_t bytes = 0;
  uint8_t *dev = nullptr;   // device address of the registered mapping, or NULL (then copied in)
  ~Arena() {
    if (dev) (void)hipHostUnregister(host);
    if (host) ::munmap(host, bytes);
  }
};
using ArenaPtr = std::shared_ptr<Arena>;

// Maps the worker's arena fd (`bytes` claimed).  The memfd must be sealed
// against shrinking, so the worker cannot pull pages out from under the GPU.
ArenaPtr map_arena(int fd, uint64_t bytes, bool register_hip) {
  struct stat st;
  const int seals = ::fcntl(fd, F_GET_SEALS);
  if (bytes == 0 || bytes > (1ull << 32) || ::fstat(fd, &st) != 0 || (uint64_t)st.st_size < bytes || seals < 0 ||
      !(seals & F_SEAL_SHRINK))
    return ArenaPtr();
  void *p = ::mmap(nullptr, (size_t)bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) return ArenaPtr();
  ArenaPtr a = std::make_shared<Arena>();
  a->host = (char *)p;
  a->bytes = (size_t)bytes;
  if (register_hip && hipHostRegister(p, (size_t)bytes, hipHostRegisterMapped) == hipSuccess) {
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) == hipSuccess && d) a->dev = (uint8_t *)d;
    else (void)hipHostUnregister(p);
  }
  return a;
}

// ---------------------------------------------------------------- daemon state
struct Pending {
  WarpReq q;
  WarpResp r;
  ArenaPtr arena;   // the shared-memory reply op: the window goes here
  std::mutex m;
  std::condition_variable cv;
  bool done = false;
  void finish() {
    {
      std::lock_guard<std::mutex> lk(m);
      done = true;
    }
    cv.notify_one();
  }
};
using PendingPtr = std::shared_ptr<Pending>;

constexpr int kSlots = 2;   // batches in flight: one prepared / launched while the other runs and reads back

struct Flight {
  WarpSlot *slot = nullptr;
  std::vector<PendingPtr> take;
  std::vector<WarpReq> reqs;
  std::vector<WarpResp> resps;
  std::vector<uint8_t *> direct;
  std::vector<int64_t> cap;
};

struct Service {
  std::mutex mu;
  std::condition_variable cv_work;   // dispatcher: work + a free slot, or stop
  std::condition_variable cv_done;   // completer: a launched batch, or stop
  std::condition_variable cv_idle;   // registrations: nothing in flight
  std::deque<PendingPtr> queue;
  std::atomic<bool> stop{false};
  bool dispatcher_done = false;
  int max_batch = 64;
  int window_us = 0;
  bool direct = true;                // windows written into registered arenas (GSKYHIP_SVC_DIRECT=0: staged)
  int listen_fd = -1;
  Flight flights[kSlots];
  std::deque<int> free_slots, launched;
  int inflight = 0, reg_waiting = 0;
  // statistics: warp requests, batches, largest batch, registered granules
  std::atomic<int64_t> n_req{0}, n_batches{0}, max_seen{0}, n_reg{0};
  // dispatcher time preparing + launching, request residence (enqueued -> answer ready), ns
  std::atomic<int64_t> batch_ns{0}, resident_ns{0};
  // replies whose window the GPU wrote into the worker's arena / that were copied
  std::atomic<int64_t> n_in_place{0}, n_copied{0};
  std::atomic<int> active{0};          // connection threads still running (detached)
  std::mutex conn_mu;
  std::set<int> conns;                 // open connection fds (shut down on stop)
  std::mutex reg_mu;
  // granule data uploaded through SVC_REGISTER, per (path, band): freed when
  // the granule is registered again or everything is unregistered
  std::map<std::pair<std::string, int32_t>, std::vector<void *>> device_allocs;
  void free_all() {
    for (auto &kv : device_allocs)
      for (void *p : kv.second) (void)hipFree(p);
    device_allocs.clear();
  }
};

// Stop the service: the flag changes under `mu`, so no thread waiting on one
// of its conditions can miss it; every connection is shut down, so threads
// blocked in recv on an idle kept connection leave too.
void request_stop(Service *s) {
  {
    std::lock_guard<std::mutex> lk(s->mu);
    s->stop = true;
  }
  s->cv_work.notify_all();
  s->cv_done.notify_all();
  s->cv_idle.notify_all();
  std::lock_guard<std::mutex> ck(s->conn_mu);
  for (int fd : s->conns) ::shutdown(fd, SHUT_RDWR);
}

Service *g_svc = nullptr;

// The dispatcher: as soon as requests are queued and a slot is free, takes
// up to max_batch of them and launches them (warp_batch_launch, which does
// not wait).  With the other slot still on the GPU it may first let the
// batch grow for window_us; with the GPU idle it dispatches at once.
void dispatch_loop(Service *s) {
  for (;;) {
    int k;
    Flight *F;
    {
      std::unique_lock<std::mutex> lk(s->mu);
      s->cv_work.wait(lk, [&] {
        return s->stop || (!s->queue.empty() && !s->free_slots.empty() && s->reg_waiting == 0);
      });
      if (s->stop) break;
      if (s->inflight > 0 && s->window_us > 0 && (int)s->queue.size() < s->max_batch) {
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(s->window_us);
        s->cv_work.wait_until(lk, until, [&] {
          return s->stop || (int)s->queue.size() >= s->max_batch || s->inflight == 0 || s->reg_waiting > 0;
        });
        if (s->stop) break;
        // a registration that started waiting during the window (it woke on
        // inflight == 0 too) changes the registry now: launching here would
        // run a batch beside it, reading uploads it may free
        if (s->reg_waiting > 0) continue;
      }
      k = s->free_slots.front();
      s->free_slots.pop_front();
      s->inflight++;
      F = &s->flights[k];
      while (!s->queue.empty() && (int)F->take.size() < s->max_batch) {
        F->take.push_back(std::move(s->queue.front()));
        s->queue.pop_front();
      }
    }
    const int m = (int)F->take.size();
    F->reqs.resize(m);
    F->resps.assign(m, WarpResp());
    F->direct.assign(m, nullptr);
    F->cap.assign(m, 0);
    for (int i = 0; i < m; i++) {
      Pending &p = *F->take[i];
      F->reqs[i] = std::move(p.q);
      if (s->direct && p.arena && p.arena->dev) {
        F->direct[i] = p.arena->dev;
        F->cap[i] = (int64_t)p.arena->bytes;
      }
    }
    const auto t0 = std::chrono::steady_clock::now();
    warp_batch_launch(*F->slot, F->reqs.data(), m, F->resps.data(), F->direct.data(), F->cap.data());
    s->batch_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    s->n_batches++;
    int64_t prev = s->max_seen.load();
    while (m > prev && !s->max_seen.compare_exchange_weak(prev, m)) {}
    {
      std::lock_guard<std::mutex> lk(s->mu);
      s->launched.push_back(k);
    }
    s->cv_done.notify_one();
  }
  {
    std::lock_guard<std::mutex> lk(s->mu);
    s->dispatcher_done = true;
  }
  s->cv_done.notify_all();
}

// The completer: finishes launched batches in order and wakes exactly the
// connections whose requests they carried.
void complete_loop(Service *s) {
  for (;;) {
    int k;
    {
      std::unique_lock<std::mutex> lk(s->mu);
      s->cv_done.wait(lk, [&] { return !s->launched.empty() || s->dispatcher_done; });
      if (s->launched.empty()) return;   // the dispatcher has stopped and everything launched is done
      k = s->launched.front();
      s->launched.pop_front();
    }
    Flight &F = s->flights[k];
    warp_batch_finish(*F.slot);
    for (size_t i = 0; i < F.take.size(); i++) {
      F.take[i]->r = std::move(F.resps[i]);
      F.take[i]->finish();
    }
    F.take.clear();
    {
      std::lock_guard<std::mutex> lk(s->mu);
      s->free_slots.push_back(k);
      s->inflight--;
    }
    s->cv_work.notify_one();
    s->cv_idle.notify_all();
  }
}

// SVC_REGISTER payload: path, band, srs, granule header (host struct; data
// pointers ignored), level-0 bytes, n_ovr x overview bytes.  Waits until no
// batch is in flight (and holds new ones back) while it changes the registry.
int do_register(Service *s, In &in) {
  const std::string path = in.get_str();
  const int32_t band = in.get<int32_t>();
  const std::string srs = in.get_str();
  gskyhip_granule g = in.get<gskyhip_granule>();
  if (!in.ok || g.n_ovr < 0 || g.n_ovr > GSKYHIP_MAX_OVR || g.xsize <= 0 || g.ysize <= 0 || type_size(g.dtype) <= 0)
    return GSKYHIP_E_ARG;
  for (int k = 0; k < g.n_ovr; k++)
    if (g.ovr_xsize[k] <= 0 || g.ovr_ysize[k] <= 0) return GSKYHIP_E_ARG;
  {
    std::unique_lock<std::mutex> lk(s->mu);
    if (s->stop) return GSKYHIP_E_SERVICE;
    s->reg_waiting++;
    s->cv_idle.wait(lk, [&] { return s->inflight == 0 || s->stop; });
  }
  struct Resume {
    Service *s;
    ~Resume() {
      {
        std::lock_guard<std::mutex> lk(s->mu);
        s->reg_waiting--;
      }
      s->cv_work.notify_all();
    }
  } resume{s};
  if (s->stop) return GSKYHIP_E_SERVICE;
  std::lock_guard<std::mutex> rl(s->reg_mu);
  std::vector<void *> mine;   // this registration's uploads: freed again on any failure
  auto fail = [&](int e) {
    for (void *p : mine) (void)hipFree(p);
    return e;
  };
  auto upload = [&](const char *p, uint64_t n, void **dev) -> int {
    if (hipMalloc(dev, n > 0 ? n : 1) != hipSuccess) return GSKYHIP_E_HIP;
    mine.push_back(*dev);
    if (n > 0 && hipMemcpy(*dev, p, n, hipMemcpyHostToDevice) != hipSuccess) return GSKYHIP_E_HIP;
    return 0;
  };
  uint64_t n = 0;
  const char *p = in.get_bytes(n);
  if (!in.ok || n != (uint64_t)g.xsize * (uint64_t)g.ysize * (uint64_t)type_size(g.dtype)) return GSKYHIP_E_ARG;
  void *dev = nullptr;
  int e = upload(p, n, &dev);
  if (e) return fail(e);
  g.data = dev;
  for (int k = 0; k < g.n_ovr; k++) {
    const char *po = in.get_bytes(n);
    if (!in.ok || n != (uint64_t)g.ovr_xsize[k] * (uint64_t)g.ovr_ysize[k] * (uint64_t)type_size(g.dtype))
      return fail(GSKYHIP_E_ARG);
    void *od = nullptr;
    if ((e = upload(po, n, &od))) return fail(e);
    g.ovr_data[k] = od;
  }
  e = gskyhip_register_granule(path.c_str(), band, &g, srs.empty() ? nullptr : srs.c_str());
  if (e) return fail(e);
  auto &slot = s->device_allocs[std::make_pair(path, band)];
  for (void *q : slot) (void)hipFree(q);   // a granule refresh replaces the old upload
  slot = std::move(mine);
  s->n_reg = (int64_t)s->device_allocs.size();
  return 0;
}

int do_unregister_all(Service *s) {
  {
    std::unique_lock<std::mutex> lk(s->mu);
    if (s->stop) return GSKYHIP_E_SERVICE;
    s->reg_waiting++;
    s->cv_idle.wait(lk, [&] { return s->inflight == 0 || s->stop; });
  }
  {
    std::lock_guard<std::mutex> rl(s->reg_mu);
    if (!s->stop) {
      gskyhip_unregister_all();
      s->free_all();
      s->n_reg = 0;
    }
  }
  {
    std::lock_guard<std::mutex> lk(s->mu);
    s->reg_waiting--;
  }
  s->cv_work.notify_all();
  return s->stop ? GSKYHIP_E_SERVICE : 0;
}

// Queue one warp and wait for its batch.
void run_warp(Service *s, const PendingPtr &pd) {
  s->n_req++;
  const auto t0 = std::chrono::steady_clock::now();
  bool queued = false;
  {
    std::lock_guard<std::mutex> lk(s->mu);
    if (!s->stop) {
      s->queue.push_back(pd);
      queued = true;
    }
  }
  if (!queued) {   // shutting down: the dispatcher may be gone, answer now
    pd->r.rc = GSKYHIP_E_SERVICE;
    return;
  }
  s->cv_work.notify_one();
  {
    std::unique_lock<std::mutex> lk(pd->m);
    pd->cv.wait(lk, [&] { return pd->done; });
  }
  s->resident_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

// recv that also collects a file descriptor passed with SCM_RIGHTS
bool read_all_fd(int fd, void *buf, size_t n, int &passed) {
  char *p = (char *)buf;
  while (n > 0) {
    iovec iov{p, n};
    alignas(cmsghdr) char cbuf[CMSG_SPACE(sizeof(int))];
    msghdr m;
    std::memset(&m, 0, sizeof(m));
    m.msg_iov = &iov;
    m.msg_iovlen = 1;
    m.msg_control = cbuf;
    m.msg_controllen = sizeof(cbuf);
    const ssize_t k = ::recvmsg(fd, &m, MSG_CMSG_CLOEXEC);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    for (cmsghdr *c = CMSG_FIRSTHDR(&m); c; c = CMSG_NXTHDR(&m, c))
      if (c->cmsg_level == SOL_SOCKET && c->cmsg_type == SCM_RIGHTS && c->cmsg_len >= CMSG_LEN(sizeof(int))) {
        int got;
        std::memcpy(&got, CMSG_DATA(c), sizeof(int));
        if (passed >= 0) ::close(passed);
        passed = got;
      }
    p += k;
    n -= (size_t)k;
  }
  return true;
}

// The reply to SVC_WARP_SHM: fixed fields, then where the window is (1: at
// offset 0 of the worker's arena; 0: inline after this word).
bool send_resp_shm(int fd, const WarpResp &r, const ArenaPtr &arena, Service *s) {
  Out o;
  // the length word is the window's length wherever it is
  put_resp_fixed(o, r, r.rc == 0 && r.in_place >= 0 ? (uint64_t)r.in_place : r.data.size());
  const char *inl = nullptr;
  size_t n_inl = 0;
  uint32_t where = 0;
  if (r.rc == 0) {
    if (r.in_place >= 0) {
      where = 1;
      s->n_in_place++;
    } else if (arena && r.data.size() <= arena->bytes) {
      if (!r.data.empty()) std::memcpy(arena->host, r.data.data(), r.data.size());
      where = 1;
      s->n_copied++;
    } else {
      inl = r.data.data();
      n_inl = r.data.size();
      s->n_copied++;
    }
  }
  o.put(where);
  char hdr[16];
  const uint32_t op = SVC_WARP_SHM;
  const uint64_t n = o.b.size() + n_inl;
  std::memcpy(hdr, &kSvcMagic, 4);
  std::memcpy(hdr + 4, &op, 4);
  std::memcpy(hdr + 8, &n, 8);
  iovec iov[3] = {{hdr, 16}, {o.b.data(), o.b.size()}, {(void *)inl, n_inl}};
  return write_allv(fd, iov, n_inl ? 3 : 2);
}

void conn_serve(Service *s, int fd) {
  ArenaPtr arena;
  int passed = -1;
  struct CloseFd {
    int &fd;
    ~CloseFd() { if (fd >= 0) ::close(fd); }
  } close_passed{passed};
  for (;;) {
    char hdr[16];
    if (!read_all_fd(fd, hdr, 16, passed)) break;
    uint32_t magic, op;
    uint64_t n;
    std::memcpy(&magic, hdr, 4);
    std::memcpy(&op, hdr + 4, 4);
    std::memcpy(&n, hdr + 8, 8);
    if (magic != kSvcMagic || n > max_payload(op)) break;
    std::vector<char> payload;
    try {
      payload.resize(n);
    } catch (const std::bad_alloc &) {
      break;
    }
    if (n > 0 && !read_all_fd(fd, payload.data(), n, passed)) break;
    In in{payload.data(), payload.data() + payload.size()};
    Out o;
    if (op == SVC_WARP || op == SVC_WARP_SHM) {
      auto pd = std::make_shared<Pending>();
      if (op == SVC_WARP_SHM) {
        const uint64_t new_bytes = in.get<uint64_t>();
        if (!in.ok) break;
        if (new_bytes > 0) {   // the worker moved to a new (bigger) arena, passed with this message
          ArenaPtr a;
          if (passed >= 0) a = map_arena(passed, new_bytes, s->direct);
          if (passed >= 0) { ::close(passed); passed = -1; }
          arena = a;           // NULL if it could not be mapped: replies go inline
        }
        pd->arena = arena;
      }
      if (!get_req(in, pd->q)) break;
      run_warp(s, pd);
      const bool sent = op == SVC_WARP_SHM ? send_resp_shm(fd, pd->r, arena, s) : send_resp(fd, pd->r);
      if (!sent) break;   // the worker died (SIGKILL): drop the reply
      continue;
    } else if (op == SVC_REGISTER) {
      o.put<int32_t>(do_register(s, in));
    } else if (op == SVC_UNREGISTER_ALL) {
      o.put<int32_t>(do_unregister_all(s));
    } else if (op == SVC_STATS) {
      o.put<int64_t>(s->n_req.load()); o.put<int64_t>(s->n_batches.load());
      o.put<int64_t>(s->max_seen.load()); o.put<int64_t>(s->n_reg.load());
      o.put<int64_t>(s->batch_ns.load()); o.put<int64_t>(s->resident_ns.load());
      int64_t wb[4];
      warp_batch_timers(wb);
      for (int k = 0; k < 3; k++) o.put<int64_t>(wb[k]);
      o.put<int64_t>(s->n_in_place.load()); o.put<int64_t>(s->n_copied.load());
    } else if (op == SVC_SHUTDOWN) {
      o.put<int32_t>(0);
      send_msg(fd, op, o.b);
      request_stop(s);
      ::shutdown(s->listen_fd, SHUT_RDWR);
      break;
    } else {
      break;
    }
    if (!send_msg(fd, op, o.b)) break;   // the worker died (SIGKILL): drop the reply
  }
}

void conn_loop(Service *s, int fd) {
  try {
    conn_serve(s, fd);
  } catch (...) {   // one bad connection must not std::terminate the daemon
  }
  {
    std::lock_guard<std::mutex> ck(s->conn_mu);
    s->conns.erase(fd);
    ::close(fd);
  }
  s->active--;
}

}  // namespace

namespace {
// the calling thread's connection to the service and its reply arena
// (reused across requests; a fresh connection after fork or a broken pipe)
struct ClientConn {
  std::string sock;
  int fd = -1;
  pid_t pid = 0;
  char *arena = nullptr;        // this thread's mapping of its arena memfd
  int arena_fd = -1;            // ... and the memfd (passed again on a new connection)
  size_t arena_bytes = 0;
  bool arena_sent = false;      // the daemon has this arena on this connection
  bool shm = true;              // memfd arenas work here (else the socket carries the window)
  ~ClientConn() {
    if (fd >= 0) ::close(fd);
    if (arena) ::munmap(arena, arena_bytes);
    if (arena_fd >= 0) ::close(arena_fd);
  }
};
thread_local ClientConn t_conn;

int client_fd(const char *sock, bool fresh) {
  ClientConn &c = t_conn;
  if (c.pid != ::getpid() && c.arena) {   // a forked child shares the parent's arena: make its own
    ::munmap(c.arena, c.arena_bytes);
    ::close(c.arena_fd);
    c.arena = nullptr;
    c.arena_fd = -1;
    c.arena_bytes = 0;
  }
  if (c.fd >= 0 && (fresh || c.pid != ::getpid() || c.sock != sock)) { ::close(c.fd); c.fd = -1; }
  if (c.fd < 0) {
    c.fd = connect_to(sock);
    c.sock = sock;
    c.pid = ::getpid();
    c.arena_sent = false;   // a new connection has no arena on the daemon side
  }
  return c.fd;
}
void client_drop() {
  if (t_conn.fd >= 0) ::close(t_conn.fd);
  t_conn.fd = -1;
  t_conn.arena_sent = false;
}

// This thread's arena becomes a sealed memfd of at least `need` bytes,
// mapped read-only here; false if memfds cannot be made.
bool client_arena(size_t need) {
  ClientConn &c = t_conn;
  size_t bytes = (size_t)2 << 20;
  while (bytes < need) bytes <<= 1;
  const int mfd = (int)::syscall(SYS_memfd_create, "gskyhip-reply", MFD_CLOEXEC | MFD_ALLOW_SEALING);
  if (mfd < 0) return false;
  void *p = MAP_FAILED;
  if (::ftruncate(mfd, (off_t)bytes) == 0 &&
      ::fcntl(mfd, F_ADD_SEALS, F_SEAL_SHRINK | F_SEAL_GROW | F_SEAL_SEAL) == 0)
    p = ::mmap(nullptr, bytes, PROT_READ, MAP_SHARED, mfd, 0);
  if (p == MAP_FAILED) {
    ::close(mfd);
    return false;
  }
  if (c.arena) ::munmap(c.arena, c.arena_bytes);
  if (c.arena_fd >= 0) ::close(c.arena_fd);
  c.arena = (char *)p;
  c.arena_fd = mfd;
  c.arena_bytes = bytes;
  c.arena_sent = false;
  return true;
}

// header + payload in one sendmsg, with `pass_fd` attached when >= 0
bool send_msg_fd(int fd, uint32_t op, const std::vector<char> &payload, int pass_fd) {
  char hdr[16];
  const uint64_t n = payload.size();
  std::memcpy(hdr, &kSvcMagic, 4);
  std::memcpy(hdr + 4, &op, 4);
  std::memcpy(hdr + 8, &n, 8);
  iovec iov[2] = {{hdr, 16}, {(void *)payload.data(), payload.size()}};
  msghdr m;
  std::memset(&m, 0, sizeof(m));
  m.msg_iov = iov;
  m.msg_iovlen = n ? 2 : 1;
  alignas(cmsghdr) char cbuf[CMSG_SPACE(sizeof(int))];
  if (pass_fd >= 0) {
    std::memset(cbuf, 0, sizeof(cbuf));
    m.msg_control = cbuf;
    m.msg_controllen = sizeof(cbuf);
    cmsghdr *c = CMSG_FIRSTHDR(&m);
    c->cmsg_level = SOL_SOCKET;
    c->cmsg_type = SCM_RIGHTS;
    c->cmsg_len = CMSG_LEN(sizeof(int));
    std::memcpy(CMSG_DATA(c), &pass_fd, sizeof(int));
  }
  ssize_t k;
  do {
    k = ::sendmsg(fd, &m, MSG_NOSIGNAL);
  } while (k < 0 && errno == EINTR);
  if (k <= 0) return false;
  if ((size_t)k == 16 + n) return true;
  // a partial send: the descriptor went with the first bytes; finish plainly
  size_t done = (size_t)k;
  if (done < 16) {
    if (!write_all(fd, hdr + done, 16 - done)) return false;
    done = 16;
  }
  return write_all(fd, payload.data() + (done - 16), n - (done - 16));
}
}  // namespace

// The window of a reply into malloc'd memory (mbuf) or r.data.
namespace {
bool take_window(const char *src, uint64_t nd, WarpResp &r, void **mbuf, size_t *mlen) {
  if (mbuf) {
    *mbuf = std::malloc(nd ? nd : 1);
    if (!*mbuf) return false;
    if (nd) std::memcpy(*mbuf, src, nd);
    *mlen = (size_t)nd;
  } else {
    r.data.assign(src, src + nd);
  }
  return true;
}
}  // namespace

int service_warp(const char *sock, const WarpReq &q, WarpResp &r, void **mbuf, size_t *mlen) {
  // a kept connection may have been closed by a restarted daemon: one retry
  // on a fresh connection (a warp request only reads, so a repeat is harmless)
  for (int attempt = 0; attempt < 2; attempt++) {
    const int fd = client_fd(sock, attempt > 0);
    if (fd < 0) return GSKYHIP_E_SERVICE;
    ClientConn &c = t_conn;
    const size_t need = (size_t)std::max(1, q.width) * (size_t)std::max(1, q.height) * 8;
    if (c.shm && c.arena_bytes < need && !client_arena(need)) c.shm = false;
    char hdr[16];
    if (c.shm) {
      Out o;
      const int pass = c.arena_sent ? -1 : c.arena_fd;   // a new arena, or a new connection
      o.put<uint64_t>(pass >= 0 ? (uint64_t)c.arena_bytes : 0);
      put_req(o, q);
      if (!send_msg_fd(fd, SVC_WARP_SHM, o.b, pass) || !read_all(fd, hdr, 16)) { client_drop(); continue; }
      c.arena_sent = true;
      uint32_t magic, op;
      uint64_t n;
      std::memcpy(&magic, hdr, 4);
      std::memcpy(&op, hdr + 4, 4);
      std::memcpy(&n, hdr + 8, 8);
      char fixed[kRespFixed + 4];
      if (magic != kSvcMagic || op != SVC_WARP_SHM || n < kRespFixed + 4 || n > (1ull << 36) ||
          !read_all(fd, fixed, kRespFixed + 4)) {
        client_drop();
        return GSKYHIP_E_SERVICE;
      }
      In in{fixed, fixed + kRespFixed};
      uint64_t nd = 0;
      uint32_t where;
      std::memcpy(&where, fixed + kRespFixed, 4);
      if (!get_resp_fixed(in, r, nd)) { client_drop(); return GSKYHIP_E_SERVICE; }
      if (r.rc) {
        if (n != kRespFixed + 4) { client_drop(); return GSKYHIP_E_SERVICE; }
        return 0;
      }
      if (where == 1) {   // in this thread's arena
        if (n != kRespFixed + 4 || nd > c.arena_bytes || !take_window(c.arena, nd, r, mbuf, mlen)) {
          client_drop();
          return GSKYHIP_E_SERVICE;
        }
        return 0;
      }
      if (nd != n - kRespFixed - 4) { client_drop(); return GSKYHIP_E_SERVICE; }
      std::vector<char> tmp(nd);
      if ((nd && !read_all(fd, tmp.data(), nd)) || !take_window(tmp.data(), nd, r, mbuf, mlen)) {
        client_drop();
        return GSKYHIP_E_SERVICE;
      }
      return 0;
    }
    // no memfd here: the window travels in the socket (SVC_WARP)
    Out o;
    put_req(o, q);
    if (!send_msg(fd, SVC_WARP, o.b) || !read_all(fd, hdr, 16)) { client_drop(); continue; }
    uint32_t magic, op;
    uint64_t n;
    std::memcpy(&magic, hdr, 4);
    std::memcpy(&op, hdr + 4, 4);
    std::memcpy(&n, hdr + 8, 8);
    char fixed[kRespFixed];
    if (magic != kSvcMagic || op != SVC_WARP || n < kRespFixed || n > (1ull << 36) ||
        !read_all(fd, fixed, kRespFixed)) {
      client_drop();
      return GSKYHIP_E_SERVICE;
    }
    In in{fixed, fixed + kRespFixed};
    uint64_t nd = 0;
    if (!get_resp_fixed(in, r, nd) || nd != n - kRespFixed) { client_drop(); return GSKYHIP_E_SERVICE; }
    char *dst;
    if (mbuf) {
      *mbuf = std::malloc(nd ? nd : 1);
      if (!*mbuf) { client_drop(); return GSKYHIP_E_SERVICE; }
      dst = (char *)*mbuf;
      *mlen = (size_t)nd;
    } else {
      r.data.resize(nd);
      dst = r.data.data();
    }
    if (nd && !read_all(fd, dst, nd)) {
      if (mbuf) { std::free(*mbuf); *mbuf = nullptr; }
      client_drop();
      return GSKYHIP_E_SERVICE;
    }
    return 0;
  }
  return GSKYHIP_E_SERVICE;
}

}  // namespace gsky

using namespace gsky;

extern "C" {

int gskyhip_service_run(const char *socket_path, int max_batch, int window_us) {
  if (!socket_path || !*socket_path || std::strlen(socket_path) >= sizeof(sockaddr_un::sun_path))
    return GSKYHIP_E_ARG;
  // heap-allocated: connection threads are detached (a long-running daemon
  // must not accumulate finished threads) and may outlive a forced shutdown
  Service &s = *new Service;
  s.max_batch = std::max(1, max_batch);
  s.window_us = std::max(0, window_us);
  const int fd = ::socket(AF_UNIX, SOCK_STREAM, 0);
  if (fd < 0) return GSKYHIP_E_SERVICE;
  sockaddr_un a;
  std::memset(&a, 0, sizeof(a));
  a.sun_family = AF_UNIX;
  std::strncpy(a.sun_path, socket_path, sizeof(a.sun_path) - 1);
  ::unlink(socket_path);
  if (::bind(fd, (sockaddr *)&a, sizeof(a)) != 0 || ::listen(fd, 256) != 0) {
    ::close(fd);
    delete &s;
    return GSKYHIP_E_SERVICE;
  }
  s.listen_fd = fd;
  // GSKYHIP_SVC_DIRECT=0: windows staged in HBM and read back by the daemon
  // (round 4's path) instead of written into the workers' arenas
  if (const char *e = std::getenv("GSKYHIP_SVC_DIRECT")) s.direct = std::atoi(e) != 0;
  for (int k = 0; k < kSlots; k++) {
    s.flights[k].slot = warp_slot_create();
    s.free_slots.push_back(k);
  }
  g_svc = &s;
  std::thread dispatcher(dispatch_loop, &s), completer(complete_loop, &s);
  while (!s.stop) {
    const int c = ::accept(fd, nullptr, nullptr);
    if (c < 0) {
      if (errno == EINTR) continue;
      break;
    }
    {
      std::lock_guard<std::mutex> ck(s.conn_mu);
      if (s.stop) { ::close(c); break; }
      s.conns.insert(c);
    }
    s.active++;
    std::thread(conn_loop, &s, c).detach();
  }
  request_stop(&s);
  dispatcher.join();
  completer.join();   // every launched batch finished and answered
  {   // release connections still waiting in the queue
    std::lock_guard<std::mutex> lk(s.mu);
    for (auto &p : s.queue) {
      p->r.rc = GSKYHIP_E_SERVICE;
      p->finish();
    }
    s.queue.clear();
  }
  // every connection was shut down: its thread leaves recv and ends
  for (int k = 0; k < 500 && s.active.load() > 0; k++) std::this_thread::sleep_for(std::chrono::milliseconds(10));
  ::close(fd);
  ::unlink(socket_path);
  for (int k = 0; k < kSlots; k++) warp_slot_destroy(s.flights[k].slot);
  {
    std::lock_guard<std::mutex> rl(s.reg_mu);
    gskyhip_unregister_all();
    s.free_all();
  }
  g_svc = nullptr;
  if (s.active.load() == 0) delete &s;
  return 0;
}

int gskyhip_service_register_granule(const char *socket_path, const char *path, int band,
                                     const gskyhip_granule *g, const void *data, const void *const *ovr_data,
                                     const char *srs) {
  if (!socket_path || !path || !g || !data) return GSKYHIP_E_ARG;
  if (g->n_ovr < 0 || g->n_ovr > GSKYHIP_MAX_OVR || (g->n_ovr > 0 && !ovr_data)) return GSKYHIP_E_ARG;
  const int ts = type_size(g->dtype);
  if (ts <= 0) return GSKYHIP_E_TYPE;
  Out o;
  o.put_str(path);
  o.put<int32_t>(band);
  o.put_str(srs ? srs : "");
  o.put(*g);
  o.put_bytes(data, (size_t)g->xsize * g->ysize * ts);
  for (int k = 0; k < g->n_ovr; k++) o.put_bytes(ovr_data[k], (size_t)g->ovr_xsize[k] * g->ovr_ysize[k] * ts);
  std::vector<char> rep;
  if (!exchange(socket_path, SVC_REGISTER, o.b, rep) || rep.size() < 4) return GSKYHIP_E_SERVICE;
  int32_t rc;
  std::memcpy(&rc, rep.data(), 4);
  return rc;
}

int gskyhip_service_unregister_all(const char *socket_path) {
  std::vector<char> rep;
  if (!socket_path || !exchange(socket_path, SVC_UNREGISTER_ALL, {}, rep) || rep.size() < 4)
    return GSKYHIP_E_SERVICE;
  int32_t rc;
  std::memcpy(&rc, rep.data(), 4);
  return rc;
}

int gskyhip_service_stats(const char *socket_path, int64_t *stats) {
  return gskyhip_service_stats_n(socket_path, stats, 4);
}

int gskyhip_service_stats_n(const char *socket_path, int64_t *stats, int n_stats) {
  std::vector<char> rep;
  if (!socket_path || !stats || n_stats < 0 || !exchange(socket_path, SVC_STATS, {}, rep) || rep.size() < 32)
    return GSKYHIP_E_SERVICE;
  const size_t n = std::min<size_t>((size_t)n_stats, rep.size() / 8);
  std::memcpy(stats, rep.data(), 8 * n);
  for (int k = (int)n; k < n_stats; k++) stats[k] = 0;
  return 0;
}

int gskyhip_service_shutdown(const char *socket_path) {
  std::vector<char> rep;
  if (!socket_path || !exchange(socket_path, SVC_SHUTDOWN, {}, rep)) return GSKYHIP_E_SERVICE;
  return 0;
}

}  // extern "C"
