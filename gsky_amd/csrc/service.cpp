// service.cpp -- per-node GPU warp service: client side (forwarding from
// warp_operation_fast) and the daemon loop (gskyhip_service_run, gskyhipd).
// See service.h for the design.
#include <errno.h>
#include <signal.h>
#include <sys/socket.h>
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
    case SVC_WARP: return 1ull << 20;
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

void put_resp_fixed(Out &o, const WarpResp &r) {
  o.put(r.rc);
  for (int32_t v : r.bbox) o.put(v);
  o.put(r.nodata); o.put(r.dtype); o.put(r.bytes_read);
  for (double v : r.src_gt) o.put(v);
  o.put<uint64_t>(r.data.size());
}

bool send_resp(int fd, const WarpResp &r) {
  Out o;
  put_resp_fixed(o, r);
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

// ---------------------------------------------------------------- daemon state
struct Pending {
  WarpReq q;
  WarpResp r;
  bool done = false;
};

struct Service {
  std::mutex mu;
  std::condition_variable cv_queue, cv_done;
  std::deque<std::shared_ptr<Pending>> queue;
  std::atomic<bool> stop{false};
  int max_batch = 64;
  int window_us = 500;
  int listen_fd = -1;
  // statistics: warp requests, batches, largest batch, registered granules
  std::atomic<int64_t> n_req{0}, n_batches{0}, max_seen{0}, n_reg{0};
  // time in warp_batch, and request residence (enqueued -> answer ready), ns
  std::atomic<int64_t> batch_ns{0}, resident_ns{0};
  std::atomic<int> active{0};          // connection threads still running (detached)
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

// Stop the service: the flag changes under `mu`, so neither the batcher nor a
// connection waiting to enqueue can miss it.
void request_stop(Service *s) {
  {
    std::lock_guard<std::mutex> lk(s->mu);
    s->stop = true;
  }
  s->cv_queue.notify_all();
  s->cv_done.notify_all();
}

Service *g_svc = nullptr;

// The batching thread: waits for work, lets the window fill (up to max_batch),
// runs one warp_batch over everything it took.
void batch_loop(Service *s) {
  for (;;) {
    std::vector<std::shared_ptr<Pending>> take;
    {
      std::unique_lock<std::mutex> lk(s->mu);
      s->cv_queue.wait(lk, [&] { return s->stop || !s->queue.empty(); });
      if (s->stop && s->queue.empty()) return;
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(s->window_us);
      s->cv_queue.wait_until(lk, until, [&] { return s->stop || (int)s->queue.size() >= s->max_batch; });
      while (!s->queue.empty() && (int)take.size() < s->max_batch) {
        take.push_back(s->queue.front());
        s->queue.pop_front();
      }
    }
    const int m = (int)take.size();
    std::vector<WarpReq> reqs(m);
    std::vector<WarpResp> resps(m);
    for (int i = 0; i < m; i++) reqs[i] = take[i]->q;
    {
      std::lock_guard<std::mutex> rl(s->reg_mu);   // registrations do not race a batch
      const auto t0 = std::chrono::steady_clock::now();
      warp_batch(reqs.data(), m, resps.data());
      s->batch_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    }
    s->n_batches++;
    int64_t prev = s->max_seen.load();
    while (m > prev && !s->max_seen.compare_exchange_weak(prev, m)) {}
    {
      std::lock_guard<std::mutex> lk(s->mu);
      for (int i = 0; i < m; i++) {
        take[i]->r = std::move(resps[i]);
        take[i]->done = true;
      }
    }
    s->cv_done.notify_all();
  }
}

// SVC_REGISTER payload: path, band, srs, granule header (host struct; data
// pointers ignored), level-0 bytes, n_ovr x overview bytes.
int do_register(Service *s, In &in) {
  const std::string path = in.get_str();
  const int32_t band = in.get<int32_t>();
  const std::string srs = in.get_str();
  gskyhip_granule g = in.get<gskyhip_granule>();
  if (!in.ok || g.n_ovr < 0 || g.n_ovr > GSKYHIP_MAX_OVR || g.xsize <= 0 || g.ysize <= 0 || type_size(g.dtype) <= 0)
    return GSKYHIP_E_ARG;
  for (int k = 0; k < g.n_ovr; k++)
    if (g.ovr_xsize[k] <= 0 || g.ovr_ysize[k] <= 0) return GSKYHIP_E_ARG;
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

void conn_serve(Service *s, int fd) {
  for (;;) {
    uint32_t op = 0;
    std::vector<char> payload;
    if (!recv_msg(fd, op, payload)) break;
    In in{payload.data(), payload.data() + payload.size()};
    Out o;
    if (op == SVC_WARP) {
      auto pd = std::make_shared<Pending>();
      if (!get_req(in, pd->q)) break;
      s->n_req++;
      const auto t0 = std::chrono::steady_clock::now();
      {
        std::unique_lock<std::mutex> lk(s->mu);
        if (s->stop) {   // shutting down: the batcher may be gone, answer now
          pd->r.rc = GSKYHIP_E_SERVICE;
          pd->done = true;
        } else {
          s->queue.push_back(pd);
          s->cv_queue.notify_one();
          s->cv_done.wait(lk, [&] { return pd->done; });
        }
      }
      s->resident_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
      if (!send_resp(fd, pd->r)) break;   // the worker died (SIGKILL): drop the reply
      continue;
    } else if (op == SVC_REGISTER) {
      o.put<int32_t>(do_register(s, in));
    } else if (op == SVC_UNREGISTER_ALL) {
      std::lock_guard<std::mutex> rl(s->reg_mu);
      gskyhip_unregister_all();
      s->free_all();
      s->n_reg = 0;
      o.put<int32_t>(0);
    } else if (op == SVC_STATS) {
      o.put<int64_t>(s->n_req.load()); o.put<int64_t>(s->n_batches.load());
      o.put<int64_t>(s->max_seen.load()); o.put<int64_t>(s->n_reg.load());
      o.put<int64_t>(s->batch_ns.load()); o.put<int64_t>(s->resident_ns.load());
      int64_t wb[4];
      warp_batch_timers(wb);
      for (int k = 0; k < 3; k++) o.put<int64_t>(wb[k]);
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
  ::close(fd);
  s->active--;
}

}  // namespace

namespace {
// the calling thread's connection to the service (reused across requests;
// round 4 connected per request, and the daemon started a thread per
// connection)
struct ClientConn {
  std::string sock;
  int fd = -1;
  pid_t pid = 0;
  ~ClientConn() { if (fd >= 0) ::close(fd); }
};
thread_local ClientConn t_conn;

int client_fd(const char *sock, bool fresh) {
  ClientConn &c = t_conn;
  if (c.fd >= 0 && (fresh || c.pid != ::getpid() || c.sock != sock)) { ::close(c.fd); c.fd = -1; }
  if (c.fd < 0) { c.fd = connect_to(sock); c.sock = sock; c.pid = ::getpid(); }
  return c.fd;
}
void client_drop() {
  if (t_conn.fd >= 0) ::close(t_conn.fd);
  t_conn.fd = -1;
}
}  // namespace

int service_warp(const char *sock, const WarpReq &q, WarpResp &r, void **mbuf, size_t *mlen) {
  Out o;
  put_req(o, q);
  // a kept connection may have been closed by a restarted daemon: one retry
  // on a fresh connection (a warp request only reads, so a repeat is harmless)
  for (int attempt = 0; attempt < 2; attempt++) {
    const int fd = client_fd(sock, attempt > 0);
    if (fd < 0) return GSKYHIP_E_SERVICE;
    char hdr[16];
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
  g_svc = &s;
  std::thread batcher(batch_loop, &s);
  while (!s.stop) {
    const int c = ::accept(fd, nullptr, nullptr);
    if (c < 0) {
      if (errno == EINTR) continue;
      break;
    }
    s.active++;
    std::thread(conn_loop, &s, c).detach();
  }
  request_stop(&s);
  batcher.join();
  {   // release connections still waiting on a batch
    std::lock_guard<std::mutex> lk(s.mu);
    for (auto &p : s.queue) { p->r.rc = GSKYHIP_E_SERVICE; p->done = true; }
    s.queue.clear();
  }
  s.cv_done.notify_all();
  // workers keep their connections: give busy ones a few seconds, then leave
  // any idle persistent connection behind (its thread ends when it closes)
  for (int k = 0; k < 500 && s.active.load() > 0; k++) std::this_thread::sleep_for(std::chrono::milliseconds(10));
  ::close(fd);
  ::unlink(socket_path);
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
