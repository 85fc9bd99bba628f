// Native HTTP/1.1 front end of the predictor (rafiki_amd/predictor/nativeserve.py).
//
// Reference: rafiki/predictor/app.py:23-30 (Flask, `POST /predict {"query": q}` -> `{"prediction": p}`,
// one query per request) behind Redis polling (predictor.py:31-74).  Python's per-request cost
// (socket handling, HTTP parsing, JSON decoding of 3072 ints, futures, response encoding: ~250 us
// under the GIL) capped single-query serving at ~4 k QPS.  Here everything per request runs in C++
// threads that never touch the GIL:
//
//   acceptor thread --round robin--> N I/O threads (epoll, non-blocking keep-alive connections)
//     * parse the request line + Content-Length, read the body;
//     * `POST /predict` whose "query" is a rectangular uint8 integer array (an image): decoded
//       straight to bytes and queued for batching;
//     * `POST /predict_batch_npy` with a uint8 .npy body: its images join the same queue as one
//       request and are answered with one .npy float32 [n, classes] array;
//     * `GET /`: answered in place;
//     * anything else: queued as a generic request for Python (same wire contract as before).
//   Python batch threads (one per predictor replica) call rt_http_next_batch(): it blocks (ctypes
//   drops the GIL) until queries are pending, then hands over EVERY pending query of one input
//   shape (up to max_batch) as one contiguous uint8 batch — batches form by construction while the
//   GPU runs the previous one, no timer.  rt_http_complete() formats each `{"prediction": [...]}`
//   response (shortest-repr doubles, as Python's json) and posts it to the owning I/O thread.
//
// Responses go out in request order per connection (HTTP/1.1 pipelining safe).  Connections are
// addressed by 64-bit ids, so a completion for a connection that closed meanwhile is dropped.
// Limits: header block <= 64 KiB, body <= max_body (413), <= 16384 connections.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <charconv>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

extern "C" long long rt_json_u8_array(const char* body, long long len, const char* key, uint8_t* out, long long cap,
                                      long long* shape, int* ndim);

namespace {

constexpr size_t kMaxHeader = 64 << 10;
constexpr size_t kMaxConns = 16384;
constexpr long long kMaxNpyBatch = 64ll << 20;   // image bytes of one .npy request on the batch path

struct Item {  // one batchable request: a JSON image query (count 1) or an npy batch of `count` images
  uint64_t conn;
  int io;
  uint64_t seq;
  bool close;
  bool npy;
  long long count;
  int ndim;
  long long shape[8];   // ONE image
  std::vector<uint8_t> data;
};

struct Ticket {  // where a response goes
  uint64_t conn;
  int io;
  uint64_t seq;
  bool close;
  bool npy = false;      // respond with an .npy float32 [count, ncls] array instead of {"prediction": [...]}
  long long count = 1;   // images of the batch that belong to this request
};

struct Generic {  // a request Python answers
  Ticket t;
  std::string method, path, body;
};

struct Outgoing {
  uint64_t conn;
  uint64_t seq;
  std::string bytes;
  bool close;
};

struct Conn {
  int fd = -1;
  uint64_t id = 0;
  std::string in;
  std::string out;
  size_t out_off = 0;
  uint64_t next_seq = 0;   // assigned to the next parsed request
  uint64_t next_send = 0;  // the response that goes out next
  std::map<uint64_t, std::pair<std::string, bool>> ready;
  bool closing = false;    // close once everything queued is written
  uint32_t mask = EPOLLIN | EPOLLRDHUP;
};

struct Server;

struct IoThread {
  Server* srv = nullptr;
  int idx = 0;
  int ep = -1;
  int evfd = -1;
  std::thread th;
  std::unordered_map<uint64_t, Conn*> conns;
  std::unordered_map<int, Conn*> by_fd;
  std::mutex mu;
  std::vector<Outgoing> mailbox;
  std::vector<int> new_fds;
};

struct Server {
  int lfd = -1;
  std::thread acceptor;
  std::vector<std::unique_ptr<IoThread>> io;
  std::atomic<bool> stop{false};
  std::atomic<uint64_t> next_conn{1}, next_id{1};
  std::atomic<long long> nconns{0};
  long long max_batch = 512;
  long long max_body = 256 << 20;
  long long max_query = 1 << 20;  // bytes of ONE image query on the batch path; larger ones go to Python
  bool batching = true;
  std::mutex qmu;
  // one condition variable per queue: a notify for an image query must never be consumed by the generic
  // thread (whose predicate stays false) while the batch threads sleep out their timeout
  std::condition_variable qcv;   // items (batch threads)
  std::condition_variable gcv;   // generic requests (the Python request thread)
  std::deque<Item> items;
  std::deque<std::pair<uint64_t, Generic>> generic;
  std::unordered_map<uint64_t, std::vector<Ticket>> batches;
  std::unordered_map<uint64_t, Generic> taken;  // generic requests handed to Python
  // stats
  std::atomic<long long> requests{0}, nbatches{0}, batched{0}, ngeneric{0}, errors{0}, accepted{0};
};

void post(Server* s, const Ticket& t, std::string bytes) {
  IoThread* io = s->io[t.io].get();
  {
    std::lock_guard<std::mutex> g(io->mu);
    io->mailbox.push_back(Outgoing{t.conn, t.seq, std::move(bytes), t.close});
  }
  uint64_t one = 1;
  ssize_t r = write(io->evfd, &one, sizeof(one));
  (void)r;
}

std::string http_response(int status, const char* ctype, const char* body, size_t n, bool close) {
  const char* reason = status == 200 ? "OK" : status == 400 ? "Bad Request" : status == 404 ? "Not Found"
                       : status == 405 ? "Method Not Allowed" : status == 413 ? "Payload Too Large"
                       : status == 503 ? "Service Unavailable" : "Internal Server Error";
  std::string r;
  r.reserve(n + 128);
  r += "HTTP/1.1 ";
  r += std::to_string(status);
  r += ' ';
  r += reason;
  r += "\r\nContent-Type: ";
  r += ctype;
  r += "\r\nContent-Length: ";
  r += std::to_string(n);
  r += close ? "\r\nConnection: close\r\n\r\n" : "\r\n\r\n";
  r.append(body, n);
  return r;
}

void close_conn(IoThread* io, Conn* c) {
  epoll_ctl(io->ep, EPOLL_CTL_DEL, c->fd, nullptr);
  close(c->fd);
  io->by_fd.erase(c->fd);
  io->conns.erase(c->id);
  io->srv->nconns--;
  delete c;
}

// epoll interest: read until the connection is closing, write while output is pending
void update_mask(IoThread* io, Conn* c) {
  uint32_t m = (c->closing ? 0u : (uint32_t)(EPOLLIN | EPOLLRDHUP)) | (c->out_off < c->out.size() ? (uint32_t)EPOLLOUT : 0u);
  if (m != c->mask) {
    epoll_event ev{};
    ev.events = m;
    ev.data.fd = c->fd;
    epoll_ctl(io->ep, EPOLL_CTL_MOD, c->fd, &ev);
    c->mask = m;
  }
}

// write what is queued; returns false if the connection was closed
bool flush(IoThread* io, Conn* c) {
  while (c->out_off < c->out.size()) {
    ssize_t w = send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off, MSG_NOSIGNAL);
    if (w > 0) {
      c->out_off += (size_t)w;
      continue;
    }
    if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    if (w < 0 && errno == EINTR) continue;
    close_conn(io, c);
    return false;
  }
  if (c->out_off == c->out.size()) {
    c->out.clear();
    c->out_off = 0;
    if (c->closing && c->ready.empty() && c->next_send == c->next_seq) {
      close_conn(io, c);
      return false;
    }
  } else if (c->out_off > (1u << 20)) {
    c->out.erase(0, c->out_off);
    c->out_off = 0;
  }
  update_mask(io, c);
  return true;
}

// queue response `seq` of `c` (in order); returns false if the connection was closed
bool deliver(IoThread* io, Conn* c, uint64_t seq, std::string bytes, bool close_after) {
  if (seq != c->next_send) {
    c->ready.emplace(seq, std::make_pair(std::move(bytes), close_after));
    return true;
  }
  c->out += bytes;
  c->next_send++;
  if (close_after) c->closing = true;
  for (auto it = c->ready.begin(); it != c->ready.end() && it->first == c->next_send;) {
    c->out += it->second.first;
    if (it->second.second) c->closing = true;
    c->next_send++;
    it = c->ready.erase(it);
  }
  return flush(io, c);
}

bool ieq(const char* a, size_t n, const char* b) {
  if (strlen(b) != n) return false;
  for (size_t i = 0; i < n; ++i) {
    char x = a[i], y = b[i];
    if (x >= 'A' && x <= 'Z') x = (char)(x - 'A' + 'a');
    if (x != y) return false;
  }
  return true;
}

// `.npy` (format 1.x-3.x) uint8 C-order array of >= 2 dims: fills the shape of ONE image (dims 1..),
// the image count and the data offset; false for anything else (the generic Python route serves it)
bool parse_npy_u8(const char* b, long long n, long long* count, long long* shape, int* ndim, long long* data_off) {
  if (n < 12 || memcmp(b, "\x93NUMPY", 6) != 0) return false;
  const int major = (unsigned char)b[6];
  long long hl, h0;
  if (major == 1) {
    hl = (unsigned char)b[8] | ((unsigned char)b[9] << 8);
    h0 = 10;
  } else if (major == 2 || major == 3) {
    hl = (long long)(unsigned char)b[8] | ((long long)(unsigned char)b[9] << 8) |
         ((long long)(unsigned char)b[10] << 16) | ((long long)(unsigned char)b[11] << 24);
    h0 = 12;
  } else {
    return false;
  }
  if (h0 + hl > n) return false;
  std::string_view hd(b + h0, (size_t)hl);
  auto value_of = [&](const char* key) -> std::string_view {
    size_t k = hd.find(key);
    if (k == std::string_view::npos) return {};
    size_t c = hd.find(':', k);
    if (c == std::string_view::npos) return {};
    size_t v = c + 1;
    while (v < hd.size() && hd[v] == ' ') ++v;
    return hd.substr(v);
  };
  std::string_view d = value_of("'descr'"), f = value_of("'fortran_order'"), sh = value_of("'shape'");
  if (!(d.substr(0, 5) == "'|u1'" || d.substr(0, 5) == "'<u1'") || f.substr(0, 5) != "False" || sh.empty() ||
      sh[0] != '(')
    return false;
  long long dims[9];
  int nd = 0;
  size_t i = 1;
  while (i < sh.size() && sh[i] != ')') {
    while (i < sh.size() && (sh[i] == ' ' || sh[i] == ',')) ++i;
    if (i < sh.size() && sh[i] == ')') break;
    long long v = 0;
    bool any = false;
    while (i < sh.size() && sh[i] >= '0' && sh[i] <= '9') {
      v = v * 10 + (sh[i++] - '0');
      any = true;
      if (v > (1ll << 40)) return false;
    }
    if (!any || nd == 9) return false;
    dims[nd++] = v;
  }
  if (nd < 2 || nd > 9) return false;
  // every product is checked BEFORE it is formed (dims <= 2^40, so a later multiply could wrap int64)
  constexpr long long kMaxBytes = 1ll << 40;
  long long per = 1;
  for (int k = 1; k < nd; ++k) {
    if (dims[k] <= 0 || dims[k] > kMaxBytes / per) return false;
    per *= dims[k];
  }
  const long long body = n - h0 - hl;
  if (dims[0] <= 0 || body <= 0 || dims[0] > kMaxBytes / per || dims[0] * per != body) return false;
  *count = dims[0];
  *ndim = nd - 1;
  for (int k = 1; k < nd; ++k) shape[k - 1] = dims[k];
  *data_off = h0 + hl;
  return true;
}

// .npy float32 [n][ncls] (format 1.0, header padded to a 64-byte boundary)
std::string npy_f32(const float* v, long long n, long long ncls) {
  std::string hd = "{'descr': '<f4', 'fortran_order': False, 'shape': (" + std::to_string(n) + ", " +
                   std::to_string(ncls) + "), }";
  const size_t total = (10 + hd.size() + 1 + 63) / 64 * 64;
  hd.append(total - 10 - hd.size() - 1, ' ');
  hd += '\n';
  std::string o("\x93NUMPY\x01\x00", 8);
  o += (char)(hd.size() & 255);
  o += (char)(hd.size() >> 8);
  o += hd;
  o.append((const char*)v, (size_t)(n * ncls) * sizeof(float));
  return o;
}

// parse + dispatch every complete request in c->in; returns false if the connection was closed
bool process(IoThread* io, Conn* c) {
  Server* s = io->srv;
  size_t off = 0;
  bool ok = true;
  while (ok && !c->closing) {
    size_t hend = c->in.find("\r\n\r\n", off);
    if (hend == std::string::npos) {
      if (c->in.size() - off > kMaxHeader) {
        ok = deliver(io, c, c->next_seq++, http_response(400, "text/plain", "", 0, true), true);
      }
      break;
    }
    const char* h = c->in.data() + off;
    size_t hlen = hend - off;
    // request line
    const char* le = (const char*)memchr(h, '\r', hlen);
    size_t llen = le ? (size_t)(le - h) : hlen;
    const char* sp1 = (const char*)memchr(h, ' ', llen);
    const char* sp2 = sp1 ? (const char*)memchr(sp1 + 1, ' ', llen - (size_t)(sp1 + 1 - h)) : nullptr;
    if (!sp1 || !sp2) {
      ok = deliver(io, c, c->next_seq++, http_response(400, "text/plain", "", 0, true), true);
      break;
    }
    std::string method(h, (size_t)(sp1 - h)), path(sp1 + 1, (size_t)(sp2 - sp1 - 1));
    bool http10 = (size_t)(h + llen - (sp2 + 1)) == 8 && !memcmp(sp2 + 1, "HTTP/1.0", 8);
    size_t qm = path.find('?');
    if (qm != std::string::npos) path.resize(qm);
    // headers
    long long clen = 0;
    bool close_req = http10, chunked = false, bad_len = false;
    const char* p = le ? le + 2 : h + hlen;
    const char* e = h + hlen;
    while (p < e) {
      const char* eol = (const char*)memchr(p, '\r', (size_t)(e - p));
      if (!eol) eol = e;
      const char* colon = (const char*)memchr(p, ':', (size_t)(eol - p));
      if (colon) {
        const char* v = colon + 1;
        while (v < eol && (*v == ' ' || *v == '\t')) ++v;
        size_t vn = (size_t)(eol - v);
        size_t kn = (size_t)(colon - p);
        if (ieq(p, kn, "content-length")) {
          const char* ve = eol;
          while (ve > v && (ve[-1] == ' ' || ve[-1] == '\t')) --ve;
          clen = 0;
          bad_len = ve == v;
          for (const char* d = v; d < ve; ++d) {
            if (*d < '0' || *d > '9') {
              bad_len = true;
              break;
            }
            if (clen <= s->max_body) clen = clen * 10 + (*d - '0');
          }
          if (clen > s->max_body) clen = s->max_body + 1;
        } else if (ieq(p, kn, "connection")) {
          if (ieq(v, vn, "close")) close_req = true;
          if (ieq(v, vn, "keep-alive")) close_req = false;
        } else if (ieq(p, kn, "transfer-encoding")) {
          chunked = true;
        }
      }
      p = eol + 2;
    }
    if (chunked || bad_len) {
      ok = deliver(io, c, c->next_seq++, http_response(400, "text/plain", "", 0, true), true);
      break;
    }
    if (clen > s->max_body) {
      ok = deliver(io, c, c->next_seq++, http_response(413, "text/plain", "", 0, true), true);
      break;
    }
    size_t bstart = hend + 4;
    if (c->in.size() < bstart + (size_t)clen) break;  // body incomplete
    const char* body = c->in.data() + bstart;
    uint64_t seq = c->next_seq++;
    off = bstart + (size_t)clen;
    s->requests++;
    Ticket t{c->id, io->idx, seq, close_req};
    if (method == "GET" && path == "/") {
      static const char kUp[] = "Rafiki Predictor is up.";
      ok = deliver(io, c, seq, http_response(200, "text/html; charset=utf-8", kUp, sizeof(kUp) - 1, close_req),
                   close_req);
      continue;
    }
    if (s->batching && method == "POST" && path == "/predict") {
      Item it;
      it.data.resize((size_t)clen);
      long long n = clen > 0 ? rt_json_u8_array(body, clen, "query", it.data.data(), clen, it.shape, &it.ndim) : -1;
      if (n > 0 && n <= s->max_query) {   // oversized queries take the generic path (bounded batch buffers)
        it.data.resize((size_t)n);
        it.conn = c->id;
        it.io = io->idx;
        it.seq = seq;
        it.close = close_req;
        it.npy = false;
        it.count = 1;
        {
          std::lock_guard<std::mutex> g(s->qmu);
          s->items.push_back(std::move(it));
        }
        s->qcv.notify_one();
        if (close_req) c->closing = true;  // stop parsing; close after this response
        continue;
      }
    }
    // an .npy uint8 image batch joins the image queue whole (one batch thread, one graph replay, one
    // .npy response); batches beyond max_batch images or max_query bytes per image go to Python
    long long cnt = 0, doff = 0;
    Item nit;
    if (s->batching && method == "POST" && path == "/predict_batch_npy" &&
        parse_npy_u8(body, clen, &cnt, nit.shape, &nit.ndim, &doff) && cnt <= s->max_batch &&
        (clen - doff) / cnt <= s->max_query && clen - doff <= kMaxNpyBatch) {
      nit.data.assign((const uint8_t*)body + doff, (const uint8_t*)body + clen);
      nit.conn = c->id;
      nit.io = io->idx;
      nit.seq = seq;
      nit.close = close_req;
      nit.npy = true;
      nit.count = cnt;
      {
        std::lock_guard<std::mutex> g(s->qmu);
        s->items.push_back(std::move(nit));
      }
      s->qcv.notify_one();
      if (close_req) c->closing = true;
      continue;
    }
    Generic g{t, method, path, std::string(body, (size_t)clen)};
    uint64_t gid = s->next_id++;
    {
      std::lock_guard<std::mutex> lk(s->qmu);
      s->generic.emplace_back(gid, std::move(g));
    }
    s->ngeneric++;
    s->gcv.notify_one();
    if (close_req) c->closing = true;
  }
  if (!ok) return false;  // the connection is gone
  if (off > 0) c->in.erase(0, off);
  update_mask(io, c);
  return true;
}

void io_loop(IoThread* io) {
  Server* s = io->srv;
  std::vector<epoll_event> evs(256);
  std::vector<char> buf(1 << 16);
  while (!s->stop.load()) {
    int n = epoll_wait(io->ep, evs.data(), (int)evs.size(), 100);
    for (int i = 0; i < n; ++i) {
      int fd = evs[i].data.fd;
      if (fd == io->evfd) {
        uint64_t v;
        ssize_t r = read(io->evfd, &v, sizeof(v));
        (void)r;
        std::vector<int> fds;
        std::vector<Outgoing> mail;
        {
          std::lock_guard<std::mutex> g(io->mu);
          fds.swap(io->new_fds);
          mail.swap(io->mailbox);
        }
        for (int nfd : fds) {
          Conn* c = new Conn();
          c->fd = nfd;
          c->id = s->next_conn++;
          io->conns[c->id] = c;
          io->by_fd[nfd] = c;
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLRDHUP;
          ev.data.fd = nfd;
          epoll_ctl(io->ep, EPOLL_CTL_ADD, nfd, &ev);
        }
        for (auto& m : mail) {
          auto it = io->conns.find(m.conn);
          if (it == io->conns.end()) continue;  // the client went away
          deliver(io, it->second, m.seq, std::move(m.bytes), m.close);
        }
        continue;
      }
      auto it = io->by_fd.find(fd);
      if (it == io->by_fd.end()) continue;
      Conn* c = it->second;
      if (evs[i].events & EPOLLOUT) {
        if (!flush(io, c)) continue;
      }
      if (evs[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
        bool eof = false;
        while (true) {
          ssize_t r = recv(fd, buf.data(), buf.size(), 0);
          if (r > 0) {
            c->in.append(buf.data(), (size_t)r);
            if (c->in.size() > (size_t)s->max_body + kMaxHeader + 4) break;
            continue;
          }
          if (r == 0) eof = true;
          else if (errno == EINTR) continue;
          else if (errno != EAGAIN && errno != EWOULDBLOCK) eof = true;
          break;
        }
        if (!c->in.empty() && !c->closing) {
          if (!process(io, c)) continue;
        }
        if (eof) {
          if (c->next_send == c->next_seq && c->out_off == c->out.size()) {
            close_conn(io, c);
          } else {
            c->closing = true;  // answer what was asked, then close
            update_mask(io, c);
          }
        }
      }
    }
  }
  for (auto& kv : io->conns) {
    close(kv.second->fd);
    delete kv.second;
  }
  io->conns.clear();
  io->by_fd.clear();
}

void accept_loop(Server* s) {
  size_t rr = 0;
  while (!s->stop.load()) {
    pollfd pf{s->lfd, POLLIN, 0};
    int r = poll(&pf, 1, 100);
    if (r <= 0) continue;
    while (true) {
      int fd = accept4(s->lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) break;
      if ((size_t)s->nconns.load() >= kMaxConns) {
        close(fd);
        continue;
      }
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      s->nconns++;
      s->accepted++;
      IoThread* io = s->io[rr++ % s->io.size()].get();
      {
        std::lock_guard<std::mutex> g(io->mu);
        io->new_fds.push_back(fd);
      }
      uint64_t v = 1;
      ssize_t w = write(io->evfd, &v, sizeof(v));
      (void)w;
    }
  }
}

void append_double(std::string& o, double v) {
  char b[32];
  if (v != v) {
    o += "NaN";
    return;
  }
  if (v == __builtin_inf() || v == -__builtin_inf()) {
    o += v > 0 ? "Infinity" : "-Infinity";
    return;
  }
  auto res = std::to_chars(b, b + sizeof(b), v);
  std::string_view sv(b, (size_t)(res.ptr - b));
  o.append(sv);
  // Python's repr keeps a ".0" on integral values and writes exponents as e-05 / e+20
  bool has = sv.find_first_of(".eEn") != std::string_view::npos;
  if (!has) o += ".0";
}

}  // namespace

extern "C" {

void* rt_http_start(const char* host, int port, int io_threads, long long max_batch, long long max_body,
                    int batching) {
  auto* s = new Server();
  s->max_batch = max_batch > 0 ? max_batch : 512;
  s->max_body = max_body > 0 ? max_body : (256 << 20);
  s->batching = batching != 0;
  s->lfd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  int one = 1;
  setsockopt(s->lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host && *host ? host : "0.0.0.0", &a.sin_addr) != 1 ||
      bind(s->lfd, (sockaddr*)&a, sizeof(a)) != 0 || listen(s->lfd, 1024) != 0) {
    close(s->lfd);
    delete s;
    return nullptr;
  }
  fcntl(s->lfd, F_SETFL, fcntl(s->lfd, F_GETFL) | O_NONBLOCK);
  int n = io_threads > 0 ? io_threads : 2;
  for (int i = 0; i < n; ++i) {
    auto io = std::make_unique<IoThread>();
    io->srv = s;
    io->idx = i;
    io->ep = epoll_create1(EPOLL_CLOEXEC);
    io->evfd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = io->evfd;
    epoll_ctl(io->ep, EPOLL_CTL_ADD, io->evfd, &ev);
    s->io.push_back(std::move(io));
  }
  for (auto& io : s->io) io->th = std::thread(io_loop, io.get());
  s->acceptor = std::thread(accept_loop, s);
  return s;
}

int rt_http_port(void* h) {
  auto* s = (Server*)h;
  sockaddr_in a{};
  socklen_t n = sizeof(a);
  if (getsockname(s->lfd, (sockaddr*)&a, &n) != 0) return -1;
  return ntohs(a.sin_port);
}

// Largest single image query (bytes) the batch path accepts; larger ones are served by the generic path.
void rt_http_set_max_query(void* h, long long bytes) {
  auto* s = (Server*)h;
  std::lock_guard<std::mutex> g(s->qmu);
  s->max_query = bytes > 0 ? bytes : (1 << 20);
}

// Blocks up to timeout_ms for pending image requests; takes every pending request whose images have
// the first one's shape (<= max_batch images, <= cap bytes; an .npy request's images stay together)
// into `out`.  Returns the image count (0: timeout, -1: stopped, -3: `out` cannot hold the first
// request); `shape`/`ndim` describe ONE image, `batch_id` identifies the batch for completion.
long long rt_http_next_batch(void* h, int timeout_ms, uint8_t* out, long long cap, long long* shape, int* ndim,
                             unsigned long long* batch_id) {
  auto* s = (Server*)h;
  std::unique_lock<std::mutex> lk(s->qmu);
  if (!s->qcv.wait_for(lk, std::chrono::milliseconds(timeout_ms),
                       [s] { return s->stop.load() || !s->items.empty(); }))
    return 0;
  if (s->stop.load()) return -1;
  const Item& first = s->items.front();
  int nd = first.ndim;
  long long sh[8];
  memcpy(sh, first.shape, sizeof(sh));
  size_t per = first.data.size() / (size_t)first.count;   // bytes of one image
  std::vector<Ticket> tickets;
  std::deque<Item> rest;
  long long n = 0;
  while (!s->items.empty()) {
    Item it = std::move(s->items.front());
    s->items.pop_front();
    bool same = it.ndim == nd && it.data.size() == per * (size_t)it.count &&
                !memcmp(it.shape, sh, sizeof(long long) * (size_t)nd);
    // a request's images stay together; the first request of a batch may alone exceed max_batch
    if (same && (n == 0 || n + it.count <= s->max_batch) && (long long)((n + it.count) * per) <= cap) {
      memcpy(out + n * per, it.data.data(), it.data.size());
      tickets.push_back(Ticket{it.conn, it.io, it.seq, it.close, it.npy, it.count});
      n += it.count;
    } else {
      rest.push_back(std::move(it));
    }
  }
  s->items.swap(rest);
  if (n == 0) {  // the first request exceeds the caller's buffer: report its shape, the caller grows the buffer
    *ndim = nd;
    for (int i = 0; i < nd; ++i) shape[i] = sh[i];
    return -3;
  }
  uint64_t bid = s->next_id++;
  s->batches.emplace(bid, std::move(tickets));
  lk.unlock();
  *ndim = nd;
  for (int i = 0; i < nd; ++i) shape[i] = sh[i];
  *batch_id = bid;
  s->nbatches++;
  s->batched += n;
  return n;
}

// `{"prediction": [...]}` per query of batch `batch_id` from probs [n, ncls] (float32).
int rt_http_complete(void* h, unsigned long long batch_id, const float* probs, long long n, long long ncls) {
  auto* s = (Server*)h;
  std::vector<Ticket> tickets;
  {
    std::lock_guard<std::mutex> g(s->qmu);
    auto it = s->batches.find(batch_id);
    if (it == s->batches.end()) return -1;
    tickets.swap(it->second);
    s->batches.erase(it);
  }
  long long total = 0;
  for (auto& t : tickets) total += t.count;
  if (total != n) return -2;
  std::string body;
  long long i = 0;
  for (const Ticket& t : tickets) {
    if (t.npy) {
      body = npy_f32(probs + i * ncls, t.count, ncls);
      post(s, t, http_response(200, "application/octet-stream", body.data(), body.size(), t.close));
      i += t.count;
      continue;
    }
    body.clear();
    body += "{\"prediction\": [";
    for (long long j = 0; j < ncls; ++j) {
      if (j) body += ", ";
      append_double(body, (double)probs[i * ncls + j]);
    }
    body += "]}";
    post(s, t, http_response(200, "application/json", body.data(), body.size(), t.close));
    ++i;
  }
  return 0;
}

int rt_http_fail(void* h, unsigned long long batch_id, const char* msg) {
  auto* s = (Server*)h;
  std::vector<Ticket> tickets;
  {
    std::lock_guard<std::mutex> g(s->qmu);
    auto it = s->batches.find(batch_id);
    if (it == s->batches.end()) return -1;
    tickets.swap(it->second);
    s->batches.erase(it);
  }
  for (auto& t : tickets) s->errors += t.count;
  size_t n = strlen(msg);
  for (auto& t : tickets) post(s, t, http_response(500, "text/plain", msg, n, t.close));
  return 0;
}

// Generic requests: blocks up to timeout_ms; returns the body length (>= 0) and fills id, method and
// path (NUL-terminated, truncated to their capacities), or -1 on timeout, -2 when stopped.
long long rt_http_next_request(void* h, int timeout_ms, unsigned long long* id, char* method, int mcap, char* path,
                               int pcap) {
  auto* s = (Server*)h;
  std::unique_lock<std::mutex> lk(s->qmu);
  if (!s->gcv.wait_for(lk, std::chrono::milliseconds(timeout_ms),
                       [s] { return s->stop.load() || !s->generic.empty(); }))
    return -1;
  if (s->stop.load()) return -2;
  auto entry = std::move(s->generic.front());
  s->generic.pop_front();
  *id = entry.first;
  snprintf(method, (size_t)mcap, "%s", entry.second.method.c_str());
  snprintf(path, (size_t)pcap, "%s", entry.second.path.c_str());
  long long n = (long long)entry.second.body.size();
  s->taken.emplace(entry.first, std::move(entry.second));
  return n;
}

int rt_http_request_body(void* h, unsigned long long id, char* dst) {
  auto* s = (Server*)h;
  std::lock_guard<std::mutex> g(s->qmu);
  auto it = s->taken.find(id);
  if (it == s->taken.end()) return -1;
  memcpy(dst, it->second.body.data(), it->second.body.size());
  return 0;
}

int rt_http_respond(void* h, unsigned long long id, int status, const char* ctype, const char* body, long long n) {
  auto* s = (Server*)h;
  Ticket t;
  {
    std::lock_guard<std::mutex> g(s->qmu);
    auto it = s->taken.find(id);
    if (it == s->taken.end()) return -1;
    t = it->second.t;
    s->taken.erase(it);
  }
  if (status >= 500) s->errors++;
  post(s, t, http_response(status, ctype, body, (size_t)n, t.close));
  return 0;
}

// requests, batches, batched queries, generic requests, errors, accepted connections, open connections,
// queued image queries
void rt_http_stats(void* h, long long* out) {
  auto* s = (Server*)h;
  out[0] = s->requests.load();
  out[1] = s->nbatches.load();
  out[2] = s->batched.load();
  out[3] = s->ngeneric.load();
  out[4] = s->errors.load();
  out[5] = s->accepted.load();
  out[6] = s->nconns.load();
  std::lock_guard<std::mutex> g(s->qmu);
  out[7] = (long long)s->items.size();
}

// Wakes every caller blocked in rt_http_next_batch / rt_http_next_request (they return "stopped");
// call it, join those callers, then rt_http_stop.
void rt_http_shutdown(void* h) {
  auto* s = (Server*)h;
  {
    std::lock_guard<std::mutex> g(s->qmu);
    s->stop.store(true);
  }
  s->qcv.notify_all();
  s->gcv.notify_all();
}

// Joins the server's threads, closes every connection and frees the server.
void rt_http_stop(void* h) {
  auto* s = (Server*)h;
  rt_http_shutdown(h);
  if (s->acceptor.joinable()) s->acceptor.join();
  for (auto& io : s->io) {
    uint64_t v = 1;
    ssize_t w = write(io->evfd, &v, sizeof(v));
    (void)w;
  }
  for (auto& io : s->io)
    if (io->th.joinable()) io->th.join();
  for (auto& io : s->io) {
    close(io->ep);
    close(io->evfd);
  }
  close(s->lfd);
  delete s;
}

}  // extern "C"
