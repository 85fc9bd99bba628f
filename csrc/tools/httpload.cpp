// Minimal closed-loop HTTP/1.1 load generator for the predictor benchmarks (scripts/bench_predictor.py).
// C connections, each with exactly one request in flight (send, wait for the full response, repeat),
// spread over T epoll threads.  A Python client spends ~50 us of GIL-bound work per request and, on a
// 16-CPU share, measures itself; this costs a few microseconds per request.
//
// usage: httpload <host> <port> <path> <body-file> <connections> <threads> <seconds>
// prints one JSON line: {"requests", "qps", "p50_ms", "p99_ms", "errors"}
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;

struct Conn {
  int fd = -1;
  std::string in;
  size_t sent = 0;
  Clock::time_point t0;
};

struct Result {
  long long requests = 0, errors = 0;
  std::vector<float> lat_ms;
};

std::atomic<bool> g_stop{false};

int connect_to(const char* host, int port) {
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  inet_pton(AF_INET, host, &a.sin_addr);
  if (connect(fd, (sockaddr*)&a, sizeof(a)) != 0) {
    close(fd);
    return -1;
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  return fd;
}

// length of one complete response at the front of `in`, 0 if incomplete, -1 if malformed
long long complete_response(const std::string& in, bool* ok) {
  size_t h = in.find("\r\n\r\n");
  if (h == std::string::npos) return 0;
  *ok = in.compare(0, 12, "HTTP/1.1 200") == 0;
  size_t p = 0;
  long long cl = -1;
  while (p < h) {
    size_t e = in.find("\r\n", p);
    if (e == std::string::npos || e > h) e = h;
    if (e - p > 15 && strncasecmp(in.data() + p, "content-length:", 15) == 0) cl = atoll(in.data() + p + 15);
    p = e + 2;
  }
  if (cl < 0) return -1;
  return in.size() >= h + 4 + (size_t)cl ? (long long)(h + 4 + cl) : 0;
}

void worker(const char* host, int port, const std::string* req, int nconn, Result* res) {
  int ep = epoll_create1(0);
  std::vector<Conn> conns((size_t)nconn);
  for (int i = 0; i < nconn; ++i) {
    conns[i].fd = connect_to(host, port);
    if (conns[i].fd < 0) {
      res->errors++;
      continue;
    }
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u32 = (uint32_t)i;
    epoll_ctl(ep, EPOLL_CTL_ADD, conns[i].fd, &ev);
    conns[i].t0 = Clock::now();
    send(conns[i].fd, req->data(), req->size(), MSG_NOSIGNAL);
  }
  std::vector<epoll_event> evs(256);
  char buf[1 << 16];
  while (!g_stop.load()) {
    int n = epoll_wait(ep, evs.data(), (int)evs.size(), 50);
    for (int k = 0; k < n; ++k) {
      Conn& c = conns[evs[k].data.u32];
      ssize_t r = recv(c.fd, buf, sizeof(buf), 0);
      if (r <= 0) {
        res->errors++;
        epoll_ctl(ep, EPOLL_CTL_DEL, c.fd, nullptr);
        close(c.fd);
        c.fd = -1;
        continue;
      }
      c.in.append(buf, (size_t)r);
      bool ok = false;
      long long len;
      while ((len = complete_response(c.in, &ok)) > 0) {
        c.in.erase(0, (size_t)len);
        auto now = Clock::now();
        res->lat_ms.push_back(std::chrono::duration<float, std::milli>(now - c.t0).count());
        if (ok) res->requests++;
        else res->errors++;
        if (g_stop.load()) break;
        c.t0 = now;
        send(c.fd, req->data(), req->size(), MSG_NOSIGNAL);
      }
      if (len < 0) res->errors++;
    }
  }
  for (auto& c : conns)
    if (c.fd >= 0) close(c.fd);
  close(ep);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 8) {
    fprintf(stderr, "usage: %s host port path body-file connections threads seconds\n", argv[0]);
    return 2;
  }
  const char* host = argv[1];
  const int port = atoi(argv[2]);
  std::ifstream f(argv[4], std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string body = ss.str();
  const int conns = std::max(1, atoi(argv[5])), threads = std::max(1, std::min(atoi(argv[6]), conns));
  const double seconds = atof(argv[7]);
  std::string req = std::string("POST ") + argv[3] + " HTTP/1.1\r\nHost: x\r\nContent-Length: " +
                    std::to_string(body.size()) + "\r\n\r\n" + body;
  std::vector<Result> res((size_t)threads);
  std::vector<std::thread> th;
  const auto t0 = Clock::now();
  for (int t = 0; t < threads; ++t) {
    int n = conns / threads + (t < conns % threads ? 1 : 0);
    th.emplace_back(worker, host, port, &req, n, &res[(size_t)t]);
  }
  std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
  g_stop.store(true);
  for (auto& t : th) t.join();
  const double el = std::chrono::duration<double>(Clock::now() - t0).count();
  long long n = 0, err = 0;
  std::vector<float> lat;
  for (auto& r : res) {
    n += r.requests;
    err += r.errors;
    lat.insert(lat.end(), r.lat_ms.begin(), r.lat_ms.end());
  }
  std::sort(lat.begin(), lat.end());
  auto pct = [&](double q) { return lat.empty() ? 0.0 : (double)lat[std::min(lat.size() - 1, (size_t)(q * lat.size()))]; };
  printf("{\"requests\": %lld, \"qps\": %.1f, \"p50_ms\": %.3f, \"p99_ms\": %.3f, \"errors\": %lld}\n", n, n / el,
         pct(0.50), pct(0.99), err);
  return 0;
}
