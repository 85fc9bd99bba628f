// Cross-process message queues in POSIX shared memory — the node-local replacement for the
// reference's Redis lists (rafiki/cache/cache.py: RPUSH/LRANGE+LTRIM query and prediction queues
// per inference worker).  One ring buffer of length-prefixed messages per queue, guarded by a
// process-shared ROBUST mutex (a worker that dies holding it cannot wedge the predictor) and two
// process-shared condition variables.  Pop is atomic (fixes the reference's non-atomic
// LRANGE+LTRIM double-delivery and its LTRIM-empties-the-list bug).
//
//   rt_mq_open(name, capacity, create) -> handle | null     rt_mq_close / rt_mq_unlink
//   rt_mq_push(h, data, len, timeout_ms) -> 0 | -1 timeout | -2 too large
//   rt_mq_pop(h, buf, cap, timeout_ms)   -> len | -1 timeout | -(needed) - 16 when buf too small
//   rt_mq_size(h)                        -> messages queued
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>

namespace {

constexpr uint64_t kMagic = 0x52414b494d513031ull;  // "RAKIMQ01"

struct Header {
  uint64_t magic;
  uint64_t capacity;  // data bytes
  uint64_t head;      // read offset
  uint64_t tail;      // write offset
  uint64_t used;      // bytes in use
  uint64_t count;     // messages
  pthread_mutex_t mu;
  pthread_cond_t not_empty;
  pthread_cond_t not_full;
};

struct Queue {
  Header* h;
  uint8_t* data;
  size_t map_bytes;
  std::string name;
};

void deadline(timespec& ts, int timeout_ms) {
  clock_gettime(CLOCK_MONOTONIC, &ts);
  ts.tv_sec += timeout_ms / 1000;
  ts.tv_nsec += (long)(timeout_ms % 1000) * 1000000L;
  if (ts.tv_nsec >= 1000000000L) { ts.tv_sec += 1; ts.tv_nsec -= 1000000000L; }
}

// Copies work on local offsets; the header (tail/used/count on push, head/used/count on pop) is
// published only after the whole frame (4-byte length + payload) is copied.  A process that dies
// mid-copy therefore leaves the previous, consistent header; one that dies between the publishing
// stores is caught by validate() below.
uint64_t ring_copy_in(Queue* q, uint64_t off, const uint8_t* src, uint64_t n) {
  const uint64_t cap = q->h->capacity;
  const uint64_t first = n < cap - off ? n : cap - off;
  memcpy(q->data + off, src, first);
  if (n > first) memcpy(q->data, src + first, n - first);
  return (off + n) % cap;
}

uint64_t ring_copy_out(Queue* q, uint64_t off, uint8_t* dst, uint64_t n) {
  const uint64_t cap = q->h->capacity;
  const uint64_t first = n < cap - off ? n : cap - off;
  memcpy(dst, q->data + off, first);
  if (n > first) memcpy(dst + first, q->data, n - first);
  return (off + n) % cap;
}

// After EOWNERDEAD: the frames from head must account for exactly `count` messages and `used`
// bytes, ending at tail; otherwise the header was torn by the dead owner -> drop the queue's
// contents (lost messages time out at the caller; a corrupt ring would misframe forever).
void validate(Queue* q) {
  Header* h = q->h;
  bool ok = h->head < h->capacity && h->tail < h->capacity && h->used <= h->capacity;
  uint64_t off = h->head, bytes = 0;
  for (uint64_t i = 0; ok && i < h->count; ++i) {
    uint32_t n32;
    off = ring_copy_out(q, off, (uint8_t*)&n32, 4);
    bytes += 4 + (uint64_t)n32;
    if (bytes > h->used) { ok = false; break; }
    off = (off + n32) % h->capacity;
  }
  ok = ok && bytes == h->used && off == (h->used == h->capacity ? h->head : h->tail);
  if (!ok) h->head = h->tail = h->used = h->count = 0;
}

int lock(Queue* q) {
  int rc = pthread_mutex_lock(&q->h->mu);
  if (rc == EOWNERDEAD) {
    validate(q);
    pthread_mutex_consistent(&q->h->mu);
    rc = 0;
  }
  return rc;
}

}  // namespace

extern "C" {

void* rt_mq_open(const char* name, long long capacity, int create) {
  std::string nm = std::string("/") + name;
  const int fd = shm_open(nm.c_str(), create ? (O_CREAT | O_RDWR) : O_RDWR, 0600);
  if (fd < 0) return nullptr;
  struct stat st;
  if (fstat(fd, &st) != 0) { close(fd); return nullptr; }
  size_t bytes = (size_t)st.st_size;
  bool init = false;
  if (bytes == 0) {
    if (!create || capacity <= 0) { close(fd); return nullptr; }
    bytes = sizeof(Header) + (size_t)capacity;
    if (ftruncate(fd, (off_t)bytes) != 0) { close(fd); return nullptr; }
    init = true;
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return nullptr;
  Queue* q = new (std::nothrow) Queue{(Header*)p, (uint8_t*)p + sizeof(Header), bytes, nm};
  if (!q) { munmap(p, bytes); return nullptr; }
  Header* h = q->h;
  if (init) {
    memset(h, 0, sizeof(Header));
    h->capacity = bytes - sizeof(Header);
    pthread_mutexattr_t ma;
    pthread_mutexattr_init(&ma);
    pthread_mutexattr_setpshared(&ma, PTHREAD_PROCESS_SHARED);
    pthread_mutexattr_setrobust(&ma, PTHREAD_MUTEX_ROBUST);
    pthread_mutex_init(&h->mu, &ma);
    pthread_mutexattr_destroy(&ma);
    pthread_condattr_t ca;
    pthread_condattr_init(&ca);
    pthread_condattr_setpshared(&ca, PTHREAD_PROCESS_SHARED);
    pthread_condattr_setclock(&ca, CLOCK_MONOTONIC);
    pthread_cond_init(&h->not_empty, &ca);
    pthread_cond_init(&h->not_full, &ca);
    pthread_condattr_destroy(&ca);
    __atomic_store_n(&h->magic, kMagic, __ATOMIC_RELEASE);
  } else {
    // another process is initialising it: wait (bounded) for the magic word
    for (int i = 0; i < 2000 && __atomic_load_n(&h->magic, __ATOMIC_ACQUIRE) != kMagic; ++i) usleep(1000);
    if (h->magic != kMagic) { munmap(p, bytes); delete q; return nullptr; }
  }
  return q;
}

void rt_mq_close(void* handle) {
  Queue* q = (Queue*)handle;
  if (!q) return;
  munmap(q->h, q->map_bytes);
  delete q;
}

int rt_mq_unlink(const char* name) {
  std::string nm = std::string("/") + name;
  return shm_unlink(nm.c_str());
}

int rt_mq_push(void* handle, const uint8_t* data, long long len, int timeout_ms) {
  Queue* q = (Queue*)handle;
  Header* h = q->h;
  const uint64_t need = 4 + (uint64_t)len;
  if (len < 0 || len > 0xFFFFFFFFll || need > h->capacity) return -2;
  timespec ts;
  deadline(ts, timeout_ms < 0 ? 0 : timeout_ms);
  if (lock(q) != 0) return -3;
  while (h->capacity - h->used < need) {
    if (timeout_ms == 0) { pthread_mutex_unlock(&h->mu); return -1; }
    const int rc = pthread_cond_timedwait(&h->not_full, &h->mu, &ts);
    if (rc == EOWNERDEAD) { validate(q); pthread_mutex_consistent(&h->mu); }
    if (rc == ETIMEDOUT && h->capacity - h->used < need) { pthread_mutex_unlock(&h->mu); return -1; }
  }
  const uint32_t n32 = (uint32_t)len;
  uint64_t off = ring_copy_in(q, h->tail, (const uint8_t*)&n32, 4);
  off = ring_copy_in(q, off, data, (uint64_t)len);
  // publish the complete frame
  h->tail = off;
  h->used += need;
  h->count += 1;
  pthread_cond_signal(&h->not_empty);
  pthread_mutex_unlock(&h->mu);
  return 0;
}

long long rt_mq_pop(void* handle, uint8_t* buf, long long cap, int timeout_ms) {
  Queue* q = (Queue*)handle;
  Header* h = q->h;
  timespec ts;
  deadline(ts, timeout_ms < 0 ? 0 : timeout_ms);
  if (lock(q) != 0) return -3;
  while (h->count == 0) {
    if (timeout_ms == 0) { pthread_mutex_unlock(&h->mu); return -1; }
    const int rc = pthread_cond_timedwait(&h->not_empty, &h->mu, &ts);
    if (rc == EOWNERDEAD) { validate(q); pthread_mutex_consistent(&h->mu); }
    if (rc == ETIMEDOUT && h->count == 0) { pthread_mutex_unlock(&h->mu); return -1; }
  }
  uint32_t n32;
  uint64_t off = ring_copy_out(q, h->head, (uint8_t*)&n32, 4);
  if ((long long)n32 > cap) {  // leave the message queued; tell the caller the size it needs
    pthread_mutex_unlock(&h->mu);
    return -(long long)n32 - 16;
  }
  off = ring_copy_out(q, off, buf, n32);
  // publish the consumed frame
  h->head = off;
  h->used -= 4 + (uint64_t)n32;
  h->count -= 1;
  pthread_cond_signal(&h->not_full);
  pthread_mutex_unlock(&h->mu);
  return (long long)n32;
}

long long rt_mq_size(void* handle) {
  Queue* q = (Queue*)handle;
  if (lock(q) != 0) return -3;
  const long long n = (long long)q->h->count;
  pthread_mutex_unlock(&q->h->mu);
  return n;
}

}  // extern "C"
