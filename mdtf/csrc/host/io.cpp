// Host-side native I/O for mdtf (C ABI, loaded with ctypes).
//
// * CRC32C (Castagnoli) with the SSE4.2 crc32 instruction over 8-byte words, plus TF's "masked" CRC used by TFRecord framing and
//   tensor-bundle entries (reference: TF's queue/reader/Saver C++ runtime that
//   distribute_input.py:92-106 and distribute_train.py:171 rely on).
// * TFRecord reader: length(u64) | masked_crc(length)(u32) | data | masked_crc(data)(u32).
// * Threaded shuffling record loader: N reader threads stream records from a
//   file list into a bounded shuffle buffer; the trainer pulls records (or
//   whole batches) without touching the GIL-held Python parser.
//
// Built by mdtf/csrc/build.py:  g++ -O3 -msse4.2 -shared -fPIC -pthread
#include <nmmintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace {

inline uint32_t crc32c_sw_byte(uint32_t crc, uint8_t b) {
  crc ^= b;
  for (int k = 0; k < 8; ++k) crc = (crc >> 1) ^ (0x82F63B78u & (0u - (crc & 1u)));
  return crc;
}

uint32_t crc32c_extend(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = crc ^ 0xFFFFFFFFu;
  // align to 8 bytes
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    c = _mm_crc32_u8(static_cast<uint32_t>(c), *p++);
    --n;
  }
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    c = _mm_crc32_u64(c, w);
    p += 8;
    n -= 8;
  }
  while (n--) c = _mm_crc32_u8(static_cast<uint32_t>(c), *p++);
  return static_cast<uint32_t>(c) ^ 0xFFFFFFFFu;
}

const uint32_t kMaskDelta = 0xa282ead8u;
inline uint32_t mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + kMaskDelta; }

struct RecordReader {
  FILE* f = nullptr;
  std::vector<char> buf;
  bool verify = true;
};

// return: >=0 record length (data in r->buf), -1 EOF, -2 corrupt header, -3 corrupt data
long long read_record(RecordReader* r) {
  uint8_t hdr[12];
  size_t got = fread(hdr, 1, 12, r->f);
  if (got == 0) return -1;
  if (got != 12) return -2;
  uint64_t len;
  memcpy(&len, hdr, 8);
  uint32_t hcrc;
  memcpy(&hcrc, hdr + 8, 4);
  if (r->verify && mask(crc32c_extend(0, hdr, 8)) != hcrc) return -2;
  if (len > (1ull << 34)) return -2;
  r->buf.resize(len + 4);
  if (fread(r->buf.data(), 1, len + 4, r->f) != len + 4) return -3;
  uint32_t dcrc;
  memcpy(&dcrc, r->buf.data() + len, 4);
  if (r->verify && mask(crc32c_extend(0, reinterpret_cast<uint8_t*>(r->buf.data()), len)) != dcrc) return -3;
  return static_cast<long long>(len);
}

// ---------------------------------------------------------------------------
struct Loader {
  std::vector<std::string> files;
  size_t capacity;
  int epochs;  // <=0: forever
  bool shuffle;
  std::mt19937_64 rng;
  std::mutex mu;
  std::condition_variable not_full, not_empty;
  std::vector<std::string> pool;  // shuffle buffer
  std::deque<std::string> fifo;   // non-shuffled
  std::vector<std::thread> threads;
  std::atomic<int> active{0};
  std::atomic<bool> stop{false};
  std::atomic<long long> errors{0};
  size_t min_after_dequeue;
  std::atomic<size_t> next_file{0};
  size_t total_files_to_read;

  size_t size_locked() const { return shuffle ? pool.size() : fifo.size(); }
};

void loader_worker(Loader* L) {
  for (;;) {
    size_t idx = L->next_file.fetch_add(1);
    if (L->stop.load() || (L->total_files_to_read && idx >= L->total_files_to_read)) break;
    const std::string& path = L->files[idx % L->files.size()];
    RecordReader r;
    r.f = fopen(path.c_str(), "rb");
    if (!r.f) {
      L->errors++;
      continue;
    }
    for (;;) {
      long long n = read_record(&r);
      if (n == -1) break;
      if (n < 0) {
        L->errors++;
        break;
      }
      std::string rec(r.buf.data(), static_cast<size_t>(n));
      std::unique_lock<std::mutex> lk(L->mu);
      L->not_full.wait(lk, [&] { return L->stop.load() || L->size_locked() < L->capacity; });
      if (L->stop.load()) break;
      if (L->shuffle)
        L->pool.emplace_back(std::move(rec));
      else
        L->fifo.emplace_back(std::move(rec));
      lk.unlock();
      L->not_empty.notify_one();
    }
    fclose(r.f);
    if (L->stop.load()) break;
  }
  L->active--;
  L->not_empty.notify_all();
}

}  // namespace

extern "C" {

uint32_t mdtf_crc32c(const void* data, size_t n, uint32_t init) {
  return crc32c_extend(init, static_cast<const uint8_t*>(data), n);
}

uint32_t mdtf_masked_crc32c(const void* data, size_t n) {
  return mask(crc32c_extend(0, static_cast<const uint8_t*>(data), n));
}

uint32_t mdtf_crc32c_sw(const void* data, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  const uint8_t* p = static_cast<const uint8_t*>(data);
  for (size_t i = 0; i < n; ++i) c = crc32c_sw_byte(c, p[i]);
  return c ^ 0xFFFFFFFFu;
}

// -- single-file record reader ----------------------------------------------
void* mdtf_tfr_open(const char* path, int verify) {
  FILE* f = fopen(path, "rb");
  if (!f) return nullptr;
  RecordReader* r = new RecordReader();
  r->f = f;
  r->verify = verify != 0;
  return r;
}

long long mdtf_tfr_next(void* h, const char** data) {
  RecordReader* r = static_cast<RecordReader*>(h);
  long long n = read_record(r);
  if (n >= 0) *data = r->buf.data();
  return n;
}

void mdtf_tfr_close(void* h) {
  RecordReader* r = static_cast<RecordReader*>(h);
  if (r->f) fclose(r->f);
  delete r;
}

// write one framed record to an open FILE* owned by the writer handle
void* mdtf_tfw_open(const char* path) { return fopen(path, "wb"); }

int mdtf_tfw_write(void* h, const void* data, unsigned long long n) {
  FILE* f = static_cast<FILE*>(h);
  uint8_t hdr[12];
  memcpy(hdr, &n, 8);
  uint32_t c = mask(crc32c_extend(0, hdr, 8));
  memcpy(hdr + 8, &c, 4);
  uint32_t dc = mask(crc32c_extend(0, static_cast<const uint8_t*>(data), n));
  if (fwrite(hdr, 1, 12, f) != 12) return -1;
  if (n && fwrite(data, 1, n, f) != n) return -1;
  if (fwrite(&dc, 1, 4, f) != 4) return -1;
  return 0;
}

int mdtf_tfw_close(void* h) { return fclose(static_cast<FILE*>(h)); }

// -- threaded shuffling loader ------------------------------------------------
void* mdtf_loader_create(const char** paths, int nfiles, int epochs, int shuffle, unsigned long long capacity,
                         unsigned long long min_after_dequeue, unsigned long long seed, int nthreads) {
  if (nfiles <= 0) return nullptr;
  Loader* L = new Loader();
  for (int i = 0; i < nfiles; ++i) L->files.emplace_back(paths[i]);
  L->epochs = epochs;
  L->shuffle = shuffle != 0;
  L->capacity = capacity ? capacity : 1024;
  L->min_after_dequeue = min_after_dequeue < L->capacity ? min_after_dequeue : L->capacity - 1;
  L->rng.seed(seed);
  L->total_files_to_read = epochs > 0 ? static_cast<size_t>(epochs) * L->files.size() : 0;
  if (nthreads < 1) nthreads = 1;
  L->active = nthreads;
  for (int t = 0; t < nthreads; ++t) L->threads.emplace_back(loader_worker, L);
  return L;
}

// Copies the next record into buf (cap bytes). Returns length, -1 at end of
// data, or -(needed+16) when buf is too small (record is kept).
long long mdtf_loader_next(void* h, char* buf, unsigned long long cap) {
  Loader* L = static_cast<Loader*>(h);
  std::unique_lock<std::mutex> lk(L->mu);
  L->not_empty.wait(lk, [&] {
    size_t s = L->size_locked();
    bool producers_done = L->active.load() == 0;
    return L->stop.load() || (s > 0 && (s > L->min_after_dequeue || producers_done)) || (s == 0 && producers_done);
  });
  size_t s = L->size_locked();
  if (s == 0) return -1;
  std::string* rec;
  size_t pick = 0;
  if (L->shuffle) {
    pick = std::uniform_int_distribution<size_t>(0, s - 1)(L->rng);
    rec = &L->pool[pick];
  } else {
    rec = &L->fifo.front();
  }
  if (rec->size() > cap) return -static_cast<long long>(rec->size() + 16);
  long long n = static_cast<long long>(rec->size());
  memcpy(buf, rec->data(), rec->size());
  if (L->shuffle) {
    std::swap(L->pool[pick], L->pool.back());
    L->pool.pop_back();
  } else {
    L->fifo.pop_front();
  }
  lk.unlock();
  L->not_full.notify_one();
  return n;
}

long long mdtf_loader_errors(void* h) { return static_cast<Loader*>(h)->errors.load(); }

void mdtf_loader_destroy(void* h) {
  Loader* L = static_cast<Loader*>(h);
  L->stop = true;
  L->not_full.notify_all();
  L->not_empty.notify_all();
  for (auto& t : L->threads) t.join();
  delete L;
}

}  // extern "C"
