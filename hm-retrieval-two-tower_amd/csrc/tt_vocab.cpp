// Host-side vocabulary lookup (StringLookup, num_oov_indices=1): the input
// pipeline's string -> embedding-row encoding.
//
// Reference: /root/reference/pkg/modelling/layers/input_layer.py:33-36 builds
// tf.keras.layers.StringLookup(vocabulary=feature.vocab, num_oov_indices=1)
// and applies it to every batch inside the graph; vocab[i] -> i + 1, anything
// else -> 0.  Here the lookup runs once per dataset on the host (the encoded
// int32 rows then stay resident in HBM, pkg/modelling/dataset.py), so it is
// plain multi-threaded C++ over an Arrow-style string arena (bytes + int64
// offsets) — no Python object per value.
//
// Table: open addressing (linear probing) over a power-of-two slot array of
// (64-bit hash, row); keys are compared byte-for-byte against a private copy
// of the vocabulary arena.  A value present twice in the vocabulary maps to
// its LAST row, as the Python dict {v: i + 1} of Feature.lookup_table does.
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "tt_common.h"

namespace {

inline uint64_t load_tail(const unsigned char* p, int64_t n) {
  uint64_t w = 0;
  std::memcpy(&w, p, static_cast<size_t>(n));
  return w;
}

inline uint64_t fmix64(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ULL;
  h ^= h >> 33;
  return h;
}

// 8 bytes per multiply-xorshift round, murmur3 finaliser.
inline uint64_t hash_bytes(const unsigned char* p, int64_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ULL ^ static_cast<uint64_t>(n);
  int64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    std::memcpy(&w, p + i, 8);
    h = (h ^ w) * 0x9E3779B97F4A7C15ULL;
    h ^= h >> 29;
  }
  if (i < n) {
    h = (h ^ load_tail(p + i, n - i)) * 0xC2B2AE3D27D4EB4FULL;
    h ^= h >> 31;
  }
  return fmix64(h);
}

struct Slot {
  uint64_t hash;
  int64_t key;  // vocabulary index (row - 1); -1 = empty
};

struct Vocab {
  std::vector<unsigned char> data;
  std::vector<int64_t> offsets;  // n + 1
  std::vector<Slot> slots;
  uint64_t mask = 0;
  int64_t size = 0;

  int32_t find(const unsigned char* p, int64_t n) const {
    const uint64_t h = hash_bytes(p, n);
    for (uint64_t s = h & mask;; s = (s + 1) & mask) {
      const Slot& sl = slots[s];
      if (sl.key < 0) return 0;  // OOV row
      if (sl.hash == h) {
        const int64_t b = offsets[sl.key], e = offsets[sl.key + 1];
        if (e - b == n && (n == 0 || std::memcmp(data.data() + b, p, static_cast<size_t>(n)) == 0))
          return static_cast<int32_t>(sl.key + 1);
      }
    }
  }
};

int check_arena(const char* what, const char* data, const int64_t* offsets, int64_t n) {
  TT_REQUIRE(n >= 0, "%s: negative count %lld", what, (long long)n);
  TT_REQUIRE(offsets != nullptr, "%s: offsets is NULL", what);
  TT_REQUIRE(offsets[0] >= 0, "%s: offsets[0] < 0", what);
  TT_REQUIRE(n == 0 || offsets[n] == offsets[0] || data != nullptr, "%s: data is NULL", what);
  return TT_OK;
}

}  // namespace

extern "C" int tt_vocab_create(const char* data, const int64_t* offsets, int64_t n, void** out) {
  tt::clear_error();
  TT_REQUIRE(out != nullptr, "tt_vocab_create: out is NULL");
  *out = nullptr;
  if (int rc = check_arena("tt_vocab_create", data, offsets, n)) return rc;
  TT_REQUIRE(n < (int64_t(1) << 31) - 1, "tt_vocab_create: %lld values exceed int32 rows", (long long)n);
  for (int64_t i = 0; i < n; ++i)
    TT_REQUIRE(offsets[i + 1] >= offsets[i], "tt_vocab_create: offsets decrease at %lld", (long long)i);
  Vocab* v = new Vocab();
  const int64_t base = offsets[0];
  v->data.assign(reinterpret_cast<const unsigned char*>(data) + base,
                 reinterpret_cast<const unsigned char*>(data) + offsets[n]);
  v->offsets.resize(static_cast<size_t>(n) + 1);
  for (int64_t i = 0; i <= n; ++i) v->offsets[i] = offsets[i] - base;
  uint64_t cap = 16;
  while (cap < static_cast<uint64_t>(2 * n + 1)) cap <<= 1;
  v->slots.assign(cap, Slot{0, -1});
  v->mask = cap - 1;
  v->size = n;
  for (int64_t i = 0; i < n; ++i) {
    const unsigned char* p = v->data.data() + v->offsets[i];
    const int64_t len = v->offsets[i + 1] - v->offsets[i];
    const uint64_t h = hash_bytes(p, len);
    for (uint64_t s = h & v->mask;; s = (s + 1) & v->mask) {
      Slot& sl = v->slots[s];
      if (sl.key < 0) {
        sl = Slot{h, i};
        break;
      }
      if (sl.hash == h) {
        const int64_t b = v->offsets[sl.key], e = v->offsets[sl.key + 1];
        if (e - b == len && (len == 0 || std::memcmp(v->data.data() + b, p, static_cast<size_t>(len)) == 0)) {
          sl.key = i;  // duplicate: the last occurrence wins
          break;
        }
      }
    }
  }
  *out = v;
  return TT_OK;
}

extern "C" int64_t tt_vocab_size(const void* vocab) {
  return vocab ? static_cast<const Vocab*>(vocab)->size : -1;
}

extern "C" int tt_vocab_encode(const void* vocab, const char* data, const int64_t* offsets, int64_t n,
                               int32_t* out_rows, int32_t num_threads) {
  tt::clear_error();
  TT_REQUIRE(vocab != nullptr, "tt_vocab_encode: vocab is NULL");
  if (int rc = check_arena("tt_vocab_encode", data, offsets, n)) return rc;
  TT_REQUIRE(n == 0 || out_rows != nullptr, "tt_vocab_encode: out_rows is NULL");
  const Vocab* v = static_cast<const Vocab*>(vocab);
  const unsigned char* bytes = reinterpret_cast<const unsigned char*>(data);
  bool bad = false;
  for (int64_t i = 0; i < n && !bad; ++i) bad = offsets[i + 1] < offsets[i];
  TT_REQUIRE(!bad, "tt_vocab_encode: offsets decrease");
  int threads = num_threads > 0 ? num_threads : static_cast<int>(std::thread::hardware_concurrency());
  threads = std::max(1, std::min<int>(threads, 64));
  const int64_t per = std::max<int64_t>(int64_t(1) << 15, tt::ceil_div(n, threads));
  auto work = [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) out_rows[i] = v->find(bytes + offsets[i], offsets[i + 1] - offsets[i]);
  };
  if (n <= per) {
    work(0, n);
    return TT_OK;
  }
  std::vector<std::thread> pool;
  for (int64_t lo = per; lo < n; lo += per) pool.emplace_back(work, lo, std::min(n, lo + per));
  work(0, std::min(n, per));
  for (auto& t : pool) t.join();
  return TT_OK;
}

extern "C" int tt_vocab_destroy(void* vocab) {
  delete static_cast<Vocab*>(vocab);
  return TT_OK;
}
