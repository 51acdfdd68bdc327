// TensorFlow checkpoint bundle (Saver V2: <prefix>.index + <prefix>.data-00000-of-00001) codec,
// with no TensorFlow dependency.
//
// Reference: src/deepSpeech_train.py:354-356,471 (tf.train.Saver(max_to_keep=100).save every 10
// steps), :383-398 (restore the latest via get_checkpoint_state), src/deepSpeech_test.py:93-109,
// 217-220 (eval restores the EMA shadows from the same files). A V2 checkpoint is
//   * <prefix>.data-00000-of-00001: the tensors' raw little-endian bytes back to back;
//   * <prefix>.index: a LevelDB-format SSTable (uncompressed blocks, masked-crc32c trailers)
//     mapping "" -> BundleHeaderProto and each variable name -> BundleEntryProto (dtype, shape,
//     shard, offset, size, masked crc32c of the bytes).
// This file holds the native parts: crc32c (SSE4.2 when the CPU has it), the SSTable writer /
// reader, and the data-shard writer that streams tensors from (pinned) host memory with one
// pwrite per tensor on a small thread pool, computing each tensor's checksum on the way. The
// protobuf messages are encoded in Python (deepspeech_amd/utils/tf_bundle.py).
//
// Cores are pybind-free; the wrappers are compiled out with DS2_NO_PYBIND.
#ifndef DS2_NO_PYBIND
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#endif

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#ifndef DS2_NO_PYBIND
namespace py = pybind11;
#endif

namespace ds2rt {

uint32_t crc32c(const uint8_t* d, size_t n);      // tfrecord.cpp (table-driven)
uint32_t crc32c_fast(const uint8_t* d, size_t n);

namespace {

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t crc32c_hw(const uint8_t* d, size_t n) {
  uint64_t c = 0xFFFFFFFFu;
  while (n && (reinterpret_cast<uintptr_t>(d) & 7)) {
    c = __builtin_ia32_crc32qi(static_cast<uint32_t>(c), *d++);
    --n;
  }
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, d, 8);
    c = __builtin_ia32_crc32di(c, v);
    d += 8;
    n -= 8;
  }
  while (n--) c = __builtin_ia32_crc32qi(static_cast<uint32_t>(c), *d++);
  return static_cast<uint32_t>(c) ^ 0xFFFFFFFFu;
}

bool have_sse42() {
  static const bool ok = __builtin_cpu_supports("sse4.2");
  return ok;
}
#endif

inline void put_fixed32(std::string& s, uint32_t v) {
  char b[4];
  std::memcpy(b, &v, 4);           // little-endian host (x86-64)
  s.append(b, 4);
}

inline void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back(static_cast<char>((v & 0x7F) | 0x80));
    v >>= 7;
  }
  s.push_back(static_cast<char>(v));
}

inline uint32_t get_fixed32(const char* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}

// returns the new position, or nullptr on a malformed / truncated varint
inline const char* get_varint(const char* p, const char* end, uint64_t* v) {
  uint64_t r = 0;
  for (int shift = 0; shift <= 63 && p < end; shift += 7) {
    const uint64_t b = static_cast<uint8_t>(*p++);
    r |= (b & 0x7F) << shift;
    if (!(b & 0x80)) {
      *v = r;
      return p;
    }
  }
  return nullptr;
}

constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;   // LevelDB / TF table footer magic
constexpr size_t kFooterLen = 48;                         // 2 x BlockHandle (<= 20 B each) + pad + magic
constexpr size_t kBlockSize = 256 * 1024;                 // TF table::Options default
constexpr int kRestartInterval = 16;

uint32_t mask_crc(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }
uint32_t unmask_crc(uint32_t m) {
  const uint32_t r = m - 0xa282ead8u;
  return (r >> 17) | (r << 15);
}

// LevelDB BlockBuilder: prefix-compressed entries, a restart point every `interval` entries
class BlockBuilder {
 public:
  explicit BlockBuilder(int interval) : interval_(interval) { restarts_.push_back(0); }
  void add(const std::string& key, const std::string& value) {
    size_t shared = 0;
    if (counter_ < interval_) {
      const size_t lim = std::min(last_.size(), key.size());
      while (shared < lim && last_[shared] == key[shared]) ++shared;
    } else {
      restarts_.push_back(static_cast<uint32_t>(buf_.size()));
      counter_ = 0;
    }
    put_varint(buf_, shared);
    put_varint(buf_, key.size() - shared);
    put_varint(buf_, value.size());
    buf_.append(key, shared, std::string::npos);
    buf_.append(value);
    last_ = key;
    ++counter_;
    ++entries_;
  }
  std::string finish() {
    std::string out = buf_;
    for (uint32_t r : restarts_) put_fixed32(out, r);
    put_fixed32(out, static_cast<uint32_t>(restarts_.size()));
    return out;
  }
  size_t estimate() const { return buf_.size() + 4 * (restarts_.size() + 1); }
  bool empty() const { return entries_ == 0; }
  const std::string& last_key() const { return last_; }
  void reset() {
    buf_.clear();
    restarts_.assign(1, 0);
    counter_ = 0;
    entries_ = 0;
    last_.clear();
  }

 private:
  int interval_;
  int counter_ = 0;
  size_t entries_ = 0;
  std::string buf_, last_;
  std::vector<uint32_t> restarts_;
};

// appends block + 5-byte trailer (type 0 = uncompressed, masked crc32c over block||type) to `file`
// and returns its handle (offset, size without the trailer)
std::pair<uint64_t, uint64_t> emit_block(std::string& file, const std::string& block) {
  const uint64_t off = file.size();
  file.append(block);
  file.push_back('\0');
  put_fixed32(file, mask_crc(crc32c_fast(reinterpret_cast<const uint8_t*>(file.data() + off), block.size() + 1)));
  return {off, block.size()};
}

void put_handle(std::string& s, std::pair<uint64_t, uint64_t> h) {
  put_varint(s, h.first);
  put_varint(s, h.second);
}

// entries of one block (keys restored from the prefix compression)
void parse_block(const char* base, size_t n, std::vector<std::pair<std::string, std::string>>& out) {
  if (n < 4) throw std::runtime_error("bundle index: block too short");
  const uint32_t nres = get_fixed32(base + n - 4);
  if (static_cast<uint64_t>(nres) * 4 + 4 > n) throw std::runtime_error("bundle index: bad restart count");
  const char* end = base + n - 4 - 4 * static_cast<size_t>(nres);
  const char* p = base;
  std::string key;
  while (p < end) {
    uint64_t shared, unshared, vlen;
    p = get_varint(p, end, &shared);
    if (p) p = get_varint(p, end, &unshared);
    if (p) p = get_varint(p, end, &vlen);
    if (!p || shared > key.size() || unshared > static_cast<uint64_t>(end - p) ||
        vlen > static_cast<uint64_t>(end - p) - unshared)
      throw std::runtime_error("bundle index: corrupt block entry");
    key.resize(shared);
    key.append(p, unshared);
    p += unshared;
    out.emplace_back(key, std::string(p, vlen));
    p += vlen;
  }
}

std::string read_block(const std::string& file, uint64_t off, uint64_t size, bool verify) {
  if (off > file.size() || size + 5 > file.size() - off) throw std::runtime_error("bundle index: block out of range");
  if (verify) {
    const uint32_t stored = get_fixed32(file.data() + off + size + 1);
    const uint32_t got = crc32c_fast(reinterpret_cast<const uint8_t*>(file.data() + off), size + 1);
    if (unmask_crc(stored) != got) throw std::runtime_error("bundle index: block checksum mismatch");
  }
  if (file[off + size] != '\0') throw std::runtime_error("bundle index: compressed blocks are not supported");
  return file.substr(off, size);
}

}  // namespace

uint32_t crc32c_fast(const uint8_t* d, size_t n) {
#if defined(__x86_64__)
  if (have_sse42()) return crc32c_hw(d, n);
#endif
  return crc32c(d, n);
}

uint32_t masked_crc32c(const uint8_t* d, size_t n) { return mask_crc(crc32c_fast(d, n)); }

// SSTable bytes of `kv` (keys strictly ascending, bytewise)
std::string build_table(const std::vector<std::pair<std::string, std::string>>& kv) {
  for (size_t i = 1; i < kv.size(); ++i)
    if (!(kv[i - 1].first < kv[i].first)) throw std::runtime_error("bundle index: keys must be strictly ascending");
  std::string file;
  BlockBuilder data(kRestartInterval), index(1);
  for (size_t i = 0; i < kv.size(); ++i) {
    data.add(kv[i].first, kv[i].second);
    if (data.estimate() >= kBlockSize || i + 1 == kv.size()) {
      const std::string last = data.last_key();       // a valid separator: >= every key of the block
      auto h = emit_block(file, data.finish());
      std::string hv;
      put_handle(hv, h);
      index.add(last, hv);
      data.reset();
    }
  }
  BlockBuilder meta(kRestartInterval);
  auto mh = emit_block(file, meta.finish());
  auto ih = emit_block(file, index.finish());
  std::string footer;
  put_handle(footer, mh);
  put_handle(footer, ih);
  footer.resize(kFooterLen - 8, '\0');
  put_fixed32(footer, static_cast<uint32_t>(kTableMagic & 0xffffffffu));
  put_fixed32(footer, static_cast<uint32_t>(kTableMagic >> 32));
  file.append(footer);
  return file;
}

std::vector<std::pair<std::string, std::string>> parse_table(const std::string& file, bool verify) {
  if (file.size() < kFooterLen) throw std::runtime_error("bundle index: file too short");
  const char* f = file.data() + file.size() - kFooterLen;
  const uint64_t magic = static_cast<uint64_t>(get_fixed32(f + 40)) | (static_cast<uint64_t>(get_fixed32(f + 44)) << 32);
  if (magic != kTableMagic) throw std::runtime_error("bundle index: bad table magic");
  uint64_t moff, msz, ioff, isz;
  const char* p = get_varint(f, f + 40, &moff);
  if (p) p = get_varint(p, f + 40, &msz);
  if (p) p = get_varint(p, f + 40, &ioff);
  if (p) p = get_varint(p, f + 40, &isz);
  if (!p) throw std::runtime_error("bundle index: bad footer");
  const std::string iblk = read_block(file, ioff, isz, verify);
  std::vector<std::pair<std::string, std::string>> handles, out;
  parse_block(iblk.data(), iblk.size(), handles);
  for (const auto& h : handles) {
    uint64_t off, sz;
    const char* e = h.second.data() + h.second.size();
    const char* q = get_varint(h.second.data(), e, &off);
    if (q) q = get_varint(q, e, &sz);
    if (!q) throw std::runtime_error("bundle index: bad block handle");
    const std::string blk = read_block(file, off, sz, verify);
    parse_block(blk.data(), blk.size(), out);
  }
  return out;
}

// Writes the chunks back to back into `path` (created / truncated) with pwrite on `threads`
// workers, largest chunks first; returns each chunk's masked crc32c.
std::vector<uint32_t> write_shard(const std::string& path, const std::vector<const uint8_t*>& ptrs,
                                  const std::vector<uint64_t>& sizes, int threads) {
  if (ptrs.size() != sizes.size()) throw std::runtime_error("write_shard: ptrs / sizes differ in length");
  const size_t n = ptrs.size();
  std::vector<uint64_t> offs(n);
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) {
    offs[i] = total;
    total += sizes[i];
  }
  const int fd = ::open(path.c_str(), O_CREAT | O_TRUNC | O_WRONLY | O_CLOEXEC, 0644);
  if (fd < 0) throw std::runtime_error("write_shard: cannot open " + path);
  if (total && ::ftruncate(fd, static_cast<off_t>(total)) != 0) {
    ::close(fd);
    throw std::runtime_error("write_shard: cannot size " + path);
  }
  std::vector<size_t> order(n);
  for (size_t i = 0; i < n; ++i) order[i] = i;
  std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return sizes[a] > sizes[b]; });
  std::vector<uint32_t> crcs(n, 0);
  std::atomic<size_t> next{0};
  std::atomic<bool> failed{false};
  auto work = [&]() {
    size_t k;
    while (!failed.load(std::memory_order_relaxed) && (k = next.fetch_add(1)) < n) {
      const size_t i = order[k];
      crcs[i] = masked_crc32c(ptrs[i], sizes[i]);
      uint64_t done = 0;
      while (done < sizes[i]) {
        const size_t piece = static_cast<size_t>(std::min<uint64_t>(sizes[i] - done, 1ull << 30));
        const ssize_t w = ::pwrite(fd, ptrs[i] + done, piece, static_cast<off_t>(offs[i] + done));
        if (w <= 0) {
          failed = true;
          break;
        }
        done += static_cast<uint64_t>(w);
      }
    }
  };
  const int nt = std::max(1, std::min<int>(threads, static_cast<int>(n)));
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  const bool ok = !failed && ::close(fd) == 0;
  if (!ok) throw std::runtime_error("write_shard: write to " + path + " failed");
  return crcs;
}

void write_file(const std::string& path, const std::string& bytes) {
  const int fd = ::open(path.c_str(), O_CREAT | O_TRUNC | O_WRONLY | O_CLOEXEC, 0644);
  if (fd < 0) throw std::runtime_error("cannot open " + path);
  size_t done = 0;
  while (done < bytes.size()) {
    const ssize_t w = ::write(fd, bytes.data() + done, bytes.size() - done);
    if (w <= 0) {
      ::close(fd);
      throw std::runtime_error("write to " + path + " failed");
    }
    done += static_cast<size_t>(w);
  }
  if (::close(fd) != 0) throw std::runtime_error("close of " + path + " failed");
}

}  // namespace ds2rt

#ifndef DS2_NO_PYBIND
void register_bundle(py::module_& m) {
  using KV = std::vector<std::pair<std::string, std::string>>;
  m.def("bundle_masked_crc32c", [](py::buffer b) {
    py::buffer_info info = b.request();
    const size_t n = static_cast<size_t>(info.size) * static_cast<size_t>(info.itemsize);
    const auto* p = static_cast<const uint8_t*>(info.ptr);
    py::gil_scoped_release nogil;
    return ds2rt::masked_crc32c(p, n);
  });
  m.def("bundle_crc32c_ptr", [](uintptr_t ptr, uint64_t n) {
    py::gil_scoped_release nogil;
    return ds2rt::masked_crc32c(reinterpret_cast<const uint8_t*>(ptr), n);
  }, "masked crc32c of n bytes at a raw host address (the caller keeps the memory alive)");
  m.def("bundle_build_table", [](const std::vector<std::pair<py::bytes, py::bytes>>& items) {
    KV kv;
    kv.reserve(items.size());
    for (const auto& it : items) kv.emplace_back(std::string(it.first), std::string(it.second));
    std::string out;
    {
      py::gil_scoped_release nogil;
      out = ds2rt::build_table(kv);
    }
    return py::bytes(out);
  });
  m.def("bundle_parse_table", [](py::bytes data, bool verify) {
    const std::string s(data);
    KV kv;
    {
      py::gil_scoped_release nogil;
      kv = ds2rt::parse_table(s, verify);
    }
    std::vector<std::pair<py::bytes, py::bytes>> out;
    out.reserve(kv.size());
    for (auto& e : kv) out.emplace_back(py::bytes(e.first), py::bytes(e.second));
    return out;
  }, py::arg("data"), py::arg("verify") = true);
  m.def("bundle_write_shard", [](const std::string& path, const std::vector<uintptr_t>& ptrs,
                                 const std::vector<uint64_t>& sizes, int threads) {
    std::vector<const uint8_t*> p(ptrs.size());
    for (size_t i = 0; i < ptrs.size(); ++i) p[i] = reinterpret_cast<const uint8_t*>(ptrs[i]);
    py::gil_scoped_release nogil;
    return ds2rt::write_shard(path, p, sizes, threads);
  }, py::arg("path"), py::arg("ptrs"), py::arg("sizes"), py::arg("threads") = 8,
     "write raw host buffers back to back (pwrite, thread pool); returns their masked crc32c");
  m.def("bundle_write_file", [](const std::string& path, py::bytes data) {
    const std::string s(data);
    py::gil_scoped_release nogil;
    ds2rt::write_file(path, s);
  });
}
#endif  // DS2_NO_PYBIND
