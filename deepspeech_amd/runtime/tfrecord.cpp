// TFRecord framing + tf.train.SequenceExample codec (no TensorFlow dependency).
//
// Reference on-disk format: src/preprocess_LibriSpeech.py:45-85 writes SequenceExamples
// with context {seq_len: int64, labels: int64 list} and feature_list {feats: T x float[161]};
// src/deepSpeech_input.py:34-49 parses them. This codec reads and writes exactly those
// records so preprocessed reference data can be consumed (and produced) here.
//
// TFRecord: uint64 len | uint32 masked_crc32c(len) | data | uint32 masked_crc32c(data)
// Cores are pybind-free (raw bytes / std containers); the wrappers are compiled out with
// DS2_NO_PYBIND for the sanitizer driver (tests/native/sanitize_driver.cpp).
#ifndef DS2_NO_PYBIND
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#endif

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#ifndef DS2_NO_PYBIND
namespace py = pybind11;
#endif

namespace ds2rt {

// ---------------------------------------------------------------- crc32c (Castagnoli)
struct CrcTable {
  uint32_t t[256];
  CrcTable() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (0x82F63B78u ^ (c >> 1)) : (c >> 1);
      t[i] = c;
    }
  }
};
uint32_t crc32c(const uint8_t* d, size_t n) {
  static const CrcTable tab;      // thread-safe one-time init (was an unsynchronised flag)
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = tab.t[(c ^ d[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}
uint32_t masked_crc(const uint8_t* d, size_t n) {
  const uint32_t c = crc32c(d, n);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

std::vector<std::string> read_records_raw(const std::string& path, bool check_crc) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  std::vector<std::string> out;
  std::vector<uint8_t> buf;
  while (true) {
    uint8_t hdr[12];
    const size_t got = std::fread(hdr, 1, 12, f);
    if (got == 0) break;
    if (got != 12) { std::fclose(f); throw std::runtime_error("truncated record header in " + path); }
    uint64_t len;
    std::memcpy(&len, hdr, 8);
    uint32_t lcrc;
    std::memcpy(&lcrc, hdr + 8, 4);
    if (check_crc && masked_crc(hdr, 8) != lcrc) { std::fclose(f); throw std::runtime_error("length crc mismatch"); }
    if (len > (1ull << 34)) { std::fclose(f); throw std::runtime_error("implausible record length"); }
    buf.resize(len + 4);
    if (std::fread(buf.data(), 1, len + 4, f) != len + 4) { std::fclose(f); throw std::runtime_error("truncated record"); }
    uint32_t dcrc;
    std::memcpy(&dcrc, buf.data() + len, 4);
    if (check_crc && masked_crc(buf.data(), len) != dcrc) { std::fclose(f); throw std::runtime_error("data crc mismatch"); }
    out.emplace_back(reinterpret_cast<const char*>(buf.data()), len);
  }
  std::fclose(f);
  return out;
}

void write_records(const std::string& path, const std::vector<std::string>& recs) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot write " + path);
  for (const auto& r : recs) {
    uint8_t hdr[12];
    const uint64_t len = r.size();
    std::memcpy(hdr, &len, 8);
    const uint32_t lc = masked_crc(hdr, 8);
    std::memcpy(hdr + 8, &lc, 4);
    const uint32_t dc = masked_crc(reinterpret_cast<const uint8_t*>(r.data()), r.size());
    std::fwrite(hdr, 1, 12, f);
    std::fwrite(r.data(), 1, r.size(), f);
    std::fwrite(&dc, 1, 4, f);
  }
  std::fclose(f);
}

// ---------------------------------------------------------------- protobuf wire helpers
struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  bool done() const { return p >= e; }
  void need(size_t n) const {
    if ((size_t)(e - p) < n) throw std::runtime_error("truncated field");
  }
  uint64_t varint() {
    uint64_t v = 0;
    int s = 0;
    while (p < e) {
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7F) << s;
      if (!(b & 0x80)) return v;
      s += 7;
    }
    throw std::runtime_error("bad varint");
  }
  Reader sub() {
    const uint64_t n = varint();
    if (n > (uint64_t)(e - p)) throw std::runtime_error("bad length");
    Reader r{p, p + n};
    p += n;
    return r;
  }
  void skip(int wt) {
    if (wt == 0) varint();
    else if (wt == 1) { need(8); p += 8; }
    else if (wt == 2) sub();
    else if (wt == 5) { need(4); p += 4; }
    else throw std::runtime_error("unsupported wire type");
  }
};

struct Feature {
  int kind = 0;                 // 2 = float_list, 3 = int64_list, 1 = bytes_list
  std::vector<float> f;
  std::vector<int64_t> i;
};

static Feature parse_feature(Reader r) {
  Feature ft;
  while (!r.done()) {
    const uint64_t key = r.varint();
    const int field = (int)(key >> 3), wt = (int)(key & 7);
    if ((field == 2 || field == 3) && wt == 2) {
      ft.kind = field;
      Reader lst = r.sub();
      while (!lst.done()) {
        const uint64_t k2 = lst.varint();
        const int wt2 = (int)(k2 & 7);
        if ((k2 >> 3) != 1) { lst.skip(wt2); continue; }
        if (wt2 == 2) {   // packed
          Reader pk = lst.sub();
          if (field == 2) {
            while (!pk.done()) { pk.need(4); float v; std::memcpy(&v, pk.p, 4); pk.p += 4; ft.f.push_back(v); }
          } else {
            while (!pk.done()) ft.i.push_back((int64_t)pk.varint());
          }
        } else if (wt2 == 5 && field == 2) {
          lst.need(4); float v; std::memcpy(&v, lst.p, 4); lst.p += 4; ft.f.push_back(v);
        } else if (wt2 == 0 && field == 3) {
          ft.i.push_back((int64_t)lst.varint());
        } else {
          lst.skip(wt2);
        }
      }
    } else {
      r.skip(wt);
    }
  }
  return ft;
}

// returns map entry (key, value reader)
static std::pair<std::string, Reader> parse_entry(Reader r) {
  std::string key;
  Reader val{nullptr, nullptr};
  while (!r.done()) {
    const uint64_t k = r.varint();
    const int f = (int)(k >> 3), wt = (int)(k & 7);
    if (f == 1 && wt == 2) { Reader s = r.sub(); key.assign(reinterpret_cast<const char*>(s.p), s.e - s.p); }
    else if (f == 2 && wt == 2) val = r.sub();
    else r.skip(wt);
  }
  return {key, val};
}

struct SeqExample {
  int64_t seq_len = 0;
  std::vector<int32_t> labels;
  std::vector<float> feats;   // [T, F] row-major
  int T = 0, F = 0;
};

// parse a SequenceExample: (seq_len, labels int32 [L], feats float32 [T, F])
SeqExample parse_sequence_example_raw(const uint8_t* data, size_t size, const std::string& feats_key) {
  Reader r{data, data + size};
  int64_t seq_len = -1;
  std::vector<int64_t> labels;
  std::vector<std::vector<float>> frames;
  while (!r.done()) {
    const uint64_t k = r.varint();
    const int f = (int)(k >> 3), wt = (int)(k & 7);
    if (f == 1 && wt == 2) {            // context: Features
      Reader feats = r.sub();
      while (!feats.done()) {
        const uint64_t k2 = feats.varint();
        if ((k2 >> 3) == 1 && (k2 & 7) == 2) {
          auto e = parse_entry(feats.sub());
          if (!e.second.p) continue;
          Feature ft = parse_feature(e.second);
          if (e.first == "seq_len" && !ft.i.empty()) seq_len = ft.i[0];
          else if (e.first == "labels") labels = ft.i;
        } else {
          feats.skip((int)(k2 & 7));
        }
      }
    } else if (f == 2 && wt == 2) {     // feature_lists
      Reader fl = r.sub();
      while (!fl.done()) {
        const uint64_t k2 = fl.varint();
        if ((k2 >> 3) == 1 && (k2 & 7) == 2) {
          auto e = parse_entry(fl.sub());
          if (e.first != feats_key || !e.second.p) continue;
          Reader lst = e.second;   // FeatureList { repeated Feature feature = 1; }
          while (!lst.done()) {
            const uint64_t k3 = lst.varint();
            if ((k3 >> 3) == 1 && (k3 & 7) == 2) frames.push_back(parse_feature(lst.sub()).f);
            else lst.skip((int)(k3 & 7));
          }
        } else {
          fl.skip((int)(k2 & 7));
        }
      }
    } else {
      r.skip(wt);
    }
  }
  SeqExample ex;
  ex.T = (int)frames.size();
  ex.F = ex.T ? (int)frames[0].size() : 0;
  ex.feats.resize((size_t)ex.T * ex.F);
  for (int t = 0; t < ex.T; ++t) {
    if ((int)frames[t].size() != ex.F) throw std::runtime_error("ragged frames");
    std::memcpy(ex.feats.data() + (size_t)t * ex.F, frames[t].data(), sizeof(float) * ex.F);
  }
  ex.labels.assign(labels.begin(), labels.end());
  ex.seq_len = seq_len < 0 ? ex.T : seq_len;
  return ex;
}

// ---------------------------------------------------------------- writer
static void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) { o.push_back((char)((v & 0x7F) | 0x80)); v >>= 7; }
  o.push_back((char)v);
}
static void put_bytes(std::string& o, int field, const std::string& b) {
  put_varint(o, ((uint64_t)field << 3) | 2);
  put_varint(o, b.size());
  o += b;
}
static std::string int64_feature(const std::vector<int64_t>& v) {
  std::string packed, lst, feat;
  for (int64_t x : v) put_varint(packed, (uint64_t)x);
  put_bytes(lst, 1, packed);
  put_bytes(feat, 3, lst);
  return feat;
}
static std::string float_feature(const float* v, int n) {
  std::string packed(reinterpret_cast<const char*>(v), sizeof(float) * n), lst, feat;
  put_bytes(lst, 1, packed);
  put_bytes(feat, 2, lst);
  return feat;
}
static std::string map_entry(const std::string& key, const std::string& val) {
  std::string e;
  put_bytes(e, 1, key);
  put_bytes(e, 2, val);
  return e;
}

std::string make_sequence_example_raw(int64_t seq_len, const float* feats, int T, int F, const int64_t* labels,
                                      size_t L, const std::string& feats_key) {
  std::vector<int64_t> lab(labels, labels + L);
  std::string ctx, fl, lst, out;
  put_bytes(ctx, 1, map_entry("seq_len", int64_feature({seq_len})));
  put_bytes(ctx, 1, map_entry("labels", int64_feature(lab)));
  for (int t = 0; t < T; ++t) put_bytes(lst, 1, float_feature(feats + (size_t)t * F, F));
  put_bytes(fl, 1, map_entry(feats_key, lst));
  put_bytes(out, 1, ctx);
  put_bytes(out, 2, fl);
  return out;
}

#ifndef DS2_NO_PYBIND
std::vector<py::bytes> read_records(const std::string& path, bool check_crc) {
  std::vector<py::bytes> out;
  for (auto& r : read_records_raw(path, check_crc)) out.emplace_back(r);
  return out;
}

py::tuple parse_sequence_example(py::bytes data, const std::string& feats_key) {
  std::string s = data;
  SeqExample ex = parse_sequence_example_raw(reinterpret_cast<const uint8_t*>(s.data()), s.size(), feats_key);
  py::array_t<float> feats({ex.T, ex.F});
  if (!ex.feats.empty()) std::memcpy(feats.mutable_data(), ex.feats.data(), sizeof(float) * ex.feats.size());
  py::array_t<int32_t> lab({(int)ex.labels.size()});
  if (!ex.labels.empty()) std::memcpy(lab.mutable_data(), ex.labels.data(), sizeof(int32_t) * ex.labels.size());
  return py::make_tuple(ex.seq_len, lab, feats);
}

py::bytes make_sequence_example(int64_t seq_len, py::array_t<float, py::array::c_style | py::array::forcecast> feats,
                                py::array_t<int64_t, py::array::c_style | py::array::forcecast> labels,
                                const std::string& feats_key) {
  if (feats.ndim() != 2) throw std::runtime_error("make_sequence_example: feats [T, F] expected");
  return py::bytes(make_sequence_example_raw(seq_len, feats.data(), (int)feats.shape(0), (int)feats.shape(1),
                                             labels.data(), (size_t)labels.size(), feats_key));
}
#endif

}  // namespace ds2rt

#ifndef DS2_NO_PYBIND
void register_tfrecord(py::module_& m) {
  m.def("crc32c", [](py::bytes b) {
    std::string s = b;
    return ds2rt::crc32c(reinterpret_cast<const uint8_t*>(s.data()), s.size());
  });
  m.def("read_records", &ds2rt::read_records, py::arg("path"), py::arg("check_crc") = true);
  m.def("write_records", &ds2rt::write_records);
  m.def("parse_sequence_example", &ds2rt::parse_sequence_example, py::arg("data"), py::arg("feats_key") = "feats");
  m.def("make_sequence_example", &ds2rt::make_sequence_example, py::arg("seq_len"), py::arg("feats"),
        py::arg("labels"), py::arg("feats_key") = "feats");
}
#endif  // DS2_NO_PYBIND
