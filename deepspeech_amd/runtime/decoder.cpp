// Native CTC decoding + edit distance for deepspeech_amd (host C++ runtime).
//
// Reference: tf.nn.ctc_greedy_decoder (src/deepSpeech_test.py:212-215) and the
// python-Levenshtein CER of src/deepSpeech_test.py:130. Adds a CTC prefix beam search
// (BASELINE config 4: streaming uni-GRU + beam-search decoder) that can carry its beam
// across streaming chunks.
// The cores take raw pointers; the pybind11 wrappers are compiled out with DS2_NO_PYBIND
// (tests/native/sanitize_driver.cpp builds the cores under ASan/UBSan and TSan).
#ifndef DS2_NO_PYBIND
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#endif

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <stdexcept>
#include <thread>
#include <cmath>
#include <limits>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#ifndef DS2_NO_PYBIND
namespace py = pybind11;
#endif

namespace ds2rt {

static inline float log_add(float a, float b) {
  if (a == -INFINITY) return b;
  if (b == -INFINITY) return a;
  const float m = std::max(a, b);
  return m + std::log1p(std::exp(-std::fabs(a - b)));
}

// ---------------------------------------------------------------- greedy
// best [T, N] argmax classes (time-major), lens [N]
std::vector<std::vector<int>> greedy_collapse_raw(const int* best, int T, int N, const int* lens, int blank) {
  std::vector<std::vector<int>> out(N);
  for (int n = 0; n < N; ++n) {
    int prev = -1;
    const int L = std::max(0, std::min<int>(T, lens[n]));
    for (int t = 0; t < L; ++t) {
      const int c = best[(size_t)t * N + n];
      if (c != prev && c != blank) out[n].push_back(c);
      prev = c;
    }
  }
  return out;
}

#ifndef DS2_NO_PYBIND
std::vector<std::vector<int>> greedy_collapse(py::array_t<int, py::array::c_style | py::array::forcecast> best,
                                              py::array_t<int, py::array::c_style | py::array::forcecast> lens,
                                              int blank) {
  if (best.ndim() != 2 || lens.ndim() != 1 || lens.shape(0) != best.shape(1))
    throw std::runtime_error("greedy_collapse: best [T, N], lens [N] expected");
  return greedy_collapse_raw(best.data(), (int)best.shape(0), (int)best.shape(1), lens.data(), blank);
}
#endif

// ---------------------------------------------------------------- edit distance
template <typename Seq>
int edit_distance(const Seq& a, const Seq& b) {
  const size_t n = a.size(), m = b.size();
  std::vector<int> prev(m + 1), cur(m + 1);
  for (size_t j = 0; j <= m; ++j) prev[j] = (int)j;
  for (size_t i = 1; i <= n; ++i) {
    cur[0] = (int)i;
    for (size_t j = 1; j <= m; ++j) {
      const int sub = prev[j - 1] + (a[i - 1] == b[j - 1] ? 0 : 1);
      cur[j] = std::min({prev[j] + 1, cur[j - 1] + 1, sub});
    }
    std::swap(prev, cur);
  }
  return prev[m];
}

int levenshtein_str(const std::string& a, const std::string& b) { return edit_distance(a, b); }
int levenshtein_ids(const std::vector<int>& a, const std::vector<int>& b) { return edit_distance(a, b); }

// ---------------------------------------------------------------- prefix beam search
// Prefixes live in a trie (node = parent + last label), so extending a prefix, testing its
// last label and merging two hypotheses that reach the same prefix are O(1) integer
// operations instead of copying and hashing label vectors. Per frame, the candidate set
// is the classes within `prune` (log) of the frame's best class.
class PrefixBeamSearch {
 public:
  PrefixBeamSearch(int beam, int blank, float prune) : beam_(beam), blank_(blank), prune_(prune) { reset(); }

  void reset() {
    nodes_.assign(1, Node{-1, -1});
    children_.clear();
    slot_.assign(1, -1);
    beams_.assign(1, Hyp{0, 0.f, -INFINITY});
  }

#ifndef DS2_NO_PYBIND
  // log_probs: [T, K] log-softmax rows of ONE utterance (a streaming chunk or the whole thing)
  void feed(py::array_t<float, py::array::c_style | py::array::forcecast> log_probs) {
    if (log_probs.ndim() != 2) throw std::runtime_error("PrefixBeamSearch.feed: [T, K] expected");
    const int T = (int)log_probs.shape(0), K = (int)log_probs.shape(1);
    const float* data = log_probs.data();
    py::gil_scoped_release rel;
    feed_raw(data, T, K, K);
  }
#endif

  // rows t at lp + t * stride (stride >= K: rows of a [T, B, K] tensor for one stream)
  void feed_raw(const float* lp, int T, int K, size_t stride) {
    std::vector<int> cand;
    std::vector<Hyp> next;
    std::vector<int> touched;
    for (int t = 0; t < T; ++t) {
      const float* row = lp + (size_t)t * stride;
      cand.clear();
      float mx = -INFINITY;
      for (int k = 0; k < K; ++k) mx = std::max(mx, row[k]);
      for (int k = 0; k < K; ++k)
        if (row[k] >= mx + prune_) cand.push_back(k);
      next.clear();
      touched.clear();
      auto get = [&](int node) -> Hyp& {
        if ((size_t)node >= slot_.size()) slot_.resize(nodes_.size(), -1);
        int& s = slot_[node];
        if (s < 0) {
          s = (int)next.size();
          next.push_back(Hyp{node, -INFINITY, -INFINITY});
          touched.push_back(node);
        }
        return next[s];
      };
      for (size_t bi = 0; bi < beams_.size(); ++bi) {
        const Hyp b = beams_[bi];
        const float tot = log_add(b.pb, b.pnb);
        const int last = nodes_[b.node].label;
        for (int k : cand) {
          const float p = row[k];
          if (k == blank_) {
            Hyp& nb = get(b.node);
            nb.pb = log_add(nb.pb, tot + p);
            continue;
          }
          const int ext = child(b.node, k);
          if (k == last) {
            Hyp& ne = get(ext);
            ne.pnb = log_add(ne.pnb, b.pb + p);        // repeated char needs a blank between
            Hyp& same = get(b.node);
            same.pnb = log_add(same.pnb, b.pnb + p);   // collapse into the same prefix
          } else {
            Hyp& ne = get(ext);
            ne.pnb = log_add(ne.pnb, tot + p);
          }
        }
      }
      for (int node : touched) slot_[node] = -1;
      const size_t keep = std::min<size_t>((size_t)beam_, next.size());
      std::partial_sort(next.begin(), next.begin() + keep, next.end(),
                        [](const Hyp& a, const Hyp& b) { return log_add(a.pb, a.pnb) > log_add(b.pb, b.pnb); });
      next.resize(keep);
      beams_.swap(next);
    }
  }

  std::vector<std::pair<std::vector<int>, float>> results() const {
    std::vector<std::pair<std::vector<int>, float>> r;
    for (const Hyp& b : beams_) r.emplace_back(prefix(b.node), log_add(b.pb, b.pnb));
    return r;
  }

  std::vector<int> best() const { return beams_.empty() ? std::vector<int>{} : prefix(beams_[0].node); }

 private:
  struct Node {
    int parent, label;
  };
  struct Hyp {
    int node;
    float pb;    // log prob ending in blank
    float pnb;   // log prob ending in non-blank
  };

  int child(int parent, int label) {
    const uint64_t key = ((uint64_t)(uint32_t)parent << 16) | (uint32_t)label;
    auto it = children_.find(key);
    if (it != children_.end()) return it->second;
    const int id = (int)nodes_.size();
    nodes_.push_back(Node{parent, label});
    children_.emplace(key, id);
    return id;
  }

  std::vector<int> prefix(int node) const {
    std::vector<int> out;
    for (int n = node; n > 0; n = nodes_[n].parent) out.push_back(nodes_[n].label);
    std::reverse(out.begin(), out.end());
    return out;
  }

  int beam_, blank_;
  float prune_;
  std::vector<Node> nodes_;
  std::unordered_map<uint64_t, int> children_;
  std::vector<int> slot_;     // node -> index into this frame's hypothesis list, -1 if none
  std::vector<Hyp> beams_;
};

// run fn(i) for i in [0, n) on up to `threads` worker threads (GIL released by the caller)
template <typename Fn>
void parallel_for(int n, int threads, Fn&& fn) {
  int nt = std::max(1, std::min(n, threads));
  if (nt == 1) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  std::atomic<int> next{0};
  std::vector<std::thread> pool;
  pool.reserve(nt);
  for (int w = 0; w < nt; ++w)
    pool.emplace_back([&]() {
      for (int i = next.fetch_add(1); i < n; i = next.fetch_add(1)) fn(i);
    });
  for (auto& th : pool) th.join();
}

int default_threads() {
  const unsigned hc = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(hc == 0 ? 1u : hc, 16u));
}

// lp [T, N, K] time-major log-probs, lens [N]; utterances spread over worker threads
std::vector<std::vector<int>> beam_search_batch_raw(const float* base, int T, int N, int K, const int* lens, int beam,
                                                    int blank, float prune, int threads) {
  std::vector<int> L(N);
  for (int n = 0; n < N; ++n) L[n] = std::max(0, std::min<int>(T, lens[n]));
  std::vector<std::vector<int>> out(N);
  parallel_for(N, threads > 0 ? threads : default_threads(), [&](int n) {
    PrefixBeamSearch bs(beam, blank, prune);
    bs.feed_raw(base + (size_t)n * K, L[n], K, (size_t)N * K);
    out[n] = bs.best();
  });
  return out;
}

#ifndef DS2_NO_PYBIND
std::vector<std::vector<int>> beam_search_batch(py::array_t<float, py::array::c_style | py::array::forcecast> lp,
                                                py::array_t<int, py::array::c_style | py::array::forcecast> lens,
                                                int beam, int blank, float prune, int threads) {
  if (lp.ndim() != 3 || lens.ndim() != 1 || lens.shape(0) != lp.shape(1))
    throw std::runtime_error("beam_search_batch: log_probs [T, N, K], lens [N] expected");
  const int T = (int)lp.shape(0), N = (int)lp.shape(1), K = (int)lp.shape(2);
  const float* base = lp.data();
  const int* l = lens.data();
  py::gil_scoped_release rel;
  return beam_search_batch_raw(base, T, N, K, l, beam, blank, prune, threads);
}
#endif

// B independent streams decoded incrementally chunk by chunk (streaming inference): the
// beams persist across feed() calls, streams are spread over worker threads.
class BatchBeamSearch {
 public:
  BatchBeamSearch(int streams, int beam, int blank, float prune, int threads)
      : threads_(threads > 0 ? threads : default_threads()) {
    for (int i = 0; i < streams; ++i) s_.emplace_back(beam, blank, prune);
  }
  void reset() {
    for (auto& b : s_) b.reset();
  }
  // log_probs [T, B, K]; lens [B] valid frames of this chunk per stream
  void feed_raw(const float* base, int T, int B, int K, const int* lens) {
    if (B != (int)s_.size()) throw std::runtime_error("BatchBeamSearch.feed: stream count mismatch");
    std::vector<int> L(B);
    for (int b = 0; b < B; ++b) L[b] = std::max(0, std::min<int>(T, lens[b]));
    parallel_for(B, threads_, [&](int b) { s_[b].feed_raw(base + (size_t)b * K, L[b], K, (size_t)B * K); });
  }
#ifndef DS2_NO_PYBIND
  void feed(py::array_t<float, py::array::c_style | py::array::forcecast> lp,
            py::array_t<int, py::array::c_style | py::array::forcecast> lens) {
    if (lp.ndim() != 3 || lens.ndim() != 1 || lens.shape(0) != lp.shape(1))
      throw std::runtime_error("BatchBeamSearch.feed: log_probs [T, B, K], lens [B] expected");
    const int T = (int)lp.shape(0), B = (int)lp.shape(1), K = (int)lp.shape(2);
    const float* base = lp.data();
    const int* l = lens.data();
    py::gil_scoped_release rel;
    feed_raw(base, T, B, K, l);
  }
#endif
  std::vector<std::vector<int>> best() const {
    std::vector<std::vector<int>> r;
    for (const auto& b : s_) r.push_back(b.best());
    return r;
  }

 private:
  int threads_;
  std::vector<PrefixBeamSearch> s_;
};

}  // namespace ds2rt

#ifndef DS2_NO_PYBIND
void register_loader(py::module_& m);
void register_tfrecord(py::module_& m);
void register_bundle(py::module_& m);

PYBIND11_MODULE(_native, m) {
  m.doc() = "deepspeech_amd native host runtime";
  m.def("greedy_collapse", &ds2rt::greedy_collapse, py::arg("best"), py::arg("lens"), py::arg("blank"));
  m.def("levenshtein", &ds2rt::levenshtein_str);
  m.def("levenshtein_ids", &ds2rt::levenshtein_ids);
  m.def("beam_search_batch", &ds2rt::beam_search_batch, py::arg("log_probs"), py::arg("lens"), py::arg("beam"),
        py::arg("blank"), py::arg("prune") = -10.0f, py::arg("threads") = 0);
  py::class_<ds2rt::BatchBeamSearch>(m, "BatchBeamSearch")
      .def(py::init<int, int, int, float, int>(), py::arg("streams"), py::arg("beam"), py::arg("blank"),
           py::arg("prune") = -10.0f, py::arg("threads") = 0)
      .def("reset", &ds2rt::BatchBeamSearch::reset)
      .def("feed", &ds2rt::BatchBeamSearch::feed)
      .def("best", &ds2rt::BatchBeamSearch::best);
  py::class_<ds2rt::PrefixBeamSearch>(m, "PrefixBeamSearch")
      .def(py::init<int, int, float>(), py::arg("beam"), py::arg("blank"), py::arg("prune") = -10.0f)
      .def("reset", &ds2rt::PrefixBeamSearch::reset)
      .def("feed", &ds2rt::PrefixBeamSearch::feed)
      .def("results", &ds2rt::PrefixBeamSearch::results)
      .def("best", &ds2rt::PrefixBeamSearch::best);
  register_loader(m);
  register_tfrecord(m);
  register_bundle(m);
}
#endif  // DS2_NO_PYBIND
