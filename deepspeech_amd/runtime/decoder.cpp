// Native CTC decoding + edit distance for deepspeech_amd (host C++ runtime).
//
// Reference: tf.nn.ctc_greedy_decoder (src/deepSpeech_test.py:212-215) and the
// python-Levenshtein CER of src/deepSpeech_test.py:130. Adds a CTC prefix beam search
// (BASELINE config 4: streaming uni-GRU + beam-search decoder) that can carry its beam
// across streaming chunks.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace ds2rt {

static inline float log_add(float a, float b) {
  if (a == -INFINITY) return b;
  if (b == -INFINITY) return a;
  const float m = std::max(a, b);
  return m + std::log1p(std::exp(-std::fabs(a - b)));
}

// ---------------------------------------------------------------- greedy
std::vector<std::vector<int>> greedy_collapse(py::array_t<int, py::array::c_style | py::array::forcecast> best,
                                              py::array_t<int, py::array::c_style | py::array::forcecast> lens,
                                              int blank) {
  auto b = best.unchecked<2>();   // [T, N]
  auto l = lens.unchecked<1>();
  const int T = (int)b.shape(0), N = (int)b.shape(1);
  std::vector<std::vector<int>> out(N);
  for (int n = 0; n < N; ++n) {
    int prev = -1;
    const int L = std::min<int>(T, l(n));
    for (int t = 0; t < L; ++t) {
      const int c = b(t, n);
      if (c != prev && c != blank) out[n].push_back(c);
      prev = c;
    }
  }
  return out;
}

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
struct Beam {
  std::vector<int> prefix;
  float pb;    // log prob ending in blank
  float pnb;   // log prob ending in non-blank
  float total() const { return log_add(pb, pnb); }
};

struct VecHash {
  size_t operator()(const std::vector<int>& v) const {
    size_t h = 1469598103934665603ull;
    for (int x : v) h = (h ^ (size_t)(x + 1)) * 1099511628211ull;
    return h;
  }
};

class PrefixBeamSearch {
 public:
  PrefixBeamSearch(int beam, int blank, float prune) : beam_(beam), blank_(blank), prune_(prune) { reset(); }

  void reset() {
    beams_.clear();
    beams_.push_back(Beam{{}, 0.f, -INFINITY});
  }

  // log_probs: [T, K] log-softmax rows of ONE utterance (a streaming chunk or the whole thing)
  void feed(py::array_t<float, py::array::c_style | py::array::forcecast> log_probs) {
    auto lp = log_probs.unchecked<2>();
    const int T = (int)lp.shape(0), K = (int)lp.shape(1);
    const float* data = log_probs.data();
    py::gil_scoped_release rel;
    feed_raw(data, T, K);
  }

  void feed_raw(const float* lp, int T, int K) {
    std::vector<int> cand;
    for (int t = 0; t < T; ++t) {
      const float* row = lp + (size_t)t * K;
      cand.clear();
      float mx = -INFINITY;
      for (int k = 0; k < K; ++k) mx = std::max(mx, row[k]);
      for (int k = 0; k < K; ++k)
        if (row[k] >= mx + prune_) cand.push_back(k);
      std::unordered_map<std::vector<int>, Beam, VecHash> next;
      next.reserve(beams_.size() * (cand.size() + 1) * 2);
      auto get = [&](const std::vector<int>& p) -> Beam& {
        auto it = next.find(p);
        if (it == next.end()) it = next.emplace(p, Beam{p, -INFINITY, -INFINITY}).first;
        return it->second;
      };
      for (const Beam& b : beams_) {
        const float tot = b.total();
        for (int k : cand) {
          const float p = row[k];
          if (k == blank_) {
            Beam& nb = get(b.prefix);
            nb.pb = log_add(nb.pb, tot + p);
            continue;
          }
          const int last = b.prefix.empty() ? -1 : b.prefix.back();
          std::vector<int> ext = b.prefix;
          ext.push_back(k);
          Beam& ne = get(ext);
          if (k == last) {
            ne.pnb = log_add(ne.pnb, b.pb + p);        // repeated char needs a blank between
            Beam& same = get(b.prefix);
            same.pnb = log_add(same.pnb, b.pnb + p);   // collapse into the same prefix
          } else {
            ne.pnb = log_add(ne.pnb, tot + p);
          }
        }
      }
      beams_.clear();
      beams_.reserve(next.size());
      for (auto& kv : next) beams_.push_back(std::move(kv.second));
      std::sort(beams_.begin(), beams_.end(), [](const Beam& a, const Beam& b) { return a.total() > b.total(); });
      if ((int)beams_.size() > beam_) beams_.resize(beam_);
    }
  }

  std::vector<std::pair<std::vector<int>, float>> results() const {
    std::vector<std::pair<std::vector<int>, float>> r;
    for (const Beam& b : beams_) r.emplace_back(b.prefix, b.total());
    return r;
  }

  std::vector<int> best() const { return beams_.empty() ? std::vector<int>{} : beams_[0].prefix; }

 private:
  int beam_, blank_;
  float prune_;
  std::vector<Beam> beams_;
};

std::vector<std::vector<int>> beam_search_batch(py::array_t<float, py::array::c_style | py::array::forcecast> lp,
                                                py::array_t<int, py::array::c_style | py::array::forcecast> lens,
                                                int beam, int blank, float prune) {
  auto a = lp.unchecked<3>();   // [T, N, K] time-major log-probs
  auto l = lens.unchecked<1>();
  const int T = (int)a.shape(0), N = (int)a.shape(1), K = (int)a.shape(2);
  std::vector<int> L(N);
  for (int n = 0; n < N; ++n) L[n] = std::min<int>(T, l(n));
  const float* base = lp.data();
  std::vector<std::vector<int>> out(N);
  py::gil_scoped_release rel;
  std::vector<float> slab;
  for (int n = 0; n < N; ++n) {
    slab.resize((size_t)L[n] * K);
    for (int t = 0; t < L[n]; ++t)
      for (int k = 0; k < K; ++k) slab[(size_t)t * K + k] = base[((size_t)t * N + n) * K + k];
    PrefixBeamSearch bs(beam, blank, prune);
    bs.feed_raw(slab.data(), L[n], K);
    out[n] = bs.best();
  }
  return out;
}

}  // namespace ds2rt

void register_loader(py::module_& m);
void register_tfrecord(py::module_& m);

PYBIND11_MODULE(_native, m) {
  m.doc() = "deepspeech_amd native host runtime";
  m.def("greedy_collapse", &ds2rt::greedy_collapse, py::arg("best"), py::arg("lens"), py::arg("blank"));
  m.def("levenshtein", &ds2rt::levenshtein_str);
  m.def("levenshtein_ids", &ds2rt::levenshtein_ids);
  m.def("beam_search_batch", &ds2rt::beam_search_batch, py::arg("log_probs"), py::arg("lens"), py::arg("beam"),
        py::arg("blank"), py::arg("prune") = -10.0f);
  py::class_<ds2rt::PrefixBeamSearch>(m, "PrefixBeamSearch")
      .def(py::init<int, int, float>(), py::arg("beam"), py::arg("blank"), py::arg("prune") = -10.0f)
      .def("reset", &ds2rt::PrefixBeamSearch::reset)
      .def("feed", &ds2rt::PrefixBeamSearch::feed)
      .def("results", &ds2rt::PrefixBeamSearch::results)
      .def("best", &ds2rt::PrefixBeamSearch::best);
  register_loader(m);
  register_tfrecord(m);
}
