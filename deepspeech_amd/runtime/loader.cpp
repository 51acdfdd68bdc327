// Native batch loader: bucketed SortaGrad batch planning + a thread pool that assembles
// padded batches from a memory-mapped feature store.
//
// Reference: the TF input pipeline of src/deepSpeech_input.py:20-97 — TFRecordReader +
// bucket_by_sequence_length(boundaries 100..1800 step 100, 16 threads, dynamic_pad) and
// length-sorted files read in order for the first (SortaGrad) epoch (README.md:93-94).
//
// MI355X design: the GPU must never wait on Python. Workers (std::thread) gather rows of
// each utterance from an mmap'ed float32 store straight into one contiguous padded
// [N, Tmax, F] buffer, ordered by a job sequence number; Python receives zero-copy numpy
// views (the buffers are owned by capsules) and stages them to pinned memory.
//
// Store format (written by deepspeech_amd/data/store.py):
//   <prefix>.feats   float32 [total_frames, F]  little-endian, row-major
//   <prefix>.index   via Python (offsets/lengths/labels arrays are passed in)
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#ifndef DS2_NO_PYBIND
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#endif

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <numeric>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#ifndef DS2_NO_PYBIND
namespace py = pybind11;
#endif

namespace ds2rt {

// ---------------------------------------------------------------- batch planning
// Returns a list of batches (lists of utterance indices). Utterances are bucketed by
// frame count (bucket width `bucket`), long utterances dropped (> max_frames) and
// infeasible ones dropped (label needs more frames than the conv front-end leaves).
// sorted=true: SortaGrad order (ascending length); else buckets shuffled with `seed`.
// Distributed: batches are grouped in runs of `world` consecutive batches taken from the
// same bucket, so every rank of a step sees the same length class (no stragglers).
std::vector<std::vector<int64_t>> plan_batches_raw(const int* L, const int* MF, int64_t n, int batch_size, int bucket,
                                                   int max_frames, bool sorted, uint64_t seed, int world,
                                                   bool drop_last) {
  if (batch_size < 1 || bucket < 1 || world < 1) throw std::runtime_error("plan_batches: sizes must be >= 1");
  std::map<int, std::vector<int64_t>> buckets;
  for (int64_t i = 0; i < n; ++i) {
    const int len = L[i];
    if (len > max_frames || len < MF[i]) continue;
    buckets[len / bucket].push_back(i);
  }
  std::mt19937_64 rng(seed);
  std::vector<std::vector<int64_t>> groups;   // each group = `world` batches
  for (auto& kv : buckets) {
    auto& ids = kv.second;
    if (sorted) {
      std::stable_sort(ids.begin(), ids.end(), [&](int64_t a, int64_t b) { return L[a] < L[b]; });
    } else {
      std::shuffle(ids.begin(), ids.end(), rng);
    }
    const size_t per_group = (size_t)batch_size * world;
    size_t i = 0;
    for (; i + per_group <= ids.size(); i += per_group)
      groups.emplace_back(ids.begin() + i, ids.begin() + i + per_group);
    if (!drop_last && i < ids.size()) groups.emplace_back(ids.begin() + i, ids.end());
  }
  if (!sorted) std::shuffle(groups.begin(), groups.end(), rng);
  std::vector<std::vector<int64_t>> out;
  for (auto& g : groups) {
    // split the group into `world` batches (the last group may be short: round-robin)
    const size_t per = (g.size() + world - 1) / world;
    for (int r = 0; r < world; ++r) {
      std::vector<int64_t> b;
      for (size_t j = r * per; j < std::min(g.size(), (r + 1) * per); ++j) b.push_back(g[j]);
      out.push_back(std::move(b));
    }
  }
  return out;
}

#ifndef DS2_NO_PYBIND
std::vector<std::vector<int64_t>> plan_batches(py::array_t<int, py::array::c_style | py::array::forcecast> lengths,
                                               py::array_t<int, py::array::c_style | py::array::forcecast> min_frames,
                                               int batch_size, int bucket, int max_frames, bool sorted, uint64_t seed,
                                               int world, bool drop_last) {
  if (lengths.ndim() != 1 || min_frames.ndim() != 1 || lengths.shape(0) != min_frames.shape(0))
    throw std::runtime_error("plan_batches: lengths and min_frames must be 1-D of equal size");
  return plan_batches_raw(lengths.data(), min_frames.data(), lengths.shape(0), batch_size, bucket, max_frames, sorted,
                          seed, world, drop_last);
}
#endif

// ---------------------------------------------------------------- mmap store
class FeatureStore {
 public:
  FeatureStore(const std::string& path, int freq) : freq_(freq) {
    if (freq < 1) throw std::runtime_error("feature store: freq must be >= 1");
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("cannot open feature store " + path);
    struct stat st;
    if (fstat(fd_, &st) != 0) {
      ::close(fd_);                  // the destructor does not run when the constructor throws
      throw std::runtime_error("stat failed on " + path);
    }
    bytes_ = (size_t)st.st_size;
    if (bytes_ > 0) {
      base_ = ::mmap(nullptr, bytes_, PROT_READ, MAP_SHARED, fd_, 0);
      if (base_ == MAP_FAILED) {
        ::close(fd_);
        throw std::runtime_error("mmap failed on " + path);
      }
      ::madvise(base_, bytes_, MADV_WILLNEED);
    }
  }
  ~FeatureStore() {
    if (base_ && base_ != MAP_FAILED) ::munmap(base_, bytes_);
    if (fd_ >= 0) ::close(fd_);
  }
  const float* rows(int64_t frame) const { return reinterpret_cast<const float*>(base_) + frame * freq_; }
  int64_t frames() const { return (int64_t)(bytes_ / (sizeof(float) * freq_)); }
  int freq() const { return freq_; }

 private:
  int fd_ = -1;
  void* base_ = nullptr;
  size_t bytes_ = 0;
  int freq_;
};

struct Assembled {
  std::vector<float> feats;     // [N, Tmax, F]
  std::vector<int32_t> seq;     // [N]
  std::vector<int32_t> labels;  // [N, Lmax], -1 padded
  std::vector<int32_t> llen;    // [N]
  int N = 0, Tmax = 0, Lmax = 0;
};

class BatchLoader {
 public:
  BatchLoader(const std::string& feat_path, int freq, std::vector<int64_t> offsets, std::vector<int32_t> lengths,
              std::vector<int32_t> labels, std::vector<int64_t> label_offsets, std::vector<int32_t> label_lens,
              int num_threads, int pad_to)
      : store_(feat_path, freq), pad_to_(std::max(1, pad_to)), off_(std::move(offsets)),
        loff_(std::move(label_offsets)), len_(std::move(lengths)), lab_(std::move(labels)),
        llen_(std::move(label_lens)) {
    const size_t n = off_.size();
    if (len_.size() != n || loff_.size() != n || llen_.size() != n)
      throw std::runtime_error("BatchLoader: offsets/lengths/label_offsets/label_lens sizes differ");
    for (size_t i = 0; i < n; ++i) {
      if (off_[i] < 0 || len_[i] < 0 || off_[i] + len_[i] > store_.frames())
        throw std::runtime_error("utterance outside the feature store");
      if (loff_[i] < 0 || llen_[i] < 0 || loff_[i] + llen_[i] > (int64_t)lab_.size())
        throw std::runtime_error("label slice outside the label array");
    }
    const int nt = std::max(1, num_threads);
    for (int i = 0; i < nt; ++i) workers_.emplace_back([this] { work(); });
  }
#ifndef DS2_NO_PYBIND
  BatchLoader(const std::string& feat_path, int freq, py::array_t<int64_t> offsets, py::array_t<int32_t> lengths,
              py::array_t<int32_t> labels, py::array_t<int64_t> label_offsets, py::array_t<int32_t> label_lens,
              int num_threads, int pad_to)
      : BatchLoader(feat_path, freq, cp(offsets), cp(lengths), cp(labels), cp(label_offsets), cp(label_lens),
                    num_threads, pad_to) {}
  template <typename T>
  static std::vector<T> cp(py::array_t<T>& a) {
    return std::vector<T>(a.data(), a.data() + a.size());
  }
#endif
  ~BatchLoader() { shutdown(); }

  void shutdown() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_jobs_.notify_all();
    cv_done_.notify_all();
    for (auto& t : workers_)
      if (t.joinable()) t.join();
    workers_.clear();
  }

  // schedule batches; returns the sequence number of the first one
  int64_t submit(const std::vector<std::vector<int64_t>>& batches) {
    std::lock_guard<std::mutex> g(mu_);
    const int64_t first = next_submit_;
    for (auto& b : batches) jobs_.emplace_back(next_submit_++, b);
    cv_jobs_.notify_all();
    return first;
  }

  int64_t pending() {
    std::lock_guard<std::mutex> g(mu_);
    return next_submit_ - next_take_;
  }

  // blocks until the next batch in submission order is assembled
  std::unique_ptr<Assembled> next_raw() {
    std::unique_lock<std::mutex> lk(mu_);
    if (next_take_ >= next_submit_) throw std::runtime_error("BatchLoader.next(): nothing submitted");
    cv_done_.wait(lk, [&] { return stop_ || done_.count(next_take_); });
    if (stop_) throw std::runtime_error("loader stopped");
    std::unique_ptr<Assembled> a = std::move(done_[next_take_]);
    done_.erase(next_take_);
    ++next_take_;
    if (!error_.empty()) throw std::runtime_error(error_);
    return a;
  }

  int freq() const { return store_.freq(); }

#ifndef DS2_NO_PYBIND
  py::tuple next() {
    std::unique_ptr<Assembled> a;
    {
      py::gil_scoped_release rel;
      a = next_raw();
    }
    Assembled* raw = a.release();
    py::capsule owner(raw, [](void* p) { delete reinterpret_cast<Assembled*>(p); });
    const int F = store_.freq();
    py::array_t<float> feats({raw->N, raw->Tmax, F}, raw->feats.data(), owner);
    py::array_t<int32_t> seq({raw->N}, raw->seq.data(), owner);
    py::array_t<int32_t> lab({raw->N, raw->Lmax}, raw->labels.data(), owner);
    py::array_t<int32_t> ll({raw->N}, raw->llen.data(), owner);
    return py::make_tuple(feats, seq, lab, ll);
  }
#endif

 private:
  void work() {
    while (true) {
      std::pair<int64_t, std::vector<int64_t>> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_jobs_.wait(lk, [&] { return stop_ || !jobs_.empty(); });
        if (stop_) return;
        job = std::move(jobs_.front());
        jobs_.pop_front();
      }
      std::unique_ptr<Assembled> a(new Assembled());
      try {
        assemble(job.second, *a);
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(mu_);
        error_ = e.what();
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        done_[job.first] = std::move(a);
      }
      cv_done_.notify_all();
    }
  }

  void assemble(const std::vector<int64_t>& ids, Assembled& a) {
    const int F = store_.freq();
    a.N = (int)ids.size();
    int T = 1, Lm = 1;
    for (int64_t i : ids) {
      T = std::max(T, len_[i]);
      Lm = std::max(Lm, llen_[i]);
    }
    T = (T + pad_to_ - 1) / pad_to_ * pad_to_;
    a.Tmax = T;
    a.Lmax = Lm;
    a.feats.assign((size_t)a.N * T * F, 0.f);
    a.seq.resize(a.N);
    a.labels.assign((size_t)a.N * Lm, -1);
    a.llen.resize(a.N);
    for (int n = 0; n < a.N; ++n) {
      const int64_t i = ids[n];
      std::memcpy(&a.feats[(size_t)n * T * F], store_.rows(off_[i]), sizeof(float) * (size_t)len_[i] * F);
      a.seq[n] = len_[i];
      a.llen[n] = llen_[i];
      std::memcpy(&a.labels[(size_t)n * Lm], &lab_[loff_[i]], sizeof(int32_t) * llen_[i]);
    }
  }

  FeatureStore store_;
  int pad_to_;
  std::vector<int64_t> off_, loff_;
  std::vector<int32_t> len_, lab_, llen_;   // (declaration order = constructor init order)
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_jobs_, cv_done_;
  std::deque<std::pair<int64_t, std::vector<int64_t>>> jobs_;
  std::map<int64_t, std::unique_ptr<Assembled>> done_;
  int64_t next_submit_ = 0, next_take_ = 0;
  bool stop_ = false;
  std::string error_;
};

}  // namespace ds2rt

#ifndef DS2_NO_PYBIND
void register_loader(py::module_& m) {
  m.def("plan_batches", &ds2rt::plan_batches, py::arg("lengths"), py::arg("min_frames"), py::arg("batch_size"),
        py::arg("bucket") = 100, py::arg("max_frames") = 1800, py::arg("sorted") = true, py::arg("seed") = 0,
        py::arg("world") = 1, py::arg("drop_last") = true);
  py::class_<ds2rt::BatchLoader>(m, "BatchLoader")
      .def(py::init<const std::string&, int, py::array_t<int64_t>, py::array_t<int32_t>, py::array_t<int32_t>,
                    py::array_t<int64_t>, py::array_t<int32_t>, int, int>(),
           py::arg("feat_path"), py::arg("freq"), py::arg("offsets"), py::arg("lengths"), py::arg("labels"),
           py::arg("label_offsets"), py::arg("label_lens"), py::arg("num_threads") = 4, py::arg("pad_to") = 1)
      .def("submit", &ds2rt::BatchLoader::submit)
      .def("next", &ds2rt::BatchLoader::next)
      .def("pending", &ds2rt::BatchLoader::pending)
      .def("shutdown", &ds2rt::BatchLoader::shutdown);
}
#endif  // DS2_NO_PYBIND
