// Host-runtime sanitizer driver (race detection / sanitizers).
//
// Builds the pybind-free cores of deepspeech_amd/runtime/*.cpp (DS2_NO_PYBIND) into one
// executable and exercises them the way the training / inference paths do, including the
// threaded parts, so that
//   g++ -fsanitize=address,undefined  catches out-of-bounds / use-after-free / UB, and
//   g++ -fsanitize=thread             catches data races in the loader's worker pool and
//                                     the multi-threaded beam search.
// tests/test_sanitizers.py compiles and runs both builds (host code only: GPU sanitizers
// and XNACK are not available on the MI355X pool).
#define DS2_NO_PYBIND 1
#include "../../deepspeech_amd/runtime/decoder.cpp"
#include "../../deepspeech_amd/runtime/loader.cpp"
#include "../../deepspeech_amd/runtime/tfrecord.cpp"

#include <cstdio>
#include <cstdlib>
#include <random>

using namespace ds2rt;

static int failures = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                       \
    }                                                                   \
  } while (0)

static std::string tmp_path(const char* name) {
  const char* d = std::getenv("DS2_SAN_TMP");
  return std::string(d ? d : "/tmp") + "/" + name;
}

static void test_tfrecord(std::mt19937& rng) {
  // SequenceExample round trip through the TFRecord framing
  std::vector<std::string> recs;
  std::vector<SeqExample> want;
  for (int r = 0; r < 6; ++r) {
    SeqExample ex;
    ex.T = 1 + (int)(rng() % 40);
    ex.F = 161;
    ex.feats.resize((size_t)ex.T * ex.F);
    for (auto& v : ex.feats) v = (float)(rng() % 1000) / 7.f;
    const int L = (int)(rng() % 30);
    std::vector<int64_t> lab(L);
    for (auto& v : lab) v = (int64_t)(rng() % 29);
    ex.labels.assign(lab.begin(), lab.end());
    ex.seq_len = ex.T;
    recs.push_back(make_sequence_example_raw(ex.seq_len, ex.feats.data(), ex.T, ex.F, lab.data(), lab.size(), "feats"));
    want.push_back(ex);
  }
  const std::string path = tmp_path("ds2_san.tfrecord");
  write_records(path, recs);
  const std::vector<std::string> back = read_records_raw(path, true);
  CHECK(back.size() == recs.size());
  for (size_t i = 0; i < back.size() && i < want.size(); ++i) {
    const SeqExample ex =
        parse_sequence_example_raw(reinterpret_cast<const uint8_t*>(back[i].data()), back[i].size(), "feats");
    CHECK(ex.T == want[i].T && ex.F == want[i].F && ex.seq_len == want[i].seq_len);
    CHECK(ex.labels == want[i].labels);
    CHECK(ex.feats == want[i].feats);
  }
  // truncated / corrupted inputs must throw, never read out of bounds
  int threw = 0;
  for (int trial = 0; trial < 400; ++trial) {
    std::string s = recs[trial % recs.size()];
    if (trial % 2) s.resize(rng() % (s.size() + 1));
    else if (!s.empty()) s[rng() % s.size()] = (char)(rng() & 0xFF);
    try {
      parse_sequence_example_raw(reinterpret_cast<const uint8_t*>(s.data()), s.size(), "feats");
    } catch (const std::exception&) {
      ++threw;
    }
  }
  CHECK(threw > 0);
  std::remove(path.c_str());
}

static void test_decoders(std::mt19937& rng) {
  const int T = 60, N = 9, K = 29;
  std::vector<float> lp((size_t)T * N * K);
  std::uniform_real_distribution<float> u(-6.f, 0.f);
  for (auto& v : lp) v = u(rng);
  std::vector<int> lens(N);
  for (int n = 0; n < N; ++n) lens[n] = (int)(rng() % (T + 5));   // some exceed T (clamped)
  // multi-threaded batch beam search == the same search on one thread
  const auto a = beam_search_batch_raw(lp.data(), T, N, K, lens.data(), 8, K - 1, -8.f, 4);
  const auto b = beam_search_batch_raw(lp.data(), T, N, K, lens.data(), 8, K - 1, -8.f, 1);
  CHECK(a == b);
  // streaming: the same frames fed in chunks give the same result as one feed
  BatchBeamSearch s(N, 8, K - 1, -8.f, 3);
  const int chunk = 7;
  for (int t0 = 0; t0 < T; t0 += chunk) {
    const int tc = std::min(chunk, T - t0);
    std::vector<int> cl(N);
    for (int n = 0; n < N; ++n) cl[n] = std::max(0, std::min(tc, std::min(lens[n], T) - t0));
    s.feed_raw(lp.data() + (size_t)t0 * N * K, tc, N, K, cl.data());
  }
  CHECK(s.best() == a);
  // greedy collapse + edit distance
  std::vector<int> best((size_t)T * N);
  for (auto& v : best) v = (int)(rng() % K);
  const auto g = greedy_collapse_raw(best.data(), T, N, lens.data(), K - 1);
  CHECK((int)g.size() == N);
  CHECK(levenshtein_ids(g[0], g[0]) == 0);
  CHECK(levenshtein_str("kitten", "sitting") == 3);
}

static void test_loader(std::mt19937& rng) {
  const int F = 17, U = 64;
  std::vector<int64_t> off(U), loff(U);
  std::vector<int32_t> len(U), llen(U), lab;
  int64_t frames = 0;
  for (int i = 0; i < U; ++i) {
    len[i] = 5 + (int)(rng() % 200);
    off[i] = frames;
    frames += len[i];
    llen[i] = (int)(rng() % 20);
    loff[i] = (int64_t)lab.size();
    for (int j = 0; j < llen[i]; ++j) lab.push_back((int32_t)(rng() % 28));
  }
  std::vector<float> store((size_t)frames * F);
  for (size_t i = 0; i < store.size(); ++i) store[i] = (float)(i % 9973);
  const std::string path = tmp_path("ds2_san.feats");
  {
    FILE* f = std::fopen(path.c_str(), "wb");
    std::fwrite(store.data(), sizeof(float), store.size(), f);
    std::fclose(f);
  }
  std::vector<int> mf(U, 0);
  const auto plan = plan_batches_raw(len.data(), mf.data(), U, 8, 50, 1000, false, 7, 2, false);
  size_t covered = 0;
  for (const auto& b : plan) covered += b.size();
  CHECK(covered == (size_t)U);
  {
    BatchLoader ld(path, F, off, len, lab, loff, llen, 4, 8);
    ld.submit(plan);
    for (size_t k = 0; k < plan.size(); ++k) {
      std::unique_ptr<Assembled> a = ld.next_raw();
      CHECK(a->N == (int)plan[k].size());
      CHECK(a->Tmax % 8 == 0);
      for (int n = 0; n < a->N; ++n) {
        const int64_t i = plan[k][n];
        CHECK(a->seq[n] == len[i]);
        CHECK(a->feats[(size_t)n * a->Tmax * F] == store[(size_t)off[i] * F]);
        if (llen[i] > 0) CHECK(a->labels[(size_t)n * a->Lmax] == lab[loff[i]]);
      }
    }
    // resubmit and shut down with work in flight (destructor joins the pool)
    ld.submit(plan);
  }
  // inconsistent index arrays are rejected before any worker touches them
  bool threw = false;
  try {
    std::vector<int32_t> bad = llen;
    bad[3] = 1 << 20;
    BatchLoader ld(path, F, off, len, lab, loff, bad, 2, 1);
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
  std::remove(path.c_str());
}

int main() {
  std::mt19937 rng(1234);
  test_tfrecord(rng);
  test_decoders(rng);
  test_loader(rng);
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("sanitize_driver ok\n");
  return 0;
}
