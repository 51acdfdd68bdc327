// CTC prefix beam search on the GPU (SURVEY K15 "beam later"; VERDICT r5 missing item 4).
//
// The host version (runtime/decoder.cpp PrefixBeamSearch) keeps a trie in a hash map and, with
// a near-uniform frame (a young model, all 29 classes within the prune window), creates ~450 trie
// nodes per frame per stream; with 32 streams that host loop, plus the per-chunk log-prob copy
// and sync, made beam-16 cost 2.6x the greedy decode in streaming inference. Here the beams stay
// on the device between chunks and one wave64 decodes one stream:
//
//   * lane i < nbeam holds hypothesis i (trie node, last label, parent node, log p ending in
//     blank / non-blank); lane k < K holds class k's log-prob of the frame;
//   * merging needs no hash map: distinct hypotheses have distinct prefixes, so the extension
//     of hypothesis j by label k reaches an existing prefix only when some hypothesis i has
//     parent(i) == node(j) and last(i) == k; it then adds into i's "stay" entry (CPU: the
//     same get(node) slot), otherwise it is a new prefix whose trie node is created only if it
//     survives the top-W selection;
//   * lane k scores the W extensions by class k (the hypotheses broadcast with readlane), the
//     selection is W rounds of a wave arg-max (ties: lower candidate id; stays before
//     extensions), and the survivors' new trie nodes (parent, label) are appended to the
//     stream's node table, which the backtrack kernel walks at the end.
//
// Every score is a log_add of at most two terms (own stay + one merged extension) or one term,
// so the float results do not depend on accumulation order; they equal the host decoder's up
// to the ulps of expf / log1pf. Reference semantics: tf.nn.ctc_beam_search_decoder (the
// reference itself decodes greedily, src/deepSpeech_test.py:212-215).
#include "common.h"

using namespace ds2;

namespace {

constexpr int BM_MAXW = 32;   // beam width bound (lane registers per class lane)

__device__ __forceinline__ float log_add(float a, float b) {
  if (a == -INFINITY) return b;
  if (b == -INFINITY) return a;
  const float m = fmaxf(a, b);
  return m + log1pf(expf(-fabsf(a - b)));
}

struct BeamArgs {
  const float* lp;     // [T][B][K] log-probs (time-major)
  const int* frames;   // [B] frames of this call per stream (<= T), nullptr: T for every stream
  int T, B, K, W, blank;
  float prune;         // classes below (frame max + prune) are not extended (<= 0)
  int* node;           // [B][W] trie node of each hypothesis (0 = empty prefix)
  int* last;           // [B][W] last label (-1: empty prefix)
  int* parent;         // [B][W] parent trie node (-1: empty prefix)
  float* pb;           // [B][W] log p(prefix, ends in blank)
  float* pnb;          // [B][W] log p(prefix, ends in a label)
  int* nbeam;          // [B] live hypotheses
  int2* nodes;         // [B][cap] trie nodes: (parent, label)
  int* nnodes;         // [B] nodes used
  int cap;
  unsigned* err;       // bit 1: node table full (host sizes it: 1 + W * frames)
};

__device__ __forceinline__ float bcast(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
__device__ __forceinline__ int bcast(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

__global__ __launch_bounds__(256) void ctc_beam_kernel(BeamArgs a) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (b >= a.B) return;                                // the whole wave leaves together
  const int W = a.W, K = a.K;
  const size_t bo = (size_t)b * W;
  int nb = a.nbeam[b];
  int nn = a.nnodes[b];
  int h_node = 0, h_last = -1, h_par = -1;
  float h_pb = -INFINITY, h_pnb = -INFINITY;
  if (lane < nb) {
    h_node = a.node[bo + lane];
    h_last = a.last[bo + lane];
    h_par = a.parent[bo + lane];
    h_pb = a.pb[bo + lane];
    h_pnb = a.pnb[bo + lane];
  }
  int2* const tab = a.nodes + (size_t)b * a.cap;
  const int T = a.frames ? min(a.frames[b], a.T) : a.T;
  for (int t = 0; t < T; ++t) {
    if (nn + W > a.cap) {                              // cannot happen when the host sized it
      if (lane == 0) atomicOr(a.err, 1u);
      break;
    }
    const float p = lane < K ? a.lp[((size_t)t * a.B + b) * K + lane] : -INFINITY;
    float mx = p;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    const unsigned long long cmask = __ballot(lane < K && p >= mx + a.prune);
    const bool live = lane < nb;
    const float tot = live ? log_add(h_pb, h_pnb) : -INFINITY;
    // merge source of my hypothesis (the one whose extension by my last label is my prefix),
    // and the labels whose extension of MY prefix lands on an existing hypothesis
    int msrc = -1;
    unsigned long long mmask = 0ull;
    for (int i = 0; i < nb; ++i) {
      const int ni = bcast(h_node, i), pi = bcast(h_par, i), li = bcast(h_last, i);
      if (live && h_par >= 0 && ni == h_par) msrc = i;
      if (pi >= 0 && pi == h_node && live) mmask |= 1ull << li;
    }
    // stay entry of my hypothesis: blank, a repeat of the last label, and the merged extension
    const float pblank = __shfl(p, a.blank, 64);
    const float plast = __shfl(p, h_last >= 0 ? h_last : 0, 64);
    const int ms = msrc >= 0 ? msrc : 0;
    const float m_pb = __shfl(h_pb, ms, 64), m_tot = __shfl(tot, ms, 64);
    const int m_last = __shfl(h_last, ms, 64);
    float s_pb = -INFINITY, s_pnb = -INFINITY;
    if (live) {
      if ((cmask >> a.blank) & 1ull) s_pb = tot + pblank;
      if (h_last >= 0 && ((cmask >> h_last) & 1ull)) {
        s_pnb = h_pnb + plast;
        if (msrc >= 0) s_pnb = log_add(s_pnb, (m_last == h_last ? m_pb : m_tot) + plast);
      }
    }
    float stay = live ? log_add(s_pb, s_pnb) : -INFINITY;
    // lane k: the extensions of every hypothesis j by class k that are new prefixes
    float ext[BM_MAXW];
    const bool kc = lane < K && lane != a.blank && ((cmask >> lane) & 1ull);
#pragma unroll
    for (int j = 0; j < BM_MAXW; ++j) {
      ext[j] = -INFINITY;
      if (j < nb) {
        const float tj = bcast(tot, j), pj = bcast(h_pb, j);
        const int lj = bcast(h_last, j);
        const unsigned long long mj = ((unsigned long long)(unsigned)bcast((int)(mmask >> 32), j) << 32) |
                                      (unsigned)bcast((int)mmask, j);
        if (kc && !((mj >> lane) & 1ull)) ext[j] = (lane == lj ? pj : tj) + p;
      }
    }
    // top-W: stays have ids 0..W-1, extension (j, k) id W + j * 64 + k
    int nsel = 0, newn = 0;
    int n_node = 0, n_last = -1, n_par = -1;
    float n_pb = -INFINITY, n_pnb = -INFINITY;
    for (int r = 0; r < W; ++r) {
      float best = stay;
      int bid = live ? lane : 0x7fffffff;
#pragma unroll
      for (int j = 0; j < BM_MAXW; ++j)
        if (ext[j] > best) {                           // ids grow with j: strict > keeps the lowest
          best = ext[j];
          bid = W + j * 64 + lane;
        }
      if (best == -INFINITY) bid = 0x7fffffff;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bid, o, 64);
        if (ob > best || (ob == best && oi < bid)) {
          best = ob;
          bid = oi;
        }
      }
      bid = __builtin_amdgcn_readfirstlane(bid);
      if (bid == 0x7fffffff) break;                    // fewer than W finite candidates
      if (bid < W) {
        const int j = bid;
        if (lane == j) stay = -INFINITY;
        const int nj = bcast(h_node, j), lj = bcast(h_last, j), pj = bcast(h_par, j);
        const float bj = bcast(s_pb, j), qj = bcast(s_pnb, j);
        if (lane == r) {
          n_node = nj;
          n_last = lj;
          n_par = pj;
          n_pb = bj;
          n_pnb = qj;
        }
      } else {
        const int e = bid - W, j = e >> 6, k = e & 63;
        if (lane == k) {
#pragma unroll
          for (int q = 0; q < BM_MAXW; ++q)
            if (q == j) ext[q] = -INFINITY;
        }
        const int nj = bcast(h_node, j);
        const int id = nn + newn;
        ++newn;
        if (lane == r) {
          n_node = id;
          n_last = k;
          n_par = nj;
          n_pb = -INFINITY;
          n_pnb = best;
          tab[id] = make_int2(nj, k);
        }
      }
      ++nsel;
    }
    nb = nsel;
    nn += newn;
    h_node = n_node;
    h_last = n_last;
    h_par = n_par;
    h_pb = n_pb;
    h_pnb = n_pnb;
  }
  if (lane < W) {
    a.node[bo + lane] = h_node;
    a.last[bo + lane] = h_last;
    a.parent[bo + lane] = h_par;
    a.pb[bo + lane] = h_pb;
    a.pnb[bo + lane] = h_pnb;
  }
  if (lane == 0) {
    a.nbeam[b] = nb;
    a.nnodes[b] = nn;
  }
}

// labels of every live hypothesis: out [B][W][Lcap] (reversed walk written back to front),
// out_len [B][W] (-1: no such hypothesis), score [B][W] = log_add(pb, pnb)
__global__ __launch_bounds__(64) void ctc_beam_backtrack_kernel(const int2* nodes, int cap, const int* node,
                                                                  const int* nbeam, const float* pb, const float* pnb,
                                                                  int B, int W, int* out, int* out_len, float* score,
                                                                  int Lcap) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= B * W) return;
  const int b = i / W, h = i - b * W;
  if (h >= nbeam[b]) {
    out_len[i] = -1;
    score[i] = -INFINITY;
    return;
  }
  const int2* tab = nodes + (size_t)b * cap;
  int len = 0;
  for (int n = node[i]; n > 0 && len <= Lcap; n = tab[n].x) ++len;
  const int L = min(len, Lcap);
  int pos = L;
  for (int n = node[i]; n > 0 && pos > 0; n = tab[n].x) out[(size_t)i * Lcap + --pos] = tab[n].y;
  out_len[i] = L;
  score[i] = log_add(pb[i], pnb[i]);
}

}  // namespace

extern "C" int ds2_ctc_beam(const float* lp, const int* frames, int T, int B, int K, int W, int blank, float prune,
                            int* node, int* last, int* parent, float* pb, float* pnb, int* nbeam, void* nodes,
                            int* nnodes, int cap, unsigned* err, hipStream_t st) {
  if (K < 2 || K > 64 || W < 1 || W > BM_MAXW || blank < 0 || blank >= K || B < 1 || T < 0 || cap < 1) return -50;
  if (T == 0) return 0;
  BeamArgs a{lp, frames, T, B, K, W, blank, prune, node, last, parent, pb, pnb, nbeam,
             static_cast<int2*>(nodes), nnodes, cap, err};
  ds2_launch(ctc_beam_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

extern "C" int ds2_ctc_beam_backtrack(const void* nodes, int cap, const int* node, const int* nbeam, const float* pb,
                                      const float* pnb, int B, int W, int* out, int* out_len, float* score, int Lcap,
                                      hipStream_t st) {
  if (B < 1 || W < 1 || Lcap < 1) return -50;
  ds2_launch(ctc_beam_backtrack_kernel, dim3((unsigned)((B * W + 63) / 64)), dim3(64), 0, st,
             static_cast<const int2*>(nodes), cap, node, nbeam, pb, pnb, B, W, out, out_len, score, Lcap);
  return (int)hipGetLastError();
}
