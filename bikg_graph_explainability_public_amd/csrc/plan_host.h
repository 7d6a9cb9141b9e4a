// Host-side receptive-field planner of a ForwardPlan (engine.plan_arrays): frontiers and the
// per-layer / degree CSRs the forward kernels read (include/xpgnn.h, xpg_plan_arrays_build).
// Plain C++ on the host: a plan of a ~1k-node computational subgraph is a few thousand integer
// operations, which numpy spent ~0.4 ms of call overhead on per Explainer.run query.
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>

namespace planhost {

struct Csr {
  std::vector<int64_t> ptr, src, eid, smul, sptr, seid;
};

struct Arrays {
  std::vector<std::vector<int64_t>> fr;  // frontiers [L + 1]
  Csr deg;                               // in-edges of every F_0 node (source node ids)
  std::vector<Csr> lay;                  // layer l: in-edges of F_l targets (source F_0 positions)
};

// In-edges (self-loops apart) of the targets tpos[node] >= 0, relation by relation, grouped by
// target position, original edge order inside a target (a stable counting sort: numpy's stable
// argsort of the target keys), absolute offsets across relations; self-loops counted per target
// (smul) with their edge columns in the self CSR.  Sources are node ids (map = nullptr) or
// map[node].
inline void build_csr(int32_t n_rel, const int64_t* rel_ptr, const int64_t* src, const int64_t* dst,
                      const int64_t* eid, const std::vector<int64_t>& tpos, int64_t n_t, const int64_t* map,
                      Csr& out) {
  int64_t off = 0, soff = 0;
  std::vector<int64_t> cnt(n_t), lcnt(n_t), nxt(n_t), lnxt(n_t);
  for (int32_t r = 0; r < n_rel; ++r) {
    std::fill(cnt.begin(), cnt.end(), 0);
    std::fill(lcnt.begin(), lcnt.end(), 0);
    const int64_t e0 = rel_ptr[r], e1 = rel_ptr[r + 1];
    for (int64_t e = e0; e < e1; ++e) {
      const int64_t t = tpos[dst[e]];
      if (t < 0) continue;
      if (src[e] != dst[e]) ++cnt[t]; else ++lcnt[t];
    }
    int64_t run = off, lrun = soff;
    out.ptr.push_back(run);
    out.sptr.push_back(lrun);
    for (int64_t t = 0; t < n_t; ++t) {
      nxt[t] = run;
      lnxt[t] = lrun;
      run += cnt[t];
      lrun += lcnt[t];
      out.ptr.push_back(run);
      out.sptr.push_back(lrun);
      out.smul.push_back(lcnt[t]);
    }
    out.src.resize(run);
    out.eid.resize(run);
    out.seid.resize(lrun);
    for (int64_t e = e0; e < e1; ++e) {
      const int64_t t = tpos[dst[e]];
      if (t < 0) continue;
      const int64_t col = eid ? eid[e] : 0;
      if (src[e] != dst[e]) {
        const int64_t k = nxt[t]++;
        out.src[k] = map ? map[src[e]] : src[e];
        out.eid[k] = col;
      } else {
        out.seid[lnxt[t]++] = col;
      }
    }
    off = run;
    soff = lrun;
  }
}

// frontiers[L] = queries; frontiers[l - 1] = frontiers[l] + the sorted new in-neighbours (every
// relation), so each frontier is a prefix of the one below it and of F_0.
inline void build(int64_t S, int32_t n_rel, const int64_t* rel_ptr, const int64_t* src, const int64_t* dst,
                  const int64_t* eid, const int64_t* queries, int64_t nq, int32_t L, Arrays& A) {
  const int64_t E = rel_ptr[n_rel];
  A.fr.assign(L + 1, {});
  A.fr[L].assign(queries, queries + nq);
  std::vector<uint8_t> mark(S), seen(S);
  for (int32_t lvl = L; lvl > 0; --lvl) {
    const std::vector<int64_t>& cur = A.fr[lvl];
    std::fill(mark.begin(), mark.end(), 0);
    for (int64_t v : cur) mark[v] = 1;
    std::vector<int64_t> nb;
    for (int64_t e = 0; e < E; ++e) {
      if (!mark[dst[e]]) continue;
      const int64_t s = src[e];
      if (!mark[s] && !seen[s]) {
        seen[s] = 1;
        nb.push_back(s);
      }
    }
    for (int64_t s : nb) seen[s] = 0;
    std::sort(nb.begin(), nb.end());
    std::vector<int64_t>& next = A.fr[lvl - 1];
    next = cur;
    next.insert(next.end(), nb.begin(), nb.end());
  }
  const int64_t n0 = static_cast<int64_t>(A.fr[0].size());
  std::vector<int64_t> pos0(S, -1);
  for (int64_t i = 0; i < n0; ++i) pos0[A.fr[0][i]] = i;
  build_csr(n_rel, rel_ptr, src, dst, eid, pos0, n0, nullptr, A.deg);
  A.lay.assign(L, {});
  std::vector<int64_t> tpos(S, -1);
  for (int32_t lvl = 1; lvl <= L; ++lvl) {
    std::fill(tpos.begin(), tpos.end(), -1);
    const std::vector<int64_t>& f = A.fr[lvl];
    for (int64_t i = 0; i < static_cast<int64_t>(f.size()); ++i) tpos[f[i]] = i;
    // sources of F_l targets lie in F_{l-1}, a prefix of F_0: their F_{l-1} and F_0 positions agree
    build_csr(n_rel, rel_ptr, src, dst, eid, tpos, static_cast<int64_t>(f.size()), pos0.data(), A.lay[lvl - 1]);
  }
}

}  // namespace planhost
