// khop.hip — k-hop computational-subgraph extraction on the GPU, included at the
// end of xpgnn.hip (shares its error plumbing and launch helpers).
//
// Replaces Data.comp_graph's call of PyG 2.0.4 k_hop_subgraph (data.py:331-333,
// flow='source_to_target', relabel_nodes=True):
//   frontier_0 = {seed};  frontier_{h+1} = { src[e] : dst[e] ∈ frontier_h }   (h < hops)
//   subset     = sorted ∪_h frontier_h;   inv = position of the seed in subset
//   edge_mask  = subset[src] ∧ subset[dst] (original edge order);  sub_ei = relabel(ei[:, edge_mask])
//
// Layout: the graph is the caller's COO edge_index (int64 [2][E], torch's own layout; no CSR
// is built).  Per hop one streaming pass over dst (8 B/edge) with byte-flag lookups into the
// frontier (N bytes, L2-resident at 1M nodes); the relabel and the ordered edge compaction are
// ballot-scanned stream compactions (wave = 16 rows of 64 items, block = 4 waves, one
// exclusive scan over the block totals).  HBM bound: ≈ hops·8E + 17E + kept·24 bytes.
namespace {

constexpr int kKhRows = 16;                         // ballot rows per wave
constexpr int kKhBlock = 256;                       // 4 waves
constexpr int kKhItems = kKhRows * kKhBlock;        // items per block (4096)

struct KhopWs {                                      // carve-up of the caller's workspace
  uint8_t *cur, *nxt, *inset;
  int32_t* remap;
  int64_t *node_off, *edge_off;
  int64_t n_pad, nb_nodes, nb_edges;
};

KhopWs khop_layout(void* base, int64_t n_nodes, int64_t n_edges, size_t* bytes) {
  KhopWs w{};
  w.nb_nodes = cdiv(n_nodes, kKhItems);
  w.nb_edges = std::max<int64_t>(1, cdiv(n_edges, kKhItems));
  w.n_pad = w.nb_nodes * kKhItems;
  size_t off = 0;
  auto take = [&](size_t b) { size_t o = off; off += (b + 255) & ~size_t(255); return o; };
  const size_t o_cur = take(w.n_pad), o_nxt = take(w.n_pad), o_in = take(w.n_pad);
  const size_t o_rm = take(sizeof(int32_t) * w.n_pad);
  const size_t o_no = take(sizeof(int64_t) * (w.nb_nodes + 1));
  const size_t o_eo = take(sizeof(int64_t) * (w.nb_edges + 1));
  if (bytes) *bytes = off;
  if (base) {
    char* p = static_cast<char*>(base);
    w.cur = reinterpret_cast<uint8_t*>(p + o_cur);
    w.nxt = reinterpret_cast<uint8_t*>(p + o_nxt);
    w.inset = reinterpret_cast<uint8_t*>(p + o_in);
    w.remap = reinterpret_cast<int32_t*>(p + o_rm);
    w.node_off = reinterpret_cast<int64_t*>(p + o_no);
    w.edge_off = reinterpret_cast<int64_t*>(p + o_eo);
  }
  return w;
}

// one hop: every edge whose target is in the current frontier puts its source into the next
// frontier and into the subset (byte flags; concurrent stores all write 1)
__global__ __launch_bounds__(256) void k_khop_hop(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                  int64_t n_edges, int64_t n_nodes, const uint8_t* __restrict__ cur,
                                                  uint8_t* __restrict__ nxt, uint8_t* __restrict__ inset,
                                                  int64_t* __restrict__ bad) {
  const int64_t base = static_cast<int64_t>(blockIdx.x) * (256 * 8) + threadIdx.x;
  int64_t d[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t e = base + k * 256;
    d[k] = e < n_edges ? __builtin_nontemporal_load(dst + e) : 0;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t e = base + k * 256;
    if (e >= n_edges) continue;
    if (static_cast<uint64_t>(d[k]) >= static_cast<uint64_t>(n_nodes)) {  // out-of-range id: flag, skip
      *bad = 1;
      continue;
    }
    if (cur[d[k]]) {
      const int64_t s = src[e];
      if (static_cast<uint64_t>(s) >= static_cast<uint64_t>(n_nodes)) {
        *bad = 1;
        continue;
      }
      nxt[s] = 1;
      inset[s] = 1;
    }
  }
}

__device__ __forceinline__ uint64_t lanes_below() {
  return (1ull << (threadIdx.x & 63)) - 1ull;
}

// block-exclusive offsets of the 4 wave totals; returns this wave's offset, *total = block sum
__device__ __forceinline__ int64_t khop_wave_offsets(int64_t wave_total, int64_t* total) {
  __shared__ int64_t tot[4];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) tot[wave] = wave_total;
  __syncthreads();
  int64_t off = 0;
  for (int w = 0; w < wave; ++w) off += tot[w];
  *total = tot[0] + tot[1] + tot[2] + tot[3];
  return off;
}

// item (block b, wave w, row r, lane l) = b*4096 + w*1024 + r*64 + l: consecutive lanes read
// consecutive items, a wave's 16 rows are consecutive, so the ballot order is the item order
__device__ __forceinline__ int64_t kh_item(int r) {
  return static_cast<int64_t>(blockIdx.x) * kKhItems + (threadIdx.x >> 6) * (kKhRows * 64) + r * 64 +
         (threadIdx.x & 63);
}

__global__ __launch_bounds__(256) void k_khop_count_nodes(const uint8_t* __restrict__ inset, int64_t* __restrict__ blk) {
  int64_t n = 0;
#pragma unroll
  for (int r = 0; r < kKhRows; ++r) n += __popcll(__ballot(inset[kh_item(r)] != 0));
  int64_t total;
  khop_wave_offsets(n, &total);
  if (threadIdx.x == 0) blk[blockIdx.x] = total;
}

// flags of the edges inside the subset (written out as edge_mask) and their block counts
__global__ __launch_bounds__(256) void k_khop_count_edges(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                          int64_t n_edges, int64_t n_nodes,
                                                          const uint8_t* __restrict__ inset, uint8_t* __restrict__ emask,
                                                          int64_t* __restrict__ blk, int64_t* __restrict__ bad) {
  int64_t n = 0;
#pragma unroll 4
  for (int r = 0; r < kKhRows; ++r) {
    const int64_t e = kh_item(r);
    bool keep = false;
    if (e < n_edges) {
      const int64_t u = __builtin_nontemporal_load(src + e), v = __builtin_nontemporal_load(dst + e);
      if (static_cast<uint64_t>(u) < static_cast<uint64_t>(n_nodes) &&
          static_cast<uint64_t>(v) < static_cast<uint64_t>(n_nodes))
        keep = inset[u] && inset[v];
      else
        *bad = 1;
      emask[e] = keep;
    }
    n += __popcll(__ballot(keep));
  }
  int64_t total;
  khop_wave_offsets(n, &total);
  if (threadIdx.x == 0) blk[blockIdx.x] = total;
}

// exclusive scan of nb block totals in place (one workgroup); blk[nb] = grand total, also
// written to *total_out
__global__ __launch_bounds__(1024) void k_khop_scan(int64_t* __restrict__ blk, int64_t nb, int64_t* __restrict__ total_out) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int64_t per = (nb + 1023) / 1024;
  const int64_t lo = min(nb, t * per), hi = min(nb, lo + per);
  int64_t s = 0;
  for (int64_t i = lo; i < hi; ++i) s += blk[i];
  part[t] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan
    const int64_t v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = t ? part[t - 1] : 0;
  for (int64_t i = lo; i < hi; ++i) {
    const int64_t v = blk[i];
    blk[i] = run;
    run += v;
  }
  if (t == 1023) {
    blk[nb] = part[1023];
    *total_out = part[1023];
  }
}

// subset = sorted node ids in the subset; remap[v] = new id; inv = remap[seed]
__global__ __launch_bounds__(256) void k_khop_emit_nodes(const uint8_t* __restrict__ inset, const int64_t* __restrict__ blk,
                                                         int64_t seed, int64_t* __restrict__ subset,
                                                         int32_t* __restrict__ remap, int64_t* __restrict__ inv_out) {
  bool f[kKhRows];
  int64_t n = 0;
#pragma unroll
  for (int r = 0; r < kKhRows; ++r) {
    f[r] = inset[kh_item(r)] != 0;
    n += __popcll(__ballot(f[r]));
  }
  int64_t total;
  int64_t pos = blk[blockIdx.x] + khop_wave_offsets(n, &total);
#pragma unroll
  for (int r = 0; r < kKhRows; ++r) {
    const uint64_t m = __ballot(f[r]);
    if (f[r]) {
      const int64_t v = kh_item(r), p = pos + __popcll(m & lanes_below());
      subset[p] = v;
      remap[v] = static_cast<int32_t>(p);
      if (v == seed) *inv_out = p;
    }
    pos += __popcll(m);
  }
}

// ordered compaction of the kept edges, relabelled
__global__ __launch_bounds__(256) void k_khop_emit_edges(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                         int64_t n_edges, const uint8_t* __restrict__ emask,
                                                         const int32_t* __restrict__ remap, const int64_t* __restrict__ blk,
                                                         int64_t* __restrict__ sub_src, int64_t* __restrict__ sub_dst) {
  bool f[kKhRows];
  int64_t n = 0;
#pragma unroll
  for (int r = 0; r < kKhRows; ++r) {
    const int64_t e = kh_item(r);
    f[r] = e < n_edges && emask[e];
    n += __popcll(__ballot(f[r]));
  }
  int64_t total;
  int64_t pos = blk[blockIdx.x] + khop_wave_offsets(n, &total);
#pragma unroll
  for (int r = 0; r < kKhRows; ++r) {
    const uint64_t m = __ballot(f[r]);
    if (f[r]) {
      const int64_t e = kh_item(r), p = pos + __popcll(m & lanes_below());
      sub_src[p] = remap[src[e]];
      sub_dst[p] = remap[dst[e]];
    }
    pos += __popcll(m);
  }
}

}  // namespace

extern "C" {

int xpg_khop_workspace(int64_t n_nodes, int64_t n_edges, size_t* bytes) {
  XPG_REQ(n_nodes > 0 && n_nodes < (int64_t(1) << 31) && n_edges >= 0 && bytes, "khop: bad shape");
  khop_layout(nullptr, n_nodes, n_edges, bytes);
  return XPG_OK;
}

int xpg_khop_subgraph(const int64_t* edge_index, int64_t n_edges, int64_t n_nodes, int64_t seed, int32_t hops,
                      int64_t* subset, int64_t* sub_src, int64_t* sub_dst, uint8_t* edge_mask, int64_t* counts,
                      void* workspace, size_t workspace_bytes, xpg_stream_t stream) {
  XPG_REQ(n_nodes > 0 && n_nodes < (int64_t(1) << 31) && n_edges >= 0 && hops >= 0, "khop: bad shape");
  XPG_REQ(seed >= 0 && seed < n_nodes, "khop: seed node out of range");
  XPG_REQ(subset && counts && workspace && (n_edges == 0 || (edge_index && sub_src && sub_dst && edge_mask)),
          "khop: null buffer");
  size_t need = 0;
  KhopWs w = khop_layout(workspace, n_nodes, n_edges, &need);
  XPG_REQ(workspace_bytes >= need, "khop: workspace too small");
  hipStream_t st = S(stream);
  const int64_t* src = edge_index;
  const int64_t* dst = edge_index + n_edges;
  // cur | nxt | inset are adjacent: one memset clears all three
  XPG_HIP(hipMemsetAsync(w.cur, 0, static_cast<size_t>(w.inset - w.cur) + w.n_pad, st));
  XPG_HIP(hipMemsetAsync(counts, 0, 4 * sizeof(int64_t), st));
  XPG_HIP(hipMemsetAsync(w.cur + seed, 1, 1, st));
  XPG_HIP(hipMemsetAsync(w.inset + seed, 1, 1, st));
  for (int h = 0; h < hops && n_edges > 0; ++h) {
    if (h) XPG_HIP(hipMemsetAsync(w.nxt, 0, w.n_pad, st));
    hipLaunchKernelGGL(k_khop_hop, dim3(static_cast<unsigned>(cdiv(n_edges, 256 * 8))), dim3(256), 0, st, src, dst,
                       n_edges, n_nodes, w.cur, w.nxt, w.inset, counts + 3);
    XPG_LAUNCHED();
    std::swap(w.cur, w.nxt);
  }
  hipLaunchKernelGGL(k_khop_count_nodes, dim3(static_cast<unsigned>(w.nb_nodes)), dim3(kKhBlock), 0, st, w.inset,
                     w.node_off);
  XPG_LAUNCHED();
  hipLaunchKernelGGL(k_khop_scan, dim3(1), dim3(1024), 0, st, w.node_off, w.nb_nodes, counts + 0);
  XPG_LAUNCHED();
  hipLaunchKernelGGL(k_khop_emit_nodes, dim3(static_cast<unsigned>(w.nb_nodes)), dim3(kKhBlock), 0, st, w.inset,
                     w.node_off, seed, subset, w.remap, counts + 2);
  XPG_LAUNCHED();
  if (n_edges == 0) {
    XPG_HIP(hipMemsetAsync(counts + 1, 0, sizeof(int64_t), st));
    return XPG_OK;
  }
  hipLaunchKernelGGL(k_khop_count_edges, dim3(static_cast<unsigned>(w.nb_edges)), dim3(kKhBlock), 0, st, src, dst,
                     n_edges, n_nodes, w.inset, edge_mask, w.edge_off, counts + 3);
  XPG_LAUNCHED();
  hipLaunchKernelGGL(k_khop_scan, dim3(1), dim3(1024), 0, st, w.edge_off, w.nb_edges, counts + 1);
  XPG_LAUNCHED();
  hipLaunchKernelGGL(k_khop_emit_edges, dim3(static_cast<unsigned>(w.nb_edges)), dim3(kKhBlock), 0, st, src, dst,
                     n_edges, edge_mask, w.remap, w.edge_off, sub_src, sub_dst);
  XPG_LAUNCHED();
  return XPG_OK;
}

}  // extern "C"
