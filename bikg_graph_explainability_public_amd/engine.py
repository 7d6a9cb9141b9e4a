"""Device engine: builds receptive-field plans and drives the HIP kernels (libxpgnn.so).

Plan (per query, built once per Explainer.run — DESIGN.md §3):
  F_L = queries; F_{l-1} = F_l ∪ in-neighbours(F_l) (all relations), F_l first so the first
  n_l entries of F_{l-1} are F_l.  Degrees are needed at F_0 (their in-edges reach hop L+1,
  which is why the reference extracts L+1 hops, data.py:325-328).
  Layer-1 tables T_k = X[F_0] W_k^T are computed once by the MFMA dense kernel (features are
  never masked, data.py:582); per mask row only the masked aggregation and the deeper layers
  (aggregate-then-transform on MFMA) run.

All device memory is owned by torch tensors held by the plan; the C-ABI never allocates.
"""
import contextlib
import ctypes
import gc
import itertools
import math

import numpy as np
import torch

from . import _lib
from ._lib import ACT, TERM, ForwardPlanDesc, HeadDesc, LayerDesc, WlmParams, call, ptr


def _rup(x, m):
    return ((int(x) + m - 1) // m) * m


def words_of(cols):
    return (int(cols) + 31) // 32


# ----------------------------------------------------------------------------- masks
def pack_masks(mask: torch.Tensor) -> torch.Tensor:
    """bool/uint8 [rows, cols] device tensor -> row bits uint32 [rows, words] (HIP)."""
    _lib.require_device(mask, "mask")
    m = mask.contiguous()
    if m.dtype == torch.bool:
        m = m.view(torch.uint8)
    rows, cols = m.shape
    bits = torch.empty((rows, words_of(cols)), dtype=torch.int32, device=m.device)
    call("xpg_pack_masks", ptr(m), rows, cols, ptr(bits), _lib.stream_of(m.device))
    return bits


def unpack_masks(bits: torch.Tensor, cols: int) -> torch.Tensor:
    _lib.require_device(bits, "bits")
    rows = bits.shape[0]
    out = torch.empty((rows, cols), dtype=torch.uint8, device=bits.device)
    call("xpg_unpack_masks", ptr(bits), rows, cols, ptr(out), _lib.stream_of(bits.device))
    return out.view(torch.bool)


class CaptureTopologyError(RuntimeError):
    """A stream dependency inside a HIP-graph capture that this HIP stack cannot end."""


@contextlib.contextmanager
def capture_guard():
    """Wrap every HIP-graph capture of the hot path (`with capture_guard(), torch.cuda.graph(g)`).

    1. Freeing a captured graph while another capture runs aborts the process on this HIP stack
       (tools/capture_probe.py, variant graph_gc, profiles/r3_capture_probe.log: the round-2
       `capture_end` crash of the pipelined bench).  A graph object reachable only from a
       reference cycle is freed whenever Python's cyclic collector runs, which can be
       mid-capture; the guard collects first and holds the collector off until the capture
       ends.  The graphs themselves must stay referenced by the caller.
    2. Two side streams that wait on each other in turn segfault hipStreamEndCapture (minimal
       construct, tools/capture_probe.py `pingpong`, profiles/r6_capture_bisect.log: A works;
       B waits A, works; A waits B, works; all joined): the guard tracks the capture's stream
       waits (Stream.wait_stream, Stream.wait_event on a recorded Event) and refuses a wait of
       side stream X on side stream Y once Y has waited on X, with CaptureTopologyError, before
       the wait is made; the side streams are joined to the capture's origin stream first, so
       the capture still ends cleanly (and its graph is not used).  Waits between the origin
       stream (the one current at the first wait) and a side stream are free in both
       directions (the bench's pipelined lanes alternate them)."""
    gc.collect()
    enabled = gc.isenabled()
    gc.disable()
    st = {"origin": None, "waited": {}, "streams": {}, "events": {}}
    S, E = torch.cuda.Stream, torch.cuda.Event
    orig_ws, orig_we, orig_rec = S.wait_stream, S.wait_event, E.record

    def note(x, y):  # stream x is about to wait on stream y
        if not torch.cuda.is_current_stream_capturing():
            return
        if st["origin"] is None:
            cur = torch.cuda.current_stream()
            st["origin"] = cur.cuda_stream
            st["streams"][cur.cuda_stream] = cur
        kx, ky = x.cuda_stream, y.cuda_stream
        st["streams"].setdefault(kx, x)
        st["streams"].setdefault(ky, y)
        if kx == ky:
            return
        o = st["origin"]
        if kx != o and ky != o and kx in st["waited"].get(ky, ()):
            origin = st["streams"][o]
            for k, s_ in st["streams"].items():
                if k != o:
                    orig_ws(origin, s_)
            raise CaptureTopologyError(
                "graph capture: side stream waits on a side stream that waited on it earlier in "
                "the capture (A -> B -> A); hipStreamEndCapture segfaults on such a capture on "
                "this HIP stack (tools/capture_probe.py pingpong).  Route the second wait through "
                "the capture's origin stream.")
        st["waited"].setdefault(kx, set()).add(ky)

    def wait_stream(self, stream):
        note(self, stream)
        return orig_ws(self, stream)

    def wait_event(self, event):
        src = st["events"].get(id(event))
        if src is not None:
            note(self, src)
        return orig_we(self, event)

    def record(self, stream=None):
        st["events"][id(self)] = stream if stream is not None else torch.cuda.current_stream()
        return orig_rec(self, stream)

    S.wait_stream, S.wait_event, E.record = wait_stream, wait_event, record
    try:
        yield
    finally:
        S.wait_stream, S.wait_event, E.record = orig_ws, orig_we, orig_rec
        if enabled:
            gc.enable()


def sample_shapley(seed: int, rows: int, cols: int, device, row_offset: int = 0,
                   with_counts: bool = False):
    """Device Shapley masks (masks.py:231-260 distribution: iid Bernoulli(1/2) bits).

    with_counts=True also returns the per-row popcounts (int32 [rows]) accumulated while
    sampling, for `shap_kernel(..., counts=...)`."""
    bits = torch.empty((rows, words_of(cols)), dtype=torch.int32, device=device)
    st = _lib.stream_of(torch.device(device))
    seed_c = ctypes.c_uint64(int(seed) & (2 ** 64 - 1))
    if not with_counts:
        call("xpg_sample_shapley", seed_c, row_offset, rows, cols, ptr(bits), st)
        return bits
    counts = torch.empty(rows, dtype=torch.int32, device=device)
    call("xpg_sample_shapley_counts", seed_c, row_offset, rows, cols, ptr(bits), ptr(counts), st)
    return bits, counts


def sample_shapley_sets(seeds, rows: int, cols: int, device):
    """len(seeds) independent `sample_shapley(seed, rows, cols)` draws as one [n, rows, words]
    tensor, in one native call (Explainer.run's repeats)."""
    n = len(seeds)
    bits = torch.empty((n, rows, words_of(cols)), dtype=torch.int32, device=device)
    arr = (ctypes.c_uint64 * max(n, 1))(*[int(s) & (2 ** 64 - 1) for s in seeds])
    call("xpg_sample_shapley_sets", arr, n, rows, cols, ptr(bits), _lib.stream_of(torch.device(device)))
    return bits


# torch.get_rng_state() of the CPU generator (at::CPUGeneratorImplState, legacy POD first):
# uint64 the_initial_seed | int32 left | int32 seeded | uint64 next | uint64 state[624] | ...
_RNG_LEFT, _RNG_NEXT, _RNG_STATE = 8, 16, 24


def compat_shapley_bits(rows: int, cols: int):
    """torch.randint(0, 2, (rows, cols), dtype=torch.bool) on torch's global CPU generator
    (masks.py:231-260), bit-identical, as bit-packed int32 [rows, ceil(cols / 32)] rows in host
    memory (pinned when a GPU is present), with the generator advanced past the draw exactly as
    torch would advance it: the library replays the generator's MT19937 state natively
    (xpg_mt19937_mask_bits, host code), without the [rows, cols] bool tensor."""
    raw, state, left, nxt = _rng_get()
    out = torch.empty((rows, words_of(cols)), dtype=torch.int32,
                      pin_memory=torch.cuda.is_available())
    call("xpg_mt19937_mask_bits", state.ctypes.data, left.ctypes.data, nxt.ctypes.data, int(rows),
         int(cols), out.data_ptr() if rows else None)
    _rng_set(raw, state, left, nxt)
    return out


_DRAWS_FORM = []  # [form] once probed: 0 / 1 (see _draws_form), None = no native form matches


def _draws_form():
    """How this torch build evaluates ATen's CPU uniform_real, x * (to - from) + from in float:
    as written (0) or contracted into one fused multiply-add (1) — the ATen kernels compiled for
    an FMA-capable CPU capability contract it, the DEFAULT build does not.  Probed once on a
    private generator (the global one is untouched) against both native forms; None when
    neither reproduces torch (the caller then draws through torch itself)."""
    if not _DRAWS_FORM:
        form = None
        g = torch.Generator().manual_seed(20260101)
        st = g.get_state()
        ref_seed = int(torch.randint(0, 2 ** 62, (1,), generator=g).item())
        ref = torch.empty(1000).uniform_(-0.3, 0.3, generator=g)
        torch.empty((), dtype=torch.int64).random_(generator=g)
        ref_next = torch.rand(3, generator=g)
        for f in (1, 0):
            raw = st.numpy().copy()
            left = raw[_RNG_LEFT:_RNG_LEFT + 4].view(np.int32).copy()
            nxt = np.array([int(raw[_RNG_NEXT:_RNG_NEXT + 8].view(np.uint64)[0])], dtype=np.int32)
            state = raw[_RNG_STATE:_RNG_STATE + 624 * 8].view(np.uint64).astype(np.uint32)
            seeds = np.empty(1, dtype=np.int64)
            w = torch.empty(1000)
            call("xpg_mt19937_repeat_draws", state.ctypes.data, left.ctypes.data, nxt.ctypes.data, 1,
                 1000, -0.3, 0.3, f, seeds.ctypes.data, w.data_ptr())
            raw[_RNG_LEFT:_RNG_LEFT + 4] = left.view(np.uint8)
            raw[_RNG_NEXT:_RNG_NEXT + 8] = np.array([nxt[0]], dtype=np.uint64).view(np.uint8)
            raw[_RNG_STATE:_RNG_STATE + 624 * 8] = state.astype(np.uint64).view(np.uint8)
            g2 = torch.Generator()
            g2.set_state(torch.from_numpy(raw))
            if int(seeds[0]) == ref_seed and torch.equal(w, ref) and \
                    torch.equal(torch.rand(3, generator=g2), ref_next):
                form = f
                break
        _DRAWS_FORM.append(form)
    return _DRAWS_FORM[0]


def repeat_draws(times: int, S: int, fma: int = None):
    """Explainer.run's per-repeat draws on torch's global CPU generator with the device Shapley
    sampler, in the reference's order (explainer.py:490-519), replayed natively
    (xpg_mt19937_repeat_draws, host code): per repeat the sampler seed
    torch.randint(0, 2**62, (1,)), LinearRegression(S)'s initial weights (wlm.py:40-45:
    kaiming_uniform_(a=sqrt(5)) = uniform_(-bound, bound)) and the DataLoader iterator's seed
    draw.  Returns (seeds: list of int, w0: float32 [times, S] host tensor); the generator is
    left exactly where the torch calls leave it.  Returns None (nothing drawn) when this torch
    build's uniform_ rounding matches neither native form (`_draws_form`)."""
    from .wlm import LinearRegression
    if fma is None:
        fma = _draws_form()
        if fma is None:
            return None
    bound = LinearRegression.init_bound(S)
    seeds = np.empty(max(times, 1), dtype=np.int64)
    w0 = torch.empty((times, S), dtype=torch.float32)
    raw, state, left, nxt = _rng_get()
    call("xpg_mt19937_repeat_draws", state.ctypes.data, left.ctypes.data, nxt.ctypes.data, int(times),
         int(S), -bound, bound, int(fma), seeds.ctypes.data,
         w0.data_ptr() if times and S else None)
    _rng_set(raw, state, left, nxt)
    return seeds[:times].tolist(), w0


def compat_community_bits(cols: int, communities, blocks):
    """The reference's compat community draws (Mask.mask_generator with communities,
    masks.py:299-348 + pathways.py:234-385) on torch's global CPU generator, bit-identical, as
    UNSHUFFLED bit-packed int32 [rows, ceil(cols / 32)] host rows (pinned when a GPU is
    present); the generator is advanced exactly as the reference's torch calls advance it, so
    the caller's row shuffle (torch.randperm) follows on the same stream.  `communities`: every
    community's member columns (each sorted ascending, as the reference sorts them in place);
    `blocks`: int32 [n_blocks, 5] {row_start, size, size_internal, own, b} (Mask.community_plan).
    Host code in the library (xpg_mt19937_community_bits)."""
    blocks = np.ascontiguousarray(np.asarray(blocks), dtype=np.int32).reshape(-1, 5)
    lens = np.fromiter((len(c) for c in communities), dtype=np.int64, count=len(communities))
    ptr_ = np.zeros(lens.size + 1, dtype=np.int32)
    np.cumsum(lens, out=ptr_[1:])
    flat = np.fromiter(itertools.chain.from_iterable(communities), dtype=np.int64,
                       count=int(lens.sum()))
    flat = np.ascontiguousarray(flat if flat.size else np.zeros(1, np.int64), dtype=np.int32)
    rows = int(blocks[-1, 0]) + int(blocks[-1, 1])
    out = torch.empty((rows, words_of(cols)), dtype=torch.int32,
                      pin_memory=torch.cuda.is_available())
    raw, state, left, nxt = _rng_get()
    call("xpg_mt19937_community_bits", state.ctypes.data, left.ctypes.data, nxt.ctypes.data,
         int(cols), int(lens.size), ptr_.ctypes.data, flat.ctypes.data, blocks.ctypes.data,
         int(blocks.shape[0]), rows, out.data_ptr())
    _rng_set(raw, state, left, nxt)
    return out


def _rng_get():
    """torch's CPU generator state as (raw bytes, state[624] uint32, left int32[1], next int32[1])."""
    raw = torch.get_rng_state().numpy().copy()
    left = raw[_RNG_LEFT:_RNG_LEFT + 4].view(np.int32).copy()
    nxt = np.array([int(raw[_RNG_NEXT:_RNG_NEXT + 8].view(np.uint64)[0])], dtype=np.int32)
    state = raw[_RNG_STATE:_RNG_STATE + 624 * 8].view(np.uint64).astype(np.uint32)
    return raw, state, left, nxt


def _rng_set(raw, state, left, nxt):
    """Write an advanced (state, left, next) back into torch's CPU generator."""
    raw[_RNG_LEFT:_RNG_LEFT + 4] = left.view(np.uint8)
    raw[_RNG_NEXT:_RNG_NEXT + 8] = np.array([nxt[0]], dtype=np.uint64).view(np.uint8)
    raw[_RNG_STATE:_RNG_STATE + 624 * 8] = state.astype(np.uint64).view(np.uint8)
    torch.set_rng_state(torch.from_numpy(raw))


def sample_shapley_dev(seed: torch.Tensor, rows: int, cols: int, row_offset: int = 0,
                       out: torch.Tensor = None):
    """`sample_shapley` with the seed read on the device from `seed` (int64 [1], the bits of a
    uint64) when the kernel runs: a captured HIP graph draws new rows on every replay once the
    caller advances the tensor on the stream (xpg_sample_shapley_dev).  `out` (int32
    [rows, words]): write the rows there (no allocation, e.g. on a side stream in a capture)."""
    _lib.require_device(seed, "seed")
    if seed.dtype != torch.int64 or seed.numel() != 1:
        raise ValueError("seed must be a device int64 tensor of one element")
    if out is None:
        bits = torch.empty((rows, words_of(cols)), dtype=torch.int32, device=seed.device)
    elif out.dtype != torch.int32 or tuple(out.shape) != (rows, words_of(cols)) or \
            not out.is_contiguous():
        raise ValueError("out must be a contiguous int32 [rows, ceil(cols / 32)] tensor")
    else:
        bits = out
    call("xpg_sample_shapley_dev", ptr(seed), row_offset, rows, cols, ptr(bits),
         _lib.stream_of(seed.device))
    return bits


def community_columns(communities, cols):
    """Column -> community CSR (int32 col_ptr [cols+1], col_comm [nnz]) of a community list."""
    lens = np.array([len(c) for c in communities], dtype=np.int64)
    members = (np.concatenate([np.asarray(c, dtype=np.int64) for c in communities])
               if lens.sum() else np.zeros(0, dtype=np.int64))
    assert members.size == 0 or (members.min() >= 0 and members.max() < cols), \
        "community member outside the mask columns"
    comm = np.repeat(np.arange(len(communities), dtype=np.int64), lens)
    order = np.argsort(members, kind="stable")
    col_ptr = np.zeros(cols + 1, dtype=np.int64)
    np.cumsum(np.bincount(members, minlength=cols), out=col_ptr[1:])
    return (torch.from_numpy(col_ptr.astype(np.int32)),
            torch.from_numpy(comm[order].astype(np.int32)))


def community_tables(plan, communities, cols: int, device, columns=None):
    """Device copies of a community plan (Mask.community_plan) and its column -> community CSR,
    uploaded once and reused by every repeat's `sample_communities(..., tables=...)`."""
    blocks, src_rows, rows, shuffle = plan
    dev = torch.device(device)
    col_ptr, col_comm = columns if columns is not None else community_columns(communities, cols)
    if col_comm.numel() == 0:
        col_comm = torch.zeros(1, dtype=torch.int32)
    up = lambda t: t.to(dev, torch.int32).contiguous()
    return (up(blocks), up(col_ptr), up(col_comm), int(src_rows), int(rows), bool(shuffle),
            len(communities), int(cols))


def sample_communities(seed: int, plan, communities, cols: int, device, columns=None,
                       tables=None, row_offset: int = 0, rows: int = None, out=None):
    """Device community masks (masks.py:81-194, pathways.py:234-385).

    plan = Mask.community_plan(); columns = community_columns(communities, cols); tables =
    community_tables(...) (skips the per-call uploads).  Returns (row bits int32 [rows, words],
    pathway_rows int32 [rows]).  row_offset / rows: only the global rows [row_offset,
    row_offset + rows) of the repeat (a rank's shard; the same rows as the full call's).  out:
    a contiguous int32 [rows, words] view to write the bits into (e.g. one repeat's slice of a
    multi-repeat buffer, instead of a torch.cat of per-repeat draws)."""
    if tables is None:
        tables = community_tables(plan, communities, cols, device, columns)
    blocks, col_ptr, col_comm, src_rows, total, shuffle, n_comm, cols = tables
    rows = total - row_offset if rows is None else rows
    if row_offset < 0 or rows < 0 or row_offset + rows > total:
        raise ValueError(f"community rows [{row_offset}, {row_offset + rows}) outside the "
                         f"repeat's {total} rows")
    dev = blocks.device
    if out is None:
        bits = torch.empty((rows, words_of(cols)), dtype=torch.int32, device=dev)
    else:
        if (out.dtype != torch.int32 or tuple(out.shape) != (rows, words_of(cols))
                or not out.is_contiguous() or out.device != dev):
            raise ValueError(f"out must be a contiguous int32 [{rows}, {words_of(cols)}] tensor "
                             f"on {dev}")
        bits = out
    prow = torch.empty(rows, dtype=torch.int32, device=dev)
    call("xpg_sample_communities_rows", ctypes.c_uint64(int(seed) & (2 ** 64 - 1)), row_offset,
         rows, cols, n_comm, ptr(blocks), blocks.shape[0], src_rows, int(shuffle),
         ptr(col_ptr), ptr(col_comm), ptr(bits), ptr(prow), _lib.stream_of(dev))
    return bits, prow


def edge_keep(bits, cols, src, dst):
    """data.py:390-451 edge mask: [rows * n_edges] bool, copy-major."""
    _lib.require_device(bits, "bits")
    rows = bits.shape[0]
    s = src.to(device=bits.device, dtype=torch.int32).contiguous()
    d = dst.to(device=bits.device, dtype=torch.int32).contiguous()
    keep = torch.empty(rows * s.numel(), dtype=torch.uint8, device=bits.device)
    call("xpg_edge_keep", ptr(bits), rows, cols, ptr(s), ptr(d), s.numel(), ptr(keep),
         _lib.stream_of(bits.device))
    return keep.view(torch.bool)


def rows_no_edge(bits, cols, src, dst):
    """bool [rows]: mask rows that keep no edge (src[e], dst[e] both kept) — the multi-node-type
    loop's empty copies (model.py:213-215), without the rows x edges keep matrix."""
    _lib.require_device(bits, "bits")
    rows = bits.shape[0]
    s = src.to(device=bits.device, dtype=torch.int32).contiguous()
    d = dst.to(device=bits.device, dtype=torch.int32).contiguous()
    out = torch.empty(rows, dtype=torch.uint8, device=bits.device)
    call("xpg_rows_no_edge", ptr(bits), rows, cols, ptr(s), ptr(d), s.numel(), ptr(out),
         _lib.stream_of(bits.device))
    return out.view(torch.bool)


# ----------------------------------------------------------------------------- k-hop subgraph
def khop_subgraph(node_idx: int, num_hops: int, edge_index: torch.Tensor, num_nodes: int):
    """Data.comp_graph's k_hop_subgraph (data.py:331-333; PyG 2.0.4 semantics, relabel_nodes=True,
    flow='source_to_target') on device: (subset int64, relabelled edge_index int64 [2, E_sub],
    inv int64 [1], edge_mask bool [E]).  One host sync (the output sizes)."""
    _lib.require_device(edge_index, "edge_index")
    dev = edge_index.device
    ei = edge_index.to(torch.int64).contiguous()
    E, N, seed = ei.shape[1], int(num_nodes), int(node_idx)
    if not 0 <= seed < N:
        raise IndexError(f"k_hop_subgraph: node {seed} out of range for {N} nodes")
    nbytes = ctypes.c_size_t(0)
    call("xpg_khop_workspace", N, E, ctypes.byref(nbytes))
    ws = _workspace(dev, nbytes.value)
    subset = torch.empty(N, dtype=torch.int64, device=dev)
    sub = torch.empty((2, max(E, 1)), dtype=torch.int64, device=dev)
    emask = torch.empty(E, dtype=torch.uint8, device=dev)
    counts = torch.empty(4, dtype=torch.int64, device=dev)
    call("xpg_khop_subgraph", ptr(ei), E, N, seed, int(num_hops), ptr(subset), ptr(sub),
         ptr(sub[1]), ptr(emask), ptr(counts), ptr(ws), ws.numel(), _lib.stream_of(dev))
    n_sub, n_e, inv, bad = counts.tolist()
    if bad:
        raise IndexError("k_hop_subgraph: edge_index holds node ids outside [0, num_nodes)")
    # inv: the seed's position, already on the device in counts[2] (no host -> device copy)
    return subset[:n_sub], sub[:, :n_e].contiguous(), counts[2:3], emask.view(torch.bool)


# ----------------------------------------------------------------------------- KernelSHAP
def shap_kernel(bits: torch.Tensor, cols: int, counts: torch.Tensor = None,
                out: torch.Tensor = None, scratch: torch.Tensor = None) -> torch.Tensor:
    """Kernel.compute (kernels.py:115-174) on device: fp64 [rows].  `counts` (row popcounts from
    `sample_shapley(..., with_counts=True)`) skips the popcount pass over the bits.  `out`
    (fp64 [rows]) and `scratch` (int32 [rows], the popcounts) let a caller that launches this on
    a side stream inside a graph capture avoid allocating there."""
    _lib.require_device(bits, "bits")
    rows = bits.shape[0]
    if out is None:
        out = torch.empty(rows, dtype=torch.float64, device=bits.device)
    elif out.dtype != torch.float64 or out.numel() != rows or not out.is_contiguous():
        raise ValueError("out must be a contiguous float64 [rows] tensor")
    st = _lib.stream_of(bits.device)
    if counts is None:
        if scratch is None:
            scratch = torch.empty(rows, dtype=torch.int32, device=bits.device)
        elif scratch.dtype != torch.int32 or scratch.numel() != rows or not scratch.is_contiguous():
            raise ValueError("scratch must be a contiguous int32 [rows] tensor")
        counts = scratch
        call("xpg_popcount_rows", ptr(bits), rows, cols, ptr(counts), st)
    else:
        _lib.require_device(counts, "counts")
        if counts.dtype != torch.int32 or counts.numel() != rows:
            raise ValueError("counts must be int32 [rows]")
        counts = counts.contiguous()
    call("xpg_shap_kernel", ptr(counts), rows, cols, ptr(out), st)
    return out


# ----------------------------------------------------------------------------- dense
def dense(A: torch.Tensor, W: torch.Tensor, bias, act=None, n_real=None) -> torch.Tensor:
    """act(A W^T + b) on the fp32 MFMA kernel.  A [M, K] and W [N, K] are zero-padded here."""
    dev = A.device
    M, K = A.shape
    N = W.shape[0] if n_real is None else n_real
    k_pad, n_pad = _rup(K, 8), _rup(max(N, 1), 32)
    Ap = A if (K == k_pad and A.is_contiguous()) else \
        torch.nn.functional.pad(A.float(), (0, k_pad - K)).contiguous()
    Wp = torch.zeros((n_pad, k_pad), dtype=torch.float32, device=dev)
    Wp[:W.shape[0], :K] = W
    bp = torch.zeros(n_pad, dtype=torch.float32, device=dev)
    if bias is not None:
        bp[:bias.shape[0]] = bias
    C = torch.empty((M, n_pad), dtype=torch.float32, device=dev)
    call("xpg_dense", ptr(Ap), M, k_pad, ptr(Wp), k_pad, k_pad, ptr(bp), N, n_pad,
         ACT[act], ptr(C), n_pad, _lib.stream_of(dev))
    return C[:, :N]


# ----------------------------------------------------------------------------- kernel timing
PROF_SLOTS = ("wide_bits", "wide_f0", "wide_degree", "wide_l1", "wide_l2")


def profile_enable(on=True):
    """Per-kernel HIP-event timing of the wide forward path (xpg_profile_enable): measurement
    only, never around a graph capture."""
    _lib.check(_lib.load().xpg_profile_enable(1 if on else 0))


def profile_read():
    """{slot: (device ms summed over launches, launches)} since profile_enable (waits for the
    recorded events; xpg_profile_read)."""
    n = len(PROF_SLOTS)
    ms = (ctypes.c_double * n)()
    cnt = (ctypes.c_int64 * n)()
    _lib.check(_lib.load().xpg_profile_read(ms, cnt, n))
    return {k: (ms[i], cnt[i]) for i, k in enumerate(PROF_SLOTS)}


# ----------------------------------------------------------------------------- forward plan
def plan_arrays(S, rel_np, queries, L, rel_eid=None):
    """Receptive-field frontiers and CSR arrays of a ForwardPlan, built on the host by the
    library (xpg_plan_arrays_build / _take, include/xpgnn.h): the same arrays as
    `plan_arrays_numpy` below (its docstring has the layout), ~20 us instead of ~0.4 ms of numpy
    calls for a ~1k-node subgraph.  (No "pos" maps: every frontier is a prefix of F_0.)"""
    q = np.ascontiguousarray(queries, dtype=np.int64).reshape(-1)
    if q.size == 0 or q.min() < 0 or q.max() >= S:
        raise ValueError("query positions out of range")
    if q.size > 1 and np.unique(q).size != q.size:
        raise ValueError("duplicate query positions")
    n_rel = len(rel_np)
    rel_ptr = np.zeros(n_rel + 1, dtype=np.int64)
    for r, e in enumerate(rel_np):
        rel_ptr[r + 1] = rel_ptr[r] + e.shape[1]

    def cat(xs):
        if len(xs) == 1:
            return np.ascontiguousarray(xs[0], dtype=np.int64)
        return np.ascontiguousarray(np.concatenate(xs) if xs else np.zeros(0), dtype=np.int64)
    src, dst = cat([e[0] for e in rel_np]), cat([e[1] for e in rel_np])
    eid = cat(list(rel_eid)) if rel_eid is not None else None
    sizes = np.zeros((L + 1) * 7, dtype=np.int64)
    h = ctypes.c_void_p()

    def vp(a):
        return ctypes.c_void_p(a.ctypes.data) if a is not None and a.size else ctypes.c_void_p(0)
    call("xpg_plan_arrays_build", int(S), n_rel, vp(rel_ptr), vp(src), vp(dst), vp(eid), vp(q),
         int(q.size), int(L), ctypes.byref(h), vp(sizes))
    out = np.empty(max(int(sizes.sum()), 1), dtype=np.int64)
    call("xpg_plan_arrays_take", h, vp(out))
    parts, o = [], 0
    for n in sizes.tolist():
        parts.append(out[o:o + n])
        o += n
    fr = parts[:L + 1]
    names = ("ptr", "src", "eid", "smul", "sptr", "seid")
    csrs = [dict(zip(names, parts[L + 1 + 6 * i:L + 7 + 6 * i])) for i in range(L + 1)]
    deg = csrs[0]
    layers = [{"agg_ptr": c["ptr"], "agg_src": c["src"], "agg_f0": c["src"], "self_mult": c["smul"],
               "agg_eid": c["eid"], "self_ptr": c["sptr"], "self_eid": c["seid"]} for c in csrs[1:]]
    return {"frontiers": fr, "deg_ptr": deg["ptr"], "deg_src": deg["src"], "deg_eid": deg["eid"],
            "layers": layers}


def plan_arrays_numpy(S, rel_np, queries, L, rel_eid=None):
    """numpy restatement of `plan_arrays` (the arrays the native builder is tested against).

    frontiers[L] = queries; frontiers[l-1] = frontiers[l] + sorted new in-neighbours (all
    relations), so frontiers[l] is a prefix of frontiers[l-1].  deg_*: in-edges (self-loops
    excluded) of every F_0 node per relation, relation-major with absolute offsets.  layers[l-1]:
    in-edges of F_l targets (self-loops excluded) with source positions in F_{l-1} and F_0, plus
    the multiplicity of (t, t) edges per relation.

    rel_eid (edge-mask plans, Data.perturb_edge): per relation the mask column of every edge;
    the CSRs then also carry each entry's column (deg_eid, agg_eid) and every target's
    self-loop columns (self_ptr / self_eid)."""
    all_src = np.concatenate([e[0] for e in rel_np]) if rel_np else np.zeros(0, np.int64)
    all_dst = np.concatenate([e[1] for e in rel_np]) if rel_np else np.zeros(0, np.int64)
    fr = [None] * (L + 1)
    fr[L] = np.asarray(queries, dtype=np.int64).reshape(-1)
    if fr[L].size == 0 or fr[L].min() < 0 or fr[L].max() >= S:
        raise ValueError("query positions out of range")
    if np.unique(fr[L]).size != fr[L].size:
        raise ValueError("duplicate query positions")
    for lvl in range(L, 0, -1):
        cur = fr[lvl]
        mark = np.zeros(S, dtype=bool)
        mark[cur] = True
        nb = np.unique(all_src[mark[all_dst]])
        fr[lvl - 1] = np.concatenate([cur, nb[~mark[nb]]])
    pos = []
    for lvl in range(L + 1):
        p = np.full(S, -1, dtype=np.int64)
        p[fr[lvl]] = np.arange(fr[lvl].size)
        pos.append(p)
    n0 = fr[0].size

    eids = rel_eid if rel_eid is not None else [np.zeros(e.shape[1], np.int64) for e in rel_np]

    def csr(targets_pos, n_t, src_pos_maps):
        ptrs, cols, off = [], [[] for _ in src_pos_maps], 0
        smul, eid, sptr, seid, soff = [], [], [], [], 0
        for (s, d), ecol in zip(rel_np, eids):
            k = s != d
            s2, d2, e2 = s[k], d[k], ecol[k]
            sel = targets_pos[d2] >= 0
            key = targets_pos[d2[sel]]
            order = np.argsort(key, kind="stable")
            src_nodes = s2[sel][order]
            eid.append(e2[sel][order])
            for j, m in enumerate(src_pos_maps):
                cols[j].append(m(src_nodes))
            cnt = np.bincount(key, minlength=n_t)
            ptrs.append(np.concatenate([[0], np.cumsum(cnt)]) + off)
            off += int(cnt.sum())
            loops, lcol = s[~k], ecol[~k]
            ls = targets_pos[loops] >= 0
            lkey = targets_pos[loops[ls]]
            smul.append(np.bincount(lkey, minlength=n_t))
            lorder = np.argsort(lkey, kind="stable")
            seid.append(lcol[ls][lorder])
            sptr.append(np.concatenate([[0], np.cumsum(smul[-1])]) + soff)
            soff += int(smul[-1].sum())
        cat = [np.concatenate(c) if c else np.zeros(0, np.int64) for c in cols]
        return (np.concatenate(ptrs), cat, np.concatenate(smul), np.concatenate(eid),
                np.concatenate(sptr), np.concatenate(seid))

    deg_ptr, (deg_src,), _, deg_eid, _, _ = csr(pos[0], n0, [lambda v: v])
    layers = []
    for lvl in range(1, L + 1):
        ptr_, (a_src, a_f0), smul, a_eid, s_ptr, s_eid = csr(
            pos[lvl], fr[lvl].size, [lambda v, l=lvl: pos[l - 1][v], lambda v: pos[0][v]])
        layers.append({"agg_ptr": ptr_, "agg_src": a_src, "agg_f0": a_f0, "self_mult": smul,
                       "agg_eid": a_eid, "self_ptr": s_ptr, "self_eid": s_eid})
    return {"frontiers": fr, "pos": pos, "deg_ptr": deg_ptr, "deg_src": deg_src,
            "deg_eid": deg_eid, "layers": layers}


_STAGING = {}  # device index -> [next slot, [(pinned host tensor, event of its last copy)] * _STAGING_SLOTS]
_STAGING_MAX = 16 << 20  # bytes: larger arrays take the pageable copy
_STAGING_SLOTS = 4  # a call's uploads take consecutive slots: none waits for the previous copy


def h2d(a, device):
    """A host numpy array (int32 / int64 / float32) as a new device tensor, copied from a pinned
    staging buffer without a host wait: a pageable host -> device copy waits for everything queued
    on the stream first (~40 us of an Explainer.run first call per plan upload, the device idle
    meanwhile).  Uploads rotate over a few pinned buffers; a buffer is reused once its previous
    copy has completed (its event: with one buffer the second upload of a call waited for the
    first copy, i.e. for everything queued before it)."""
    a = np.ascontiguousarray(a)
    dev = torch.device(device)
    if a.nbytes > _STAGING_MAX or a.nbytes == 0:
        return torch.from_numpy(a).to(dev)
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    ring = _STAGING.get(key)
    if ring is None:  # every slot pinned up front: a pinned allocation costs ~0.2 ms per call
        ring = _STAGING[key] = [0, [(torch.empty(1 << 20, dtype=torch.uint8, pin_memory=True), None)
                                    for _ in range(_STAGING_SLOTS)]]
    slot = ring[0]
    ring[0] = (slot + 1) % _STAGING_SLOTS
    buf, ev = ring[1][slot]
    if ev is not None:
        ev.synchronize()
    if buf is None or buf.numel() < a.nbytes:
        buf = torch.empty(max(a.nbytes, 1 << 20), dtype=torch.uint8, pin_memory=True)
    buf[:a.nbytes].numpy()[:] = a.view(np.uint8).reshape(-1)
    out = torch.empty(a.shape, dtype=torch.from_numpy(a[:0]).dtype, device=dev)
    out.view(-1).view(torch.uint8).copy_(buf[:a.nbytes], non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    ring[1][slot] = (buf, ev)
    return out


# ForwardPlan drops the relation terms of other destination types from a layer whose targets
# share one node type (they add exactly 0); False keeps every term (the parity suite's reference)
PLAN_DROP_OTHER_TYPES = True


class ForwardPlan:
    """Receptive-field plan of one (subgraph, model program, query set)."""

    def __init__(self, program, sub_feat, rel_edges, queries, device=None, node_type=None,
                 edge_cols=None, link=None):
        """`node_type` ([S] node type of every subgraph node) is required by multi-node-type
        programs: per layer, every target's type gates the relation terms (xpgnn.h).

        Edge problems (Data.perturb_edge, data.py:500-554): `edge_cols` = per relation the mask
        column of every edge (mask columns are the subgraph's edges; `cols` becomes their
        count) and `link` = (a, b, act): the output is the link decoder act(<h_a, h_b>) of
        queries a and b instead of one column per query."""
        device = torch.device(device) if device is not None else sub_feat.device
        _lib.require_device(torch.empty(0, device=device), "plan device")
        if len(program.convs) == 0:
            raise ValueError("program has no conv layer")
        self.device = device
        self.program = program
        S = int(sub_feat.shape[0])  # subgraph nodes
        self.n_rel = len(rel_edges)
        self._keep = []  # device tensors referenced by descriptors
        self._staged = []  # (descriptor, field, int32 array) awaiting the one upload

        rel_np = [np.asarray(e.detach().cpu().numpy(), dtype=np.int64).reshape(2, -1)
                  for e in rel_edges]
        rel_eid = None
        if edge_cols is not None:
            rel_eid = [np.asarray(torch.as_tensor(c).detach().cpu().numpy(), dtype=np.int64).reshape(-1)
                       for c in edge_cols]
            if len(rel_eid) != len(rel_np) or any(c.size != e.shape[1] for c, e in zip(rel_eid, rel_np)):
                raise ValueError("edge_cols must give one mask column per edge of every relation")
            if program.n_types > 1:
                raise ValueError("edge masks on multi-node-type programs are not supported")
        self.edge_masks = rel_eid is not None
        self.cols = (int(max((int(c.max()) for c in rel_eid if c.size), default=-1)) + 1
                     if self.edge_masks else S)
        if self.edge_masks:
            ncol = sum(c.size for c in rel_eid)
            allc = np.concatenate(rel_eid) if ncol else np.zeros(0, np.int64)
            if ncol and (allc.min() < 0 or np.unique(allc).size != ncol or self.cols != ncol):
                raise ValueError("edge mask columns must be 0..E-1, one per edge")
            if ncol == 0:
                raise ValueError("edge masks need at least one edge")
        L = len(program.convs)
        arr = plan_arrays(S, rel_np, queries, L, rel_eid)
        self.arrays = arr
        fr = arr["frontiers"]
        n0 = fr[0].size
        self.n0 = n0
        self.frontiers = fr

        X0 = sub_feat.to(device=device, dtype=torch.float32)[h2d(fr[0], device)]
        f_in0 = program.convs[0].f_in
        nt_np = None
        if program.n_types > 1:
            if node_type is None:
                raise ValueError("multi-node-type program needs the subgraph node types")
            nt_np = np.asarray(torch.as_tensor(node_type).detach().cpu().numpy()).astype(np.int64)
            if nt_np.shape != (S,) or nt_np.min() < 0 or nt_np.max() >= program.n_types:
                raise ValueError("node types out of range")
            if X0.shape[1] > f_in0:  # widest types are zero-padded beyond every relation's input
                X0 = X0[:, :f_in0]
        if X0.shape[1] != f_in0:
            raise ValueError(f"feature width {X0.shape[1]} != first conv input {f_in0}")

        self._layers = (LayerDesc * L)()
        prev_pad = None
        self.terms_kept = []  # per layer: terms after dropping other node types' relations
        self.lowering = []  # per layer: (kind, relation, destination type) of every kept term
        for li, conv in enumerate(program.convs):
            lvl = li + 1
            n_t = fr[lvl].size
            f_out_pad = _rup(conv.f_out, 32)
            if f_out_pad > 256 or len(conv.terms) > _lib.MAX_TERMS:
                raise ValueError("conv wider than 256 or more than 8 terms is not supported")
            terms = list(conv.terms)
            if nt_np is not None:
                # every target of this layer has one node type: a relation term of another
                # destination type adds exactly 0 to every target (HeteroConv sums per
                # destination), so it is dropped — fewer aggregate columns and a shorter K of
                # the layer's dense product (the query layer of a multi-type plan)
                tt = np.unique(nt_np[fr[lvl]])
                if tt.size == 1 and PLAN_DROP_OTHER_TYPES:
                    kept = [t for t in terms if t.dst_type < 0 or t.dst_type == int(tt[0])]
                    terms = kept or terms
            self.terms_kept.append(len(terms))
            self.lowering.append(tuple((t.kind, t.rel, t.dst_type) for t in terms))
            ld = self._layers[li]
            ld.n_terms = len(terms)
            ld.act = ACT[conv.act]
            ld.f_out = conv.f_out
            ld.f_out_pad = f_out_pad
            ld.n_tgt = n_t
            ld.n_edges = int(arr["layers"][li]["agg_src"].size)
            ld.f_in_pad = 0 if li == 0 else prev_pad
            nz = lambda a: a if a.size else np.zeros(1)
            self._i32(ld, "tgt_prev", np.arange(n_t))  # F_l is a prefix of F_{l-1}
            self._i32(ld, "tgt_f0", np.arange(n_t))  # F_l is a prefix of F_0 too
            lay = arr["layers"][li]
            self._i32(ld, "agg_ptr", lay["agg_ptr"])
            self._i32(ld, "agg_src", nz(lay["agg_src"]))
            self._i32(ld, "agg_f0", nz(lay["agg_f0"]))
            self._i32(ld, "self_mult", lay["self_mult"])
            if self.edge_masks:
                self._i32(ld, "agg_eid", nz(lay["agg_eid"]))
                self._i32(ld, "self_ptr", lay["self_ptr"])
                self._i32(ld, "self_eid", nz(lay["self_eid"]))
            n_types = program.n_types

            def make_bias(conv=conv, f_out_pad=f_out_pad):
                b = torch.zeros((n_types, f_out_pad), dtype=torch.float32, device=device)
                b[:, :conv.f_out] = conv.bias.to(device).reshape(-1, conv.f_out)
                return b
            bias = self._program_tensor(program, ("bias", li), make_bias)
            self._keep.append(bias)
            ld.bias = bias.data_ptr()
            ld.n_types = n_types
            if nt_np is not None:
                self._i32(ld, "tgt_type", nt_np[fr[lvl]])
            else:
                ld.tgt_type = None
            for k, term in enumerate(terms):
                ld.terms[k].kind = TERM[term.kind]
                ld.terms[k].rel = term.rel
                ld.terms[k].dst_type = term.dst_type
            if li == 0:
                for k, term in enumerate(terms):
                    T = dense(X0, term.weight.to(device), None, None)
                    Tp = torch.zeros((n0, f_out_pad), dtype=torch.float32, device=device)
                    Tp[:, :conv.f_out] = T
                    self._keep.append(Tp)
                    ld.terms[k].table = Tp.data_ptr()
                ld.weight = None
            else:
                def make_wc(conv=conv, terms=terms, prev_pad=prev_pad, f_out_pad=f_out_pad):
                    w = torch.zeros((f_out_pad, len(terms) * prev_pad), dtype=torch.float32,
                                    device=device)
                    for k, term in enumerate(terms):
                        w[:conv.f_out, k * prev_pad:k * prev_pad + conv.f_in] = term.weight.to(device)
                    return w
                Wc = self._program_tensor(program, ("wc", li, tuple(id(t) for t in terms)), make_wc)
                self._keep.append(Wc)
                ld.weight = Wc.data_ptr()
            prev_pad = f_out_pad

        self._head = (HeadDesc * max(1, len(program.head)))()
        for i, h in enumerate(program.head):
            n_real, k_real = h.weight.shape
            n_pad = _rup(n_real, 32)
            if n_pad > 256:
                raise ValueError("head layer wider than 256 is not supported")
            def make_head(h=h, n_real=n_real, k_real=k_real, n_pad=n_pad, prev_pad=prev_pad):
                w = torch.zeros((n_pad, prev_pad), dtype=torch.float32, device=device)
                w[:n_real, :k_real] = h.weight.to(device)
                b = torch.zeros(n_pad, dtype=torch.float32, device=device)
                if h.bias is not None:
                    b[:n_real] = h.bias.to(device)
                return w, b
            Wp, bp = self._program_tensor(program, ("head", i), make_head)
            self._keep += [Wp, bp]
            hd = self._head[i]
            hd.k_pad, hd.n_real, hd.n_pad, hd.act = prev_pad, n_real, n_pad, ACT[h.act]
            hd.weight, hd.bias = Wp.data_ptr(), bp.data_ptr()
            prev_pad = n_pad

        self.n_out = fr[L].size
        self.desc = ForwardPlanDesc(
            cols=self.cols, n_rel=self.n_rel, n0=n0,
            n_deg_edges=int(arr["deg_src"].size), n_layers=L,
            layers=self._layers, n_head=len(program.head), head=self._head,
            out_col=program.out_col)
        self._i32(self.desc, "f0_node", fr[0])
        self._i32(self.desc, "deg_ptr", arr["deg_ptr"])
        self._i32(self.desc, "deg_src", arr["deg_src"] if arr["deg_src"].size else np.zeros(1))
        if self.edge_masks:
            self.desc.edge_masks = 1
            self._i32(self.desc, "deg_eid", arr["deg_eid"] if arr["deg_eid"].size else np.zeros(1))
        self.link = link
        if link is not None:
            a, b, act = link
            if not (0 <= a < self.n_out and 0 <= b < self.n_out):
                raise ValueError("link decoder targets out of range")
            self.desc.edge_dot, self.desc.dot_a, self.desc.dot_b = 1, int(a), int(b)
            self.desc.dot_act = ACT[act]
            self.n_out = 1
        self._upload_i32()
        self._ws = None
        self._ws_stream = None  # raw handle of the stream that last used self._ws

    def _program_tensor(self, program, key, make):
        """Device tensors derived from the program's weights alone (padded biases, the stacked
        dense weights of layers >= 1, head layers): built once per (program, device) and shared by
        every plan of that program (pipeline.compiled_program reuses a program while the module's
        parameters are unchanged), so a new query's plan only builds its own arrays and tables."""
        cache = program.__dict__.setdefault("_device_tensors", {})
        k = (str(self.device),) + key
        if k not in cache:
            cache[k] = make()
        return cache[k]

    def _i32(self, obj, field, a):
        """Stage an int32 array for descriptor field `obj.field`; `_upload_i32` moves every
        staged array to the device in ONE host -> device copy (a plan has ~15-25 of them: one
        synchronous copy each was ~0.4 ms of Explainer.run) and fills the pointers."""
        self._staged.append((obj, field, np.ascontiguousarray(a, dtype=np.int32).reshape(-1)))

    def _upload_i32(self):
        sizes = [(a.size + 15) // 16 * 16 for _, _, a in self._staged]  # 64-B aligned slices
        offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        host = np.zeros(int(offs[-1]), dtype=np.int32)
        for (_, _, a), o in zip(self._staged, offs):
            host[o:o + a.size] = a
        buf = h2d(host, self.device)
        self._keep.append(buf)
        self.int_arrays = buf  # every staged array, one allocation
        base = buf.data_ptr()
        for (obj, field, _), o in zip(self._staged, offs):
            setattr(obj, field, base + 4 * int(o))
        self._staged = []

    def device_bytes(self):
        """Device memory the plan holds: its arrays, tables, weights and forward workspace."""
        held = self._keep + ([self._ws] if self._ws is not None else [])
        return sum(t.numel() * t.element_size() for t in held)

    def workspace_bytes(self, rows):
        n = ctypes.c_size_t(0)
        _lib.check(_lib.load().xpg_forward_workspace(ctypes.byref(self.desc), rows, ctypes.byref(n)))
        return n.value

    def forward(self, bits: torch.Tensor, max_ws_bytes=8 << 30, out: torch.Tensor = None,
                workspace: torch.Tensor = None) -> torch.Tensor:
        """y [rows, n_out] fp32: model output at each target of the last conv layer, per mask
        row (wlm.py:349-436 for one batch, all batches at once).  `out`: a contiguous fp32
        [rows, n_out] tensor to write y into (no allocation once the workspace exists).
        `workspace`: a uint8 device tensor of at least workspace_bytes(rows) to use instead of the
        plan's own — forwards running at the same time on different streams need one each (the
        workspace holds the launch's block-scheduling counters).  Without it, forwards on
        different streams through one plan are ordered: each waits for the stream that used the
        plan's workspace last."""
        _lib.require_device(bits, "bits")
        rows = bits.shape[0]
        if out is None:
            y = torch.empty((rows, self.n_out), dtype=torch.float32, device=self.device)
        elif out.dtype != torch.float32 or tuple(out.shape) != (rows, self.n_out) or \
                not out.is_contiguous():
            raise ValueError("out must be a contiguous float32 [rows, n_out] tensor")
        else:
            y = out
        if rows == 0:
            return y
        st = _lib.stream_of(self.device)
        if workspace is not None:
            if workspace.dtype != torch.uint8 or workspace.device != self.device or \
                    workspace.numel() < self.workspace_bytes(rows):
                raise ValueError("workspace must be a uint8 device tensor of workspace_bytes(rows)")
            call("xpg_masked_forward", ctypes.byref(self.desc), ptr(bits), rows, ptr(y),
                 ptr(workspace), workspace.numel(), st)
            return y
        w1, w2 = self.workspace_bytes(1), self.workspace_bytes(2)
        per_row = max(0, w2 - w1)  # 0: a rows-independent workspace (the wide 32-row passes)
        fixed = max(0, w1 - per_row)
        chunk = rows if per_row == 0 else \
            max(1, min(rows, max(0, max_ws_bytes - fixed) // per_row))
        need = self.workspace_bytes(chunk)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        # the plan's own workspace (and the block counters in it) is reused in stream order: a
        # forward on another stream than the last user's first waits for what that stream has
        # queued (two streams forwarding through one plan then take turns instead of racing)
        cur = st.value or 0  # 0: the null stream
        if self._ws_stream is not None and self._ws_stream != cur and \
                not torch.cuda.is_current_stream_capturing():
            torch.cuda.current_stream(self.device).wait_stream(
                torch.cuda.ExternalStream(self._ws_stream, device=self.device))
        self._ws_stream = cur
        for r0 in range(0, rows, chunk):
            n = min(chunk, rows - r0)
            call("xpg_masked_forward", ctypes.byref(self.desc), ptr(bits[r0:r0 + n]), n,
                 ptr(y[r0:r0 + n]), ptr(self._ws), self._ws.numel(), st)
        return y


# ----------------------------------------------------------------------------- surrogate
_WS = {}


def _workspace(dev, nbytes):
    """Reusable per-device scratch (stream-ordered reuse: every user is on the current stream)."""
    key = (dev.type, dev.index)
    t = _WS.get(key)
    if t is None or t.numel() < nbytes:
        # grown with 25 % headroom, in whole MiB (>= 4 MiB): queries of somewhat larger sizes
        # reuse it instead of each first call on a larger one paying a device allocation; an
        # allocation the headroom does not fit falls back to the exact size
        _WS.pop(key, None)
        del t
        grow = max(4 << 20, (nbytes + nbytes // 4 + (1 << 20) - 1) >> 20 << 20)
        try:
            t = torch.empty(grow, dtype=torch.uint8, device=dev)
        except torch.OutOfMemoryError:
            t = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
        _WS[key] = t
    return t


def check_fit_status(status):
    """Raise FitExchangeError when a fit's device status word (see wlm_fit) is nonzero.  Reads
    the word, i.e. waits for the stream to reach the end of that fit."""
    if int(status.max().item()) != 0:
        raise _lib.FitExchangeError(
            "surrogate fit: the multi-workgroup exchange timed out (workgroups not co-resident, "
            "e.g. another kernel or process held the GPU's CUs); the fitted weights are invalid. "
            "XPG_WLM=single selects the single-workgroup fit.")


_STATUS_HOST = {}


def status_to_host(status):
    """Queue a copy of a fit's device status word into pinned host memory (no host wait) and
    return the host tensor: once a later synchronising read on the stream (e.g. the results'
    .cpu()) has returned, check_status_host(...) reads it without a second synchronisation."""
    key = status.device.index
    h = _STATUS_HOST.get(key)
    if h is None:
        h = _STATUS_HOST[key] = torch.zeros(1, dtype=torch.int32, pin_memory=True)
    h.copy_(status.reshape(-1)[:1], non_blocking=True)
    return h


def check_status_host(h):
    """check_fit_status on a word copied by status_to_host (after the stream reached the copy)."""
    if int(h[0]) != 0:
        check_fit_status(torch.ones(1, dtype=torch.int32))


WLM_KINDS = {0: "single", 1: "multi", 2: "grid", 3: "grid_fused"}


def wlm_plan(n_fits, rows, cols, batch):
    """(kind, parts) of the fit kernel a shape takes on the current device (xpg_wlm_plan):
    kind "single" (one workgroup per fit), "multi" (`parts` co-resident workgroups per fit),
    "grid" (the many-column streaming fit, three launches per step) or "grid_fused" (the
    many-column fit as one persistent launch per fit over `parts` workgroups); the grid kinds
    have no prepared form."""
    kind, parts = ctypes.c_int32(0), ctypes.c_int32(0)
    _lib.check(_lib.load().xpg_wlm_plan(int(n_fits), int(rows), int(cols), int(batch),
                                        ctypes.byref(kind), ctypes.byref(parts)))
    return WLM_KINDS[kind.value], parts.value


class PreparedFit:
    """A fresh surrogate fit (`wlm_fit` from w0) split in its two launches on static buffers of
    one shape (xpg_wlm_prepare / xpg_wlm_fit_prepared, ABI v12): `prepare` runs the prologue
    (per-step constants, column bit vectors, w = w0, zero Adam moments), `fit` the Adam steps and
    returns w [F, cols].  Nothing is allocated after construction, so both can be captured on
    any stream; with two instances the next fit is prepared while the current one runs.
    `status` is the device status word (check_fit_status; sticky over every fit of the
    instance).  Shapes that take the many-column grid fit have no prepared form: ValueError at
    construction (use wlm_fit)."""

    def __init__(self, n_fits, rows, cols, batch, params, device):
        self.kind, self.parts = wlm_plan(n_fits, rows, cols, batch)
        if self.kind.startswith("grid"):
            raise ValueError(f"PreparedFit: {cols} columns take the many-column grid fit, which "
                             "has no prologue / prepared form; use wlm_fit")
        self.shape = (int(n_fits), int(rows), int(cols), int(batch))
        n = ctypes.c_size_t(0)
        _lib.check(_lib.load().xpg_wlm_workspace(n_fits, rows, cols, batch, ctypes.byref(n)))
        self.ws = torch.empty(max(n.value, 1), dtype=torch.uint8, device=device)
        self.w = torch.empty((n_fits, cols), dtype=torch.float32, device=device)
        self.m = torch.empty_like(self.w)
        self.v = torch.empty_like(self.w)
        self.losses = torch.empty((n_fits, math.ceil(rows / batch)), dtype=torch.float64, device=device)
        self.best = torch.empty(n_fits, dtype=torch.int32, device=device)
        self.status = torch.zeros(1, dtype=torch.int32, device=device)
        self.p = WlmParams(lr=abs(float(params["lr"])), l1_lambda=float(params["l1_lambda"]), beta1=0.9,
                           beta2=0.999, eps=1e-8, weight_decay=1e-2)

    def _check(self, name, t, dtype, numel):
        if t.dtype != dtype or t.numel() != numel or not t.is_contiguous():
            raise ValueError(f"{name} must be a contiguous {dtype} tensor of {numel} elements")

    def prepare(self, bits, y, kernel, w0):
        F, R, S, B = self.shape
        self._check("bits", bits, torch.int32, F * R * words_of(S))
        self._check("y", y, torch.float32, F * R)
        self._check("kernel", kernel, torch.float64, F * R)
        self._check("w0", w0, torch.float32, F * S)
        call("xpg_wlm_prepare", F, ptr(bits), R, S, B, ptr(y), ptr(kernel), ctypes.byref(self.p),
             ptr(w0), ptr(self.w), ptr(self.m), ptr(self.v), ptr(self.ws), self.ws.numel(),
             _lib.stream_of(bits.device))

    def fit(self, bits, kernel):
        F, R, S, B = self.shape
        self._check("bits", bits, torch.int32, F * R * words_of(S))
        self._check("kernel", kernel, torch.float64, F * R)
        call("xpg_wlm_fit_prepared", F, ptr(bits), R, S, B, ptr(kernel), ctypes.byref(self.p),
             ptr(self.w), ptr(self.m), ptr(self.v), ptr(self.losses), ptr(self.best), ptr(self.status),
             ptr(self.ws), self.ws.numel(), _lib.stream_of(bits.device))
        return self.w

    def fit_steps(self, bits, kernel):
        """`fit` without its losses / best epoch / status launch (xpg_wlm_fit_steps, ABI v17):
        only the Adam steps on the current stream; call `losses` afterwards (any stream ordered
        after this one) before the workspace is prepared again."""
        F, R, S, B = self.shape
        self._check("bits", bits, torch.int32, F * R * words_of(S))
        self._check("kernel", kernel, torch.float64, F * R)
        call("xpg_wlm_fit_steps", F, ptr(bits), R, S, B, ptr(kernel), ctypes.byref(self.p),
             ptr(self.w), ptr(self.m), ptr(self.v), ptr(self.ws), self.ws.numel(),
             _lib.stream_of(bits.device))
        return self.w

    def finish(self, kernel):
        """The losses, first best epoch and status word of the last `fit_steps`
        (xpg_wlm_fit_losses) on the current stream."""
        F, R, S, B = self.shape
        self._check("kernel", kernel, torch.float64, F * R)
        call("xpg_wlm_fit_losses", F, R, S, B, ptr(kernel), ctypes.byref(self.p), ptr(self.losses),
             ptr(self.best), ptr(self.status), ptr(self.ws), self.ws.numel(),
             _lib.stream_of(kernel.device))
        return self.losses, self.best


def wlm_fit(bits, cols, batch, y, kernel, w0, params, m0=None, v0=None, step0=0, check=True,
            status=None):
    """train_model (wlm.py:132-278) epoch loop on device for one or many independent fits.

    bits [R, W] or [F, R, W]; y / kernel [R] or [F, R]; w0 [S] or [F, S].  Returns
    (w, losses, best_epoch, adam_m, adam_v) with the same leading fit dimension (if any).

    check=True reads the fit's status word and raises FitExchangeError if the multi-workgroup
    exchange failed (one stream sync).  check=False leaves that to the caller: pass `status`
    (device int32 [1], zeroed once) and call check_fit_status(status) later (e.g. after a timed
    region); the word is sticky (ABI v13), so it reports a failure of any fit that used it."""
    dev = bits.device
    batched = bits.dim() == 3
    F = bits.shape[0] if batched else 1
    rows = bits.shape[-2]
    if batch <= 0:
        raise ValueError("batch_size should be a positive integer value, but got "
                         f"batch_size={batch}")
    nsteps = math.ceil(rows / batch)
    # a fresh fit (no Adam state handed in) starts from w0 inside the fit's prologue kernel
    # (xpg_wlm_fit_from): no copy / fill launches on the latency-bound chain
    fresh = m0 is None and v0 is None and int(step0) == 0
    w0f = w0.detach().to(device=dev, dtype=torch.float32).reshape(F, cols).contiguous()
    if fresh:
        w = torch.empty((F, cols), dtype=torch.float32, device=dev)
        m = torch.empty((F, cols), dtype=torch.float32, device=dev)
        v = torch.empty((F, cols), dtype=torch.float32, device=dev)
    else:
        w = w0f.clone()
        m = torch.zeros((F, cols), dtype=torch.float32, device=dev) if m0 is None else \
            m0.reshape(F, cols).clone()
        v = torch.zeros((F, cols), dtype=torch.float32, device=dev) if v0 is None else \
            v0.reshape(F, cols).clone()
    losses = torch.empty((F, nsteps), dtype=torch.float64, device=dev)
    best = torch.empty(F, dtype=torch.int32, device=dev)
    p = WlmParams(lr=abs(float(params["lr"])), l1_lambda=float(params["l1_lambda"]), beta1=0.9,
                  beta2=0.999, eps=1e-8, weight_decay=1e-2)
    yy = y.to(device=dev, dtype=torch.float32).reshape(F, rows).contiguous()
    kk = kernel.to(device=dev, dtype=torch.float64).reshape(F, rows).contiguous()
    bb = bits.contiguous()
    n = ctypes.c_size_t(0)
    _lib.check(_lib.load().xpg_wlm_workspace(F, rows, cols, batch, ctypes.byref(n)))
    ws = _workspace(dev, n.value)
    if status is None:  # sticky word (the fit ORs its error into it): starts at 0
        status = torch.zeros(1, dtype=torch.int32, device=dev)
    if fresh:
        call("xpg_wlm_fit_from", F, ptr(bb), rows, cols, batch, ptr(yy), ptr(kk), ctypes.byref(p),
             ptr(w0f), ptr(w), ptr(m), ptr(v), ptr(losses), ptr(best), ptr(status), ptr(ws),
             ws.numel(), _lib.stream_of(dev))
    else:
        call("xpg_wlm_fit", F, ptr(bb), rows, cols, batch, ptr(yy), ptr(kk), ctypes.byref(p),
             int(step0), ptr(w), ptr(m), ptr(v), ptr(losses), ptr(best), ptr(status), ptr(ws),
             ws.numel(), _lib.stream_of(dev))
    if check:
        check_fit_status(status)
    if not batched:
        return w[0], losses[0], best[0:1], m[0], v[0]
    return w, losses, best, m, v
