"""GPU parity: the HIP engine (through the C-ABI) vs the numpy oracle and the reference's own
golden vectors.  Tolerances: integer/bit work bit-exact; fp64 KernelSHAP rtol 1e-10 (device
binomial via lgamma vs scipy); fp32 GNN outputs atol 1e-5; surrogate weights / explanation
scores atol 1e-4 (BASELINE north_star: 1e-4 fp32)."""
import copy
import math

import numpy as np
import pytest
import torch

import oracle
from golden_utils import CASES, GOLDEN, load_case, oracle_spec, repeat_masks, state_dict

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from bikg_graph_explainability_public_amd import _lib
    _lib.load()


def _eng():
    from bikg_graph_explainability_public_amd import engine
    return engine


@pytest.fixture(params=["rows", "fused", "unfused", "wide", "wide-exact", "wide-gather"])
def fwd_path(request, monkeypatch):
    """xpg_masked_forward has four HIP paths: the lanes-=-rows fused kernel for 1-2 layer plans
    (default for small frontiers), the wave-per-row fused kernel (XPG_FORWARD=fused), the
    32-samples-per-pass wide path for 2-layer plans (XPG_FORWARD=wide; default for frontiers of
    8192+ nodes) and the multi-kernel path (XPG_FORWARD=unfused, also the fallback for plans the
    others do not take).  "wide-exact" = layer 2 on the exact fp32 MFMA instead of the
    three-piece bf16 products (XPG_WIDE_B3=0); "wide-gather" = the wide path with its
    16-lane-group gather layer-1 kernel instead of k_wide_l1s (the kernel plans that k_wide_l1s
    does not take run; a diagnostics switch)."""
    monkeypatch.setenv("XPG_FORWARD", request.param.split("-")[0])
    if request.param == "wide-exact":
        monkeypatch.setenv("XPG_WIDE_B3", "0")
    if request.param == "wide-gather":
        monkeypatch.setenv("XPG_DIAGNOSTICS", "1")
        monkeypatch.setenv("XPG_WIDE_L1_GATHER", "1")
    return request.param


# ------------------------------------------------------------------ masks / perturbation
@pytest.mark.parametrize("shape", [(1, 1), (3, 7), (5, 31), (7, 32), (9, 33), (64, 1177),
                                   (513, 20000)])
def test_pack_unpack_roundtrip(shape):
    e = _eng()
    g = torch.Generator().manual_seed(shape[0] * 131 + shape[1])
    m = torch.rand(shape, generator=g) < 0.37
    bits = e.pack_masks(m.to(DEV))
    np.testing.assert_array_equal(bits.cpu().numpy().view(np.uint32), oracle.pack_bits(m.numpy()))
    back = e.unpack_masks(bits, shape[1]).cpu()
    assert torch.equal(back, m)


def test_edge_keep_known_answer_and_random():
    """tests/test_data.py:1761-1845 vectors, then random graphs vs the oracle."""
    e = _eng()
    m = torch.tensor([[1, 0, 1, 0, 1, 0, 1], [1, 1, 1, 1, 0, 0, 0], [0, 0, 0, 0, 1, 1, 1]],
                     dtype=torch.bool)
    ei = torch.tensor([[0, 2, 3, 6, 4, 5], [5, 6, 4, 1, 2, 0]])
    keep = e.edge_keep(e.pack_masks(m.to(DEV)), 7, ei[0], ei[1]).cpu().numpy()
    assert np.flatnonzero(keep).tolist() == [1, 4]
    rng = np.random.default_rng(3)
    for S, E, B in [(50, 300, 17), (1000, 5000, 40)]:
        mm = rng.random((B, S)) < 0.5
        eei = rng.integers(0, S, (2, E))
        got = e.edge_keep(e.pack_masks(torch.as_tensor(mm).to(DEV)), S,
                          torch.as_tensor(eei[0]), torch.as_tensor(eei[1])).cpu().numpy()
        ref, _ = oracle.build_edge_mask(mm, eei)
        np.testing.assert_array_equal(got, ref)


def test_rows_no_edge_vs_edge_keep_oracle():
    """xpg_rows_no_edge (the multi-node-type loop's empty copies, model.py:213-215) == no kept
    edge in the oracle's edge mask, on sparse rows (many empty), all-off / all-on rows, edges
    past the first 64-edge round, and an edge list of a single edge."""
    e = _eng()
    rng = np.random.default_rng(9)
    for S, E, B, dens in [(50, 300, 40, 0.05), (1000, 5000, 70, 0.01), (700, 1, 20, 0.5),
                          (3000, 200, 33, 0.03)]:
        mm = rng.random((B, S)) < dens
        mm[0] = False
        mm[1] = True
        eei = rng.integers(0, S, (2, E))
        got = e.rows_no_edge(e.pack_masks(torch.as_tensor(mm).to(DEV)), S,
                             torch.as_tensor(eei[0]), torch.as_tensor(eei[1])).cpu().numpy()
        ref, _ = oracle.build_edge_mask(mm, eei)
        np.testing.assert_array_equal(got, ~ref.reshape(B, E).any(1))
        assert got[0] and not got[1]


def test_perturb_node_seam():
    from bikg_graph_explainability_public_amd.data import Data
    m = torch.tensor([[1, 0, 1, 0, 1, 0, 1], [1, 1, 1, 1, 0, 0, 0], [0, 0, 0, 0, 1, 1, 1]],
                     dtype=torch.bool, device=DEV)
    ei = torch.tensor([[0, 2, 3, 6, 4, 5], [5, 6, 4, 1, 2, 0]], device=DEV)
    pe, et = Data(torch.zeros(7, 4, device=DEV), ei).perturb_node(
        m, torch.tensor([0, 0, 0, 1, 1, 1], device=DEV))
    assert pe.cpu().tolist() == [[2, 4], [6, 2]] and et.cpu().tolist() == [0, 1]


def test_shapley_sampler_properties():
    e = _eng()
    R, S = 4096, 1255
    a = e.sample_shapley(7, R, S, DEV)
    b = e.sample_shapley(7, R, S, DEV)
    assert torch.equal(a, b)
    m = e.unpack_masks(a, S).float()
    dens = m.mean().item()
    assert abs(dens - 0.5) < 0.005
    assert abs(m.mean(0) - 0.5).max().item() < 0.05
    tail = a.cpu().numpy().view(np.uint32)[:, -1] >> (S % 32)
    assert (tail == 0).all()
    part = e.sample_shapley(7, 100, S, DEV, row_offset=1000)
    assert torch.equal(part, a[1000:1100])
    c = e.sample_shapley(8, R, S, DEV)
    assert not torch.equal(a, c)
    # one call per repeat set (Explainer.run): set k == sample_shapley(seeds[k]) bit for bit
    seeds = [7, 2 ** 62 - 1, 8, 2 ** 64 - 5]
    sets = e.sample_shapley_sets(seeds, 300, S, DEV)
    assert sets.shape == (4, 300, (S + 31) // 32)
    for k, s in enumerate(seeds):
        assert torch.equal(sets[k], e.sample_shapley(s, 300, S, DEV))
    assert e.sample_shapley_sets([], 300, S, DEV).shape == (0, 300, (S + 31) // 32)


def test_shapley_sampler_device_seed_and_graph_replay():
    """xpg_sample_shapley_dev (seed read on the device) gives the host-seeded rows bit for bit,
    and a captured HIP graph that advances the seed tensor draws seed s, s+1, ... on its
    replays (the bench's graph-replayed headline step relies on both)."""
    e = _eng()
    R, S = 1000, 1193
    seed_t = torch.full((1,), 41, dtype=torch.int64, device=DEV)
    assert torch.equal(e.sample_shapley_dev(seed_t, R, S, row_offset=77),
                       e.sample_shapley(41, R, S, DEV, row_offset=77))
    big = torch.full((1,), -5, dtype=torch.int64, device=DEV)  # the uint64 bits 2^64 - 5
    assert torch.equal(e.sample_shapley_dev(big, 64, S), e.sample_shapley(2 ** 64 - 5, 64, S, DEV))
    out = torch.empty((R, (S + 31) // 32), dtype=torch.int32, device=DEV)
    e.sample_shapley_dev(seed_t, R, S)  # warm-up outside the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with _eng().capture_guard(), torch.cuda.graph(g):
        out.copy_(e.sample_shapley_dev(seed_t, R, S))
        seed_t.add_(1)
    for s in (41, 42, 43):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, e.sample_shapley(s, R, S, DEV))


def _community_case(S, lens, samples, seed=0):
    from bikg_graph_explainability_public_amd.masks import Mask
    rng = np.random.default_rng(seed)
    perm = rng.permutation(S)
    pathways, o = [], 0
    for n in lens:
        pathways.append(sorted(perm[o:o + n].tolist()))
        o += n
    m = Mask(torch.zeros((S, 1)), torch.zeros((2, 0), dtype=torch.long), pathways,
             {"interpret_samples": samples, "epochs": 2}, "node_prediction")
    return pathways, m.community_plan()


@pytest.mark.parametrize("S, lens, samples", [(300, [40, 7, 2, 1, 25, 60, 3], 100),
                                              (3000, [1000, 700, 33, 300, 5], 2000),
                                              (70, [70], 10),
                                              (4000, [20] * 100 + [7] * 50, 500),  # LDS flags
                                              (20000, [5000, 3000, 40, 7], 200)])  # unstaged
def test_community_sampler_structure(S, lens, samples):
    """Device community sampler (masks.py:81-194, pathways.py:234-385), unshuffled: every block
    row has the reference's structure — uncovered columns off; internal rows touch only the own
    community; external rows switch whole communities, the sorted-position column off, and the
    first 2h rows are antithetic pairs; pathway_rows = the own community.  Shuffled: the same
    rows, permuted.  Deterministic in the seed."""
    e = _eng()
    pathways, plan = _community_case(S, lens, samples)
    blocks, src_rows, rows, _ = plan
    bits, prow = e.sample_communities(5, (blocks, src_rows, src_rows, False), pathways, S, DEV)
    m = e.unpack_masks(bits, S).cpu().numpy()
    prow = prow.cpu().numpy()
    covered = np.zeros(S, bool)
    for p in pathways:
        covered[p] = True
    assert not m[:, ~covered].any()
    tail = bits.cpu().numpy().view(np.uint32)[:, -1] >> (S % 32) if S % 32 else 0
    assert np.all(tail == 0)
    P = len(pathways)
    own_bits = []
    for start, size, size_int, own, off in blocks.tolist():
        blk = m[start:start + size]
        assert (prow[start:start + size] == own).all()
        own_bits.append(blk[:, pathways[own]])
        others = [c for c in range(P) if c != own]
        if not others:
            continue
        flags = np.stack([blk[:, pathways[c]].all(1) for c in others], 1)
        anyon = np.stack([blk[:, pathways[c]].any(1) for c in others], 1)
        assert np.array_equal(flags, anyon)                # whole communities switch together
        assert not anyon[:size_int].any()                  # internal rows: own community only
        if off != own:
            assert not flags[size_int:, others.index(off)].any()
        h = (size - size_int) // 2
        keep = [i for i, c in enumerate(others) if c != off]
        a, b = flags[size_int:size_int + h][:, keep], flags[size_int + h:size_int + 2 * h][:, keep]
        assert np.array_equal(a, ~b)                       # antithetic pairs
    ob = np.concatenate([x.ravel() for x in own_bits])
    assert abs(ob.mean() - 0.5) < 0.05
    # shuffled: a permutation of the same rows; deterministic; seed-dependent
    sb, sp = e.sample_communities(5, (blocks, src_rows, src_rows, True), pathways, S, DEV)
    key = lambda x: sorted(map(bytes, x.cpu().numpy().view(np.uint8).reshape(x.shape[0], -1)))
    assert key(sb) == key(bits) and not torch.equal(sb, bits)
    assert np.array_equal(np.sort(sp.cpu().numpy()), np.sort(prow))
    sb2, _ = e.sample_communities(5, (blocks, src_rows, src_rows, True), pathways, S, DEV)
    assert torch.equal(sb, sb2)
    sb3, _ = e.sample_communities(6, (blocks, src_rows, src_rows, True), pathways, S, DEV)
    assert not torch.equal(sb, sb3)
    tb, tp = e.sample_communities(5, plan, pathways, S, DEV)
    assert tb.shape[0] == rows
    # a rank's shard: rows [a, b) of the repeat == the same rows of the full call (shuffled and
    # truncated plans), the pathway rows too
    for a_, b_ in [(0, 1), (rows // 3, rows // 3 + 5), (rows - 7, rows), (1, rows)]:
        if not 0 <= a_ < b_ <= rows:
            continue
        pb, pp = e.sample_communities(5, plan, pathways, S, DEV, row_offset=a_, rows=b_ - a_)
        assert torch.equal(pb, tb[a_:b_]) and torch.equal(pp, tp[a_:b_])
    # out=: written in place into a slice of a bigger buffer, the rows around it untouched
    big = torch.full((rows + 6, tb.shape[1]), -7, dtype=torch.int32, device=DEV)
    ob, _ = e.sample_communities(5, plan, pathways, S, DEV, out=big[3:3 + rows])
    assert ob.data_ptr() == big[3].data_ptr() and torch.equal(big[3:3 + rows], tb)
    assert bool((big[:3] == -7).all()) and bool((big[3 + rows:] == -7).all())
    with pytest.raises(ValueError):
        e.sample_communities(5, plan, pathways, S, DEV, out=big[:rows, :-1])
    with pytest.raises(ValueError):
        e.sample_communities(5, plan, pathways, S, DEV, row_offset=rows - 1, rows=2)


@pytest.mark.parametrize("S, lens, samples, overlap", [(300, [40, 7, 2, 1, 25, 60, 3], 100, 0),
                                                       (3000, [1000, 700, 33, 300, 5], 2000, 0),
                                                       (70, [70], 10, 0),
                                                       (700, [10] * 64, 300, 0),
                                                       (1436, [72] * 20, 2000, 150),
                                                       (5, [2, 2, 1], 4, 2)])
def test_community_sampler_column_masks_equal_per_column_rule(S, lens, samples, overlap,
                                                              monkeypatch):
    """The column-bitmask sampler (one mask per community in LDS, a word per lane) writes the
    same bits and pathway rows as the per-column lookup (XPG_COMM_PERCOL=1), overlapping members
    included, shuffled / unshuffled, whole repeat and row ranges (words > 64 too)."""
    e = _eng()
    pathways, _ = _community_case(S, lens, samples)
    rng = np.random.default_rng(3)
    for _ in range(overlap):  # members shared by two communities
        a, b = rng.choice(len(pathways), 2, replace=False)
        pathways[b] = sorted(set(pathways[b]) | {int(rng.choice(pathways[a]))})
    from bikg_graph_explainability_public_amd.masks import Mask
    plan = Mask(torch.zeros((S, 1)), torch.zeros((2, 0), dtype=torch.long), pathways,
                {"interpret_samples": samples, "epochs": 2}, "node_prediction").community_plan()
    blocks, src_rows, rows, _ = plan
    outs = {}
    monkeypatch.setenv("XPG_DIAGNOSTICS", "1")
    for mode in ("0", "1"):
        monkeypatch.setenv("XPG_COMM_PERCOL", "1" if mode == "0" else "0")
        outs[mode] = [e.sample_communities(s, (blocks, src_rows, src_rows, sh), pathways, S, DEV)
                      for s in (5, 9) for sh in (False, True)]
        outs[mode].append(e.sample_communities(5, plan, pathways, S, DEV, row_offset=rows // 3,
                                               rows=rows - rows // 3))
    for (b0, p0), (b1, p1) in zip(outs["0"], outs["1"]):
        assert torch.equal(b0, b1) and torch.equal(p0, p1)


def test_community_sampler_dead_mask_and_overlap():
    """Lone external rows with no community on get one other community switched on
    (activate_dead_mask, pathways.py:285-334); overlapping members are on if any active
    community holds them, except own-community members, which take the internal bits.
    Distinct lengths fix the order, so own == off in every block and the switched-on community
    is always visible (without the activation a quarter of these rows would be empty)."""
    e = _eng()
    from bikg_graph_explainability_public_amd.masks import Mask
    pathways = [[0, 1, 2], [2, 3], [4]]
    m = Mask(torch.zeros((5, 1)), torch.zeros((2, 0), dtype=torch.long), pathways,
             {"interpret_samples": 2, "epochs": 1}, "node_prediction")
    blocks, src_rows, rows, _ = m.community_plan()
    assert blocks.tolist() == [[0, 2, 1, 0, 0], [2, 2, 1, 1, 1], [4, 2, 1, 2, 2]]
    for seed in range(64):
        bits, _ = e.sample_communities(seed, (blocks, src_rows, src_rows, False), pathways, 5, DEV)
        mm = e.unpack_masks(bits, 5).cpu().numpy()
        for start, size, size_int, own, off in blocks.tolist():
            row = mm[start + 1]                            # the lone external row
            outside = [s for s in range(5) if s not in pathways[own]]
            on = [c for c in range(3) if c != own
                  and all(row[s] for s in pathways[c] if s not in pathways[own])]
            assert on, f"seed {seed}: dead external row in block {own}"
            want = np.zeros(5, bool)
            for c in on:
                want[pathways[c]] = True
            assert np.array_equal(row[outside], want[outside])


# ------------------------------------------------------------------ KernelSHAP
@pytest.mark.parametrize("cols", [9, 200, 1001, 1002, 1500, 3000, 20000])
def test_shap_kernel_vs_reference(cols):
    e = _eng()
    z = np.load(GOLDEN + "/kernels.npz")
    m = np.unpackbits(z[f"c{cols}_mask_bits"], axis=1, bitorder="little")[:, :cols].astype(bool)
    got = e.shap_kernel(e.pack_masks(torch.as_tensor(m).to(DEV)), cols).cpu().numpy()
    ref = z[f"c{cols}_kernel"]
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=0)
    np.testing.assert_array_equal(got == 0, ref == 0)


@pytest.mark.parametrize("rows", ["all_active", "all_active_and_empty", "one_empty"])
def test_shap_kernel_approx_backoff_edge_batches(rows):
    """The approximate branch's back-off loop (kernels.py:148-162) runs while the kernel SUMS to
    0: a batch of all-active rows has a negative sum (quirk Q5) and must stop at ref = 1000 like
    the reference (a test for 'some value > 0' would back off ~60 times and return other values);
    an empty row is +inf (sum +inf: stop, then cleaned to 0); a lone empty row sums to +inf too."""
    e = _eng()
    cols = 1500
    m = {"all_active": np.ones((5, cols), bool),
         "all_active_and_empty": np.concatenate([np.ones((3, cols), bool), np.zeros((2, cols), bool)]),
         "one_empty": np.zeros((1, cols), bool)}[rows]
    got = e.shap_kernel(e.pack_masks(torch.as_tensor(m).to(DEV)), cols).cpu().numpy()
    ref = oracle.shap_kernel(m)
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=0)
    np.testing.assert_array_equal(got == 0, ref == 0)
    if rows == "all_active":
        assert (ref < 0).all()


def test_kernel_class_seam():
    from bikg_graph_explainability_public_amd.kernels import Kernel
    m = torch.tensor([[1, 0, 1, 0, 1, 0, 1, 0, 0], [0, 1, 0, 1, 0, 1, 0, 1, 1],
                      [1, 1, 0, 0, 0, 1, 1, 1, 0], [1, 0, 1, 1, 1, 0, 0, 0, 1]],
                     dtype=torch.bool, device=DEV)
    k = Kernel(m).compute().cpu().numpy()
    np.testing.assert_allclose(k, oracle.shap_kernel(m.cpu().numpy()), rtol=1e-12)
    assert abs(k.mean() - 1 / 315) < 1e-3  # tests/test_wlm.py:280-291 (~1/305 within 1e-3)


# ------------------------------------------------------------------ dense MFMA
@pytest.mark.parametrize("M,K,N", [(1, 8, 1), (31, 12, 5), (32, 64, 32), (100, 84, 16),
                                   (257, 128, 256), (1000, 64, 64), (4099, 256, 200)])
def test_dense_mfma_vs_torch_fp32(M, K, N):
    e = _eng()
    g = torch.Generator().manual_seed(M + K + N)
    A = torch.randn((M, K), generator=g)
    W = torch.randn((N, K), generator=g) * torch.linspace(0.5, 2.0, K)  # asymmetric
    b = torch.randn(N, generator=g)
    for act, fn in [(None, lambda x: x), ("relu", torch.relu), ("sigmoid", torch.sigmoid)]:
        got = e.dense(A.to(DEV), W.to(DEV), b.to(DEV), act).cpu()
        ref = fn(A.double() @ W.double().T + b.double()).float()
        torch.testing.assert_close(got, ref, rtol=0, atol=2e-5 * max(1.0, K ** 0.5))


# ------------------------------------------------------------------ masked forward
def _plan_for(name):
    from bikg_graph_explainability_public_amd import pipeline
    from case_builders import build_explainer
    exp, z, meta = build_explainer(name)
    exp.arch = exp.arch.to(DEV)
    ctx = exp.prepare(meta["element"], DEV)
    plan = pipeline.build_plan(exp.arch, ctx["sub_feat"], ctx["sub_ei"], [ctx["sub_ind"]],
                               ctx["sub_nt"], ctx["sub_et"], ctx["h_ntypes"], ctx["h_etypes"],
                               ctx["padded_dims"])
    return exp, z, meta, ctx, plan


@pytest.mark.parametrize("name", CASES)
def test_masked_forward_vs_reference_outputs(name, fwd_path):
    e = _eng()
    exp, z, meta, ctx, plan = _plan_for(name)
    assert plan is not None, "engine must compile every golden architecture"
    for i, m in enumerate(repeat_masks(z, meta)):
        y = plan.forward(e.pack_masks(torch.as_tensor(m).to(DEV)))[:, 0].cpu().numpy()
        np.testing.assert_allclose(y, z[f"r{i}_output"], rtol=0, atol=1e-5)


def test_masked_forward_vs_oracle_fp64(fwd_path):
    """Same as above against the fp64 oracle on fresh random masks (all golden archs)."""
    e = _eng()
    from test_oracle_golden import prepare
    for name in CASES:
        zz, meta, spec, sub_x, rel_ei, sub_ind = prepare(name)
        exp, z, meta, ctx, plan = _plan_for(name)
        rng = np.random.default_rng(len(name))
        m = rng.random((97, sub_x.shape[0])) < rng.random((97, 1))
        ref = oracle.masked_query_outputs(spec, sub_x, rel_ei, m, sub_ind)
        got = plan.forward(e.pack_masks(torch.as_tensor(m).to(DEV)))[:, 0].cpu().numpy()
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-5)


@pytest.mark.parametrize("S, R, B", [(1193, 12800, 256), (300, 640, 64)])
def test_prepared_fit_equals_fit_from(S, R, B):
    """xpg_wlm_prepare + xpg_wlm_fit_prepared (engine.PreparedFit) == xpg_wlm_fit_from bit for
    bit (w, losses, best epoch), twice on the same instance (the second prepare resets w / m / v
    and the exchange slots; the second time as xpg_wlm_fit_steps + xpg_wlm_fit_losses, the
    losses on another stream), and two instances interleaved as the pipelined bench uses them."""
    e = _eng()
    params = {"lr": 0.01, "l1_lambda": 1e-4}
    g = torch.Generator().manual_seed(S)
    fits = []
    for s in range(2):
        bits = e.sample_shapley(50 + s, R, S, DEV)
        y = torch.rand(R, generator=g).to(DEV)
        k = e.shap_kernel(bits, S)
        w0 = (torch.rand((1, S), generator=g) - 0.5).to(DEV)
        ref = e.wlm_fit(bits.view(1, R, -1), S, B, y.view(1, R), k.view(1, R), w0, params)
        fits.append((bits, y, k, w0, ref))
    pf = [e.PreparedFit(1, R, S, B, params, DEV), e.PreparedFit(1, R, S, B, params, DEV)]
    for rep in range(2):
        for i, (bits, y, k, w0, ref) in enumerate(fits):
            pf[i].prepare(bits, y, k, w0)
        for i, (bits, y, k, w0, ref) in enumerate(fits):
            if rep == 0:
                w = pf[i].fit(bits, k)
            else:  # the split launches (ABI v17): steps, then losses on a second stream
                w = pf[i].fit_steps(bits, k)
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    pf[i].finish(k)
                torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            e.check_fit_status(pf[i].status)
            assert torch.equal(w, ref[0]), (rep, i)
            assert torch.equal(pf[i].losses, ref[1]) and torch.equal(pf[i].best, ref[2])


def test_pipelined_prepared_fits_equal_eager():
    """bench.py's pipelined form: two PreparedFit buffer sets and a captured graph of two
    consecutive steps, where step j fits set j & 1 on the capture stream while the next repeat's
    masks -> forward -> KernelSHAP -> fit prologue fill the other set on a side stream.  Every
    step of every replay equals the eager fit_from on the same seed bit for bit (w and losses),
    and both sets' sticky status words stay clean over all replays."""
    e = _eng()
    exp, z, meta, ctx, plan = _plan_for(CASES[0])
    S, R, B = plan.cols, 640, 64
    W, steps = (S + 31) // 32, -(-R // B)
    params = {"lr": 0.01, "l1_lambda": 1e-4}
    w0 = torch.zeros((1, S), device=DEV)
    seed_t = torch.full((1,), 700, dtype=torch.int64, device=DEV)
    sets = [dict(bits=torch.empty((R, W), dtype=torch.int32, device=DEV),
                 y=torch.empty((R, 1), dtype=torch.float32, device=DEV),
                 k=torch.empty(R, dtype=torch.float64, device=DEV),
                 cnt=torch.empty(R, dtype=torch.int32, device=DEV),
                 fit=e.PreparedFit(1, R, S, B, params, DEV)) for _ in range(2)]
    snaps = [(torch.empty((1, S), device=DEV), torch.empty((1, steps), dtype=torch.float64, device=DEV))
             for _ in range(2)]
    s1 = torch.cuda.Stream(device=DEV)

    def produce(d):
        e.sample_shapley_dev(seed_t, R, S, out=d["bits"])
        seed_t.add_(1)
        plan.forward(d["bits"], out=d["y"])
        e.shap_kernel(d["bits"], S, out=d["k"], scratch=d["cnt"])
        d["fit"].prepare(d["bits"], d["y"][:, 0], d["k"], w0)

    prod_ev = torch.cuda.Event()

    def pipe_step(i, snap):  # bench.py's form: the fit's losses and outputs on the side stream
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        d = sets[i]
        w = d["fit"].fit_steps(d["bits"], d["k"])
        with torch.cuda.stream(s1):
            produce(sets[1 - i])
            prod_ev.record(s1)
            s1.wait_stream(cur)
            d["fit"].finish(d["k"])
            snap[0].copy_(w)
            snap[1].copy_(d["fit"].losses)
        cur.wait_event(prod_ev)

    produce(sets[0])  # prologue: seed 700
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with _eng().capture_guard(), torch.cuda.graph(g):
        for j in range(2):
            pipe_step(j, snaps[j])
        torch.cuda.current_stream().wait_stream(s1)
    for rep in range(3):
        g.replay()
        torch.cuda.synchronize()
        for j in range(2):
            seed = 700 + 2 * rep + j
            bits = e.sample_shapley(seed, R, S, DEV)
            y = plan.forward(bits)[:, 0]
            k = e.shap_kernel(bits, S)
            ref = e.wlm_fit(bits.view(1, R, -1), S, B, y.view(1, R), k.view(1, R), w0, params)
            assert torch.equal(snaps[j][0], ref[0]), (rep, j)
            assert torch.equal(snaps[j][1], ref[1]), (rep, j)
    for d in sets:
        e.check_fit_status(d["fit"].status)


def test_captured_repeat_equals_eager():
    """One repeat (device-seeded masks -> masked forward, KernelSHAP on a side stream ->
    fresh surrogate fit) captured in a HIP graph, as bench.py's headline replays it: every
    replay gives bitwise the eager repeat on seed s, s+1, ...  The side stream must fork from
    the CAPTURE stream, or its kernels run once at capture time and never replay."""
    e = _eng()
    exp, z, meta, ctx, plan = _plan_for(CASES[0])
    S, R, B = plan.cols, 640, 64
    params = {"lr": 0.01, "l1_lambda": 1e-4}
    w0 = torch.zeros((1, S), device=DEV)
    seed_t = torch.full((1,), 300, dtype=torch.int64, device=DEV)
    k_buf = torch.empty(R, dtype=torch.float64, device=DEV)
    cnt_buf = torch.empty(R, dtype=torch.int32, device=DEV)
    st = torch.zeros(1, dtype=torch.int32, device=DEV)
    side = torch.cuda.Stream(device=DEV)

    def repeat(dev_seed, seed=None):
        cur = torch.cuda.current_stream()
        bits = e.sample_shapley_dev(seed_t, R, S) if dev_seed else e.sample_shapley(seed, R, S, DEV)
        side.wait_stream(cur)
        y = plan.forward(bits)[:, 0]
        with torch.cuda.stream(side):
            k = e.shap_kernel(bits, S, out=k_buf, scratch=cnt_buf) if dev_seed else e.shap_kernel(bits, S)
        cur.wait_stream(side)
        w = e.wlm_fit(bits.view(1, R, -1), S, B, y.view(1, R), k.view(1, R), w0, params,
                      check=False, status=st)[0]
        if dev_seed:
            seed_t.add_(1)
        return w

    repeat(True)  # workspaces allocated outside the capture
    seed_t.fill_(300)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with _eng().capture_guard(), torch.cuda.graph(g):
        w_g = repeat(True)
    for s in (300, 301, 302):
        g.replay()
        torch.cuda.synchronize()
        e.check_fit_status(st)
        w_e = repeat(False, s)
        torch.cuda.synchronize()
        assert torch.isfinite(w_g).all()
        assert torch.equal(w_g, w_e), s


@pytest.mark.parametrize("kind,dims,fc", [("gcn", [16, 32], [32, 1]),
                                           ("sage", [16, 32], [32, 8, 1]),
                                           ("gcn", [16, 128, 64], [64, 1]),
                                           ("sage", [16, 64, 32], [32, 16, 1]),
                                           ("gcn", [16, 32, 32, 32], [32, 1])])
def test_masked_forward_synthetic_archs(kind, dims, fc, fwd_path):
    """1-, 2- and 3-layer GCN / SAGE stacks of several widths (each fused kernel's template
    variants and the fallback) on a random graph with self-loops and duplicate edges, vs the
    fp64 oracle."""
    from golden_utils import oracle_spec
    from bikg_graph_explainability_public_amd import pipeline
    from bikg_graph_explainability_public_amd.nn import ConvStack
    e = _eng()
    g = torch.Generator().manual_seed(17)
    S, E = 300, 1500
    x = torch.randn((S, dims[0]), generator=g)
    ei = torch.randint(0, S, (2, E), generator=g)
    ei[:, :20] = ei[0, :20]  # self-loops
    ei[:, 20:40] = ei[:, 40:60]  # duplicate edges
    torch.manual_seed(3)
    arch = ConvStack(kind, dims, fc).eval()
    q = int(ei[1, 100])
    plan = pipeline.build_plan(arch.to(DEV), x.to(DEV), ei.to(DEV), [q])
    spec = oracle_spec({"arch_spec": {"kind": kind, "dims": dims, "fc": fc}},
                       {k: v.detach().cpu().numpy() for k, v in arch.state_dict().items()})
    rng = np.random.default_rng(5)
    m = rng.random((130, S)) < rng.random((130, 1))
    ref = oracle.masked_query_outputs(spec, x.numpy(), {None: ei.numpy()}, m, q)
    got = plan.forward(e.pack_masks(torch.as_tensor(m).to(DEV)))[:, 0].cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-5)


@pytest.mark.parametrize("kind,dims,fc", [("gcn", [16, 32, 32], [32, 1]),
                                           ("sage", [16, 64, 64], [64, 8, 1]),
                                           ("sage", [24, 128, 128], [128, 1]),
                                           ("gcn", [16, 64, 128], [128, 16, 1])])
def test_full_graph_forward_all_targets(kind, dims, fc, fwd_path):
    """Every node a target (the full-graph regime): outputs of all S nodes per
    mask row in one plan, vs the fp64 oracle run per query, on a graph with self-loops and
    duplicate edges; 70 rows = two full 32-sample passes of the wide path plus a partial one."""
    from golden_utils import oracle_spec
    from bikg_graph_explainability_public_amd import pipeline
    from bikg_graph_explainability_public_amd.nn import ConvStack
    e = _eng()
    g = torch.Generator().manual_seed(23)
    S, E = 400, 2400
    x = torch.randn((S, dims[0]), generator=g)
    ei = torch.randint(0, S, (2, E), generator=g)
    ei[:, :25] = ei[0, :25]  # self-loops
    ei[:, 25:50] = ei[:, 50:75]  # duplicate edges
    torch.manual_seed(4)
    arch = ConvStack(kind, dims, fc).eval()
    plan = pipeline.build_plan(arch.to(DEV), x.to(DEV), ei.to(DEV), list(range(S)))
    spec = oracle_spec({"arch_spec": {"kind": kind, "dims": dims, "fc": fc}},
                       {k: v.detach().cpu().numpy() for k, v in arch.state_dict().items()})
    rng = np.random.default_rng(9)
    m = rng.random((70, S)) < rng.random((70, 1))
    m[0] = True
    m[1] = False
    got = plan.forward(e.pack_masks(torch.as_tensor(m).to(DEV))).cpu().numpy()
    assert got.shape == (70, S)
    pos = plan.frontiers[-1]  # output column i is node pos[i]
    for i in list(range(0, S, 37)) + [S - 1]:
        ref = oracle.masked_query_outputs(spec, x.numpy(), {None: ei.numpy()}, m, int(pos[i]))
        np.testing.assert_allclose(got[:, i], ref, rtol=0, atol=1e-5)


def test_generic_path_matches_engine():
    from bikg_graph_explainability_public_amd import pipeline
    for name in ["test_run", "hetero_single", "sage_shapley"]:
        exp, z, meta, ctx, plan = _plan_for(name)
        ok, err = pipeline.verify_plan(plan, exp.arch, ctx["sub_feat"], ctx["sub_ei"],
                                       ctx["sub_ind"], ctx["sub_nt"], ctx["sub_et"],
                                       ctx["h_ntypes"], ctx["h_etypes"], ctx["padded_dims"],
                                       rows=16)
        assert ok, (name, err)


# ------------------------------------------------------------------ surrogate
@pytest.mark.parametrize("wlm_path", ["auto", "mc"])
@pytest.mark.parametrize("name", CASES)
def test_wlm_fit_vs_reference(name, wlm_path, monkeypatch):
    if wlm_path != "auto":
        monkeypatch.setenv("XPG_WLM", wlm_path)
    e = _eng()
    z, meta = load_case(name)
    for i, m in enumerate(repeat_masks(z, meta)):
        bits = e.pack_masks(torch.as_tensor(m).to(DEV))
        w, losses, best, _, _ = e.wlm_fit(bits, m.shape[1], meta[f"r{i}_batch_size"],
                                          torch.as_tensor(z[f"r{i}_output"]),
                                          torch.as_tensor(z[f"r{i}_kernel"]),
                                          torch.as_tensor(z[f"r{i}_w0"]), meta["params"])
        np.testing.assert_allclose(w.cpu().numpy(), z[f"r{i}_w_final"], rtol=0, atol=1e-4)
        np.testing.assert_allclose(losses.cpu().numpy(), z[f"r{i}_losses"], rtol=1e-4)
        assert int(best.item()) == meta[f"r{i}_best_epoch"]


@pytest.mark.parametrize("R,S,B", [(4096, 3000, 512),   # 3 columns per thread, LDS too small
                                   (12800, 1193, 256),  # the c2 bench shape (LDS-staged)
                                   (3000, 1193, 256),   # short last batch (quirk Q7)
                                   (2000, 700, 100),    # batch not a multiple of 32
                                   (640, 4100, 64)])    # > 4096 columns
@pytest.mark.parametrize("wlm_path", ["single", "mc", "grid", "grid3"])
def test_wlm_fit_vs_oracle_large(R, S, B, wlm_path, monkeypatch):
    """Fresh data vs the fp64 oracle at sizes the golden fixtures do not reach, through each of
    the fit kernels: one workgroup per fit (XPG_WLM=single), P co-resident workgroups per fit
    (mc, the default from 256 columns), the many-column grid fit (S > 16384) as one persistent
    launch (grid: k_gw_fused) and as three launches per step (grid3)."""
    monkeypatch.setenv("XPG_WLM", wlm_path)
    e = _eng()
    if wlm_path.startswith("grid"):
        assert e.wlm_plan(1, R, S, B)[0] == ("grid_fused" if wlm_path == "grid" else "grid")
    rng = np.random.default_rng(11)
    m = rng.random((R, S)) < 0.5
    y = rng.random(R).astype(np.float32)
    k = oracle.shap_kernel(m)
    w0 = ((rng.random(S) - 0.5) * 0.05).astype(np.float32)
    params = {"lr": 0.01, "l1_lambda": 1e-4}
    ref, rl, rb = oracle.train_wlm(m, B, y, k, w0, params)
    w, losses, best, _, _ = e.wlm_fit(e.pack_masks(torch.as_tensor(m).to(DEV)), S, B,
                                      torch.as_tensor(y), torch.as_tensor(k),
                                      torch.as_tensor(w0), params)
    np.testing.assert_allclose(w.cpu().numpy(), ref, rtol=0, atol=1e-4)
    np.testing.assert_allclose(losses.cpu().numpy(), rl, rtol=1e-5)


def test_wlm_fit_midsize_many_fits_multi_vs_oracle():
    """S = 10,000 columns, 8 fits in one launch (the graph_queries shape, batch 256): the
    multi-workgroup fit takes it with more than 16 parts per fit (two poll rounds; it went to
    the single-workgroup fit before), every fit vs the fp64 oracle."""
    e = _eng()
    F, R, S, B = 8, 2560, 10_000, 256
    kind, parts = e.wlm_plan(F, R, S, B)
    assert kind == "multi" and parts > 16, (kind, parts)
    rng = np.random.default_rng(8)
    m = rng.random((F, R, S)) < 0.5
    y = rng.random((F, R)).astype(np.float32)
    k = np.stack([oracle.shap_kernel(m[f]) for f in range(F)])
    w0 = ((rng.random((F, S)) - 0.5) * 0.02).astype(np.float32)
    params = {"lr": 0.01, "l1_lambda": 1e-4}
    bits = torch.stack([e.pack_masks(torch.as_tensor(m[f]).to(DEV)) for f in range(F)])
    w, losses, best, _, _ = e.wlm_fit(bits, S, B, torch.as_tensor(y), torch.as_tensor(k),
                                      torch.as_tensor(w0), params)
    for f in range(F):
        ref, rl, rb = oracle.train_wlm(m[f], B, y[f], k[f], w0[f], params)
        np.testing.assert_allclose(w[f].cpu().numpy(), ref, rtol=0, atol=1e-4)
        np.testing.assert_allclose(losses[f].cpu().numpy(), rl, rtol=1e-5)
        assert int(best[f]) == rb


def test_wlm_fit_many_columns_vs_oracle():
    """S = 40,000 columns (> 16384: the grid fit), two independent fits in one call."""
    e = _eng()
    rng = np.random.default_rng(3)
    F, R, S, B = 2, 768, 40_000, 256
    m = rng.random((F, R, S)) < 0.5
    y = rng.random((F, R)).astype(np.float32)
    k = np.stack([oracle.shap_kernel(m[f]) for f in range(F)])
    w0 = ((rng.random((F, S)) - 0.5) * 0.01).astype(np.float32)
    params = {"lr": 0.01, "l1_lambda": 1e-4}
    bits = torch.stack([e.pack_masks(torch.as_tensor(m[f]).to(DEV)) for f in range(F)])
    w, losses, best, _, _ = e.wlm_fit(bits, S, B, torch.as_tensor(y), torch.as_tensor(k),
                                      torch.as_tensor(w0), params)
    for f in range(F):
        ref, rl, rb = oracle.train_wlm(m[f], B, y[f], k[f], w0[f], params)
        np.testing.assert_allclose(w[f].cpu().numpy(), ref, rtol=0, atol=1e-4)
        np.testing.assert_allclose(losses[f].cpu().numpy(), rl, rtol=1e-5)
        assert int(best[f]) == rb


@pytest.mark.parametrize("F,R,S,B", [(1, 2500, 20_000, 1000),   # 32 row blocks: one chunk per workgroup
                                     (1, 1100, 70_000, 96),     # 3 row blocks, short last batch
                                     (3, 1024, 17_000, 512),    # 3 fits: one launch each
                                     (1, 1500, 20_000, 320),    # 3 waves per chunk (runtime slot sum)
                                     (1, 1400, 40_000, 700)])   # 6 waves per chunk, one chunk
def test_wlm_fit_fused_grid_shapes_vs_oracle(F, R, S, B):
    """The persistent many-column fit (k_gw_fused) on shapes at its limits vs the fp64 oracle:
    the largest batch it holds in registers, a batch that is not a multiple of 32 with a short
    last batch, several fits in one call, and waves per chunk (column-sum slots added by Adam)
    outside the unrolled counts 2 / 4 / 8."""
    e = _eng()
    kind, parts = e.wlm_plan(F, R, S, B)
    assert kind == "grid_fused" and parts >= 1, (kind, parts)
    rng = np.random.default_rng(21)
    m = rng.random((F, R, S)) < 0.5
    y = rng.random((F, R)).astype(np.float32)
    k = np.stack([oracle.shap_kernel(m[f]) for f in range(F)])
    w0 = ((rng.random((F, S)) - 0.5) * 0.02).astype(np.float32)
    params = {"lr": 0.01, "l1_lambda": 1e-4}
    bits = torch.stack([e.pack_masks(torch.as_tensor(m[f]).to(DEV)) for f in range(F)])
    w, losses, best, _, _ = e.wlm_fit(bits, S, B, torch.as_tensor(y), torch.as_tensor(k),
                                      torch.as_tensor(w0), params)
    for f in range(F):
        ref, rl, rb = oracle.train_wlm(m[f], B, y[f], k[f], w0[f], params)
        np.testing.assert_allclose(w[f].cpu().numpy(), ref, rtol=0, atol=1e-4)
        # fp32 predictions summed over up to 70,000 columns vs the fp64 oracle: a loss that is a
        # small difference of such sums carries ~1e-5 relative error in any fp32 order
        np.testing.assert_allclose(losses[f].cpu().numpy(), rl, rtol=5e-5)
        assert int(best[f]) == rb


def _train_wlm_fp64_device(mask, batch, y, k, w0, params):
    """oracle.train_wlm (wlm.py:132-278) restated with torch float64 on the GPU, for fits whose
    mask is too large for the numpy oracle (S = 1M columns): the same per-batch algebra, in fp64
    (test infrastructure: the reference the device fits are checked against)."""
    R, S = mask.shape
    w = w0.double().clone()
    ma = torch.zeros_like(w)
    va = torch.zeros_like(w)
    lr, lam = abs(params["lr"]), params["l1_lambda"]
    b1, b2, eps, wd = 0.9, 0.999, 1e-8, 1e-2
    losses = []
    for t, r0 in enumerate(range(0, R, batch), start=1):
        mb = mask[r0:r0 + batch].double()
        yy, kk = y[r0:r0 + batch].double(), k[r0:r0 + batch].double()
        B = mb.shape[0]
        p = mb @ w
        ksum = kk.sum()
        losses.append(float((kk[None, :] * (p[None, :] - yy[:, None]) ** 2).mean() / ksum +
                            lam * w.abs().mean()))
        g = mb.T @ (2.0 * kk * (p - yy.mean()) / (B * ksum)) + lam * torch.sign(w) / S + wd * w
        ma = ma + (1 - b1) * (g - ma)
        va = b2 * va + (1 - b2) * g * g
        w = w - (lr / (1 - b1 ** t)) * ma / (va.sqrt() / math.sqrt(1 - b2 ** t) + eps)
        del mb
    return w, np.asarray(losses)


@pytest.mark.parametrize("R", [2560, 2300])
def test_wlm_fit_fused_grid_c3_scale_vs_fp64(R, monkeypatch):
    """graph_prediction at the c3 size (S = 1M columns, batch 512: 489 chunks on 245
    workgroups, every workgroup a reducer), R = 2300 ending with a short batch: the persistent
    fit and the three-launch grid fit each against an fp64 restatement of train_wlm run on the
    GPU (the numpy oracle's algebra; it pins both kernels within 1e-4 at smaller S): at most
    0.01 % of the 1M weights more than 1e-5 from the fp64 fit and none more than 5e-4, losses
    within 1e-5 relative, the same best epoch.  (Both fp32 kernels add the same products in
    different orders; Adam's m / sqrt(v) amplifies rounding for columns whose gradient is near
    0, so they are compared with the fp64 fit, not with each other bit for bit.)"""
    e = _eng()
    S, B = 1_000_000, 512
    g = torch.Generator(device=DEV).manual_seed(5)
    mask = torch.rand((R, S), generator=g, device=DEV) < 0.5
    bits = e.pack_masks(mask)
    y = torch.rand(R, generator=g, device=DEV)
    k = torch.rand(R, generator=g, device=DEV, dtype=torch.float64) + 0.5
    w0 = (torch.rand(S, generator=g, device=DEV) - 0.5) * 0.02
    params = {"lr": 0.01, "l1_lambda": 1e-4}
    ref_w, ref_l = _train_wlm_fp64_device(mask, B, y, k, w0, params)
    del mask
    assert e.wlm_plan(1, R, S, B)[0] == "grid_fused"
    w1, l1, b1, _, _ = e.wlm_fit(bits, S, B, y, k, w0, params)
    monkeypatch.setenv("XPG_WLM", "grid3")
    w3, l3, b3, _, _ = e.wlm_fit(bits, S, B, y, k, w0, params)
    best = int(np.argmin(ref_l))
    for name, w, l, b in (("fused", w1, l1, b1), ("grid3", w3, l3, b3)):
        err = (w.double() - ref_w).abs()
        # an fp32 Adam step moves a column by ~lr when its gradient's sign flips under rounding:
        # at 1M columns a handful of near-zero-gradient columns land ~1e-4 from the fp64 fit
        # in ANY fp32 order; every other column stays within 1e-5
        assert float(err.max()) <= 5e-4, (name, float(err.max()))
        assert float((err > 1e-5).double().mean()) <= 1e-4, (name, int((err > 1e-5).sum()))
        np.testing.assert_allclose(l.cpu().numpy(), ref_l, rtol=1e-5, err_msg=name)
        assert int(b[0]) == best, name


def test_wlm_fit_fused_grid_exchange_failure_raises(monkeypatch):
    """A workgroup of the persistent many-column fit that never publishes (test hook) ends the
    fit with the error word set: FitExchangeError, and a clean fit afterwards matches the oracle."""
    from bikg_graph_explainability_public_amd import _lib
    e = _eng()
    rng = np.random.default_rng(4)
    R, S, B = 600, 20_000, 128
    m = rng.random((R, S)) < 0.5
    y = rng.random(R).astype(np.float32)
    k = oracle.shap_kernel(m)
    w0 = ((rng.random(S) - 0.5) * 0.05).astype(np.float32)
    params = {"lr": 0.01, "l1_lambda": 1e-4}
    bits = e.pack_masks(torch.as_tensor(m).to(DEV))
    args = (bits, S, B, torch.as_tensor(y), torch.as_tensor(k), torch.as_tensor(w0), params)
    assert e.wlm_plan(1, R, S, B)[0] == "grid_fused"
    monkeypatch.setenv("XPG_DIAGNOSTICS", "1")
    monkeypatch.setenv("XPG_MC_SPIN", "20000")
    monkeypatch.setenv("XPG_MC_FAULT", "3")
    with pytest.raises(_lib.FitExchangeError):
        e.wlm_fit(*args)
    monkeypatch.delenv("XPG_MC_FAULT")
    w, _, _, _, _ = e.wlm_fit(*args)
    ref, _, _ = oracle.train_wlm(m, B, y, k, w0, params)
    np.testing.assert_allclose(w.cpu().numpy(), ref, rtol=0, atol=1e-4)


@pytest.mark.parametrize("F,S", [(5, 200), (11, 700)])
@pytest.mark.parametrize("wlm_path", ["single", "mc"])
def test_wlm_fit_batched_independent_fits(wlm_path, F, S, monkeypatch):
    """n_fits independent surrogates in one launch == separate fits (F = 11 spans two groups of
    the multi-workgroup fit's XCD-local block mapping)."""
    monkeypatch.setenv("XPG_WLM", wlm_path)
    e = _eng()
    rng = np.random.default_rng(5)
    R, B = 1002, 20
    m = rng.random((F, R, S)) < 0.5
    y = rng.random((F, R)).astype(np.float32)
    k = np.stack([oracle.shap_kernel(m[f]) for f in range(F)])
    w0 = ((rng.random((F, S)) - 0.5) * 0.1).astype(np.float32)
    params = {"lr": 0.01, "l1_lambda": 1e-4}
    bits = torch.stack([e.pack_masks(torch.as_tensor(m[f]).to(DEV)) for f in range(F)])
    w, losses, best, _, _ = e.wlm_fit(bits, S, B, torch.as_tensor(y), torch.as_tensor(k),
                                      torch.as_tensor(w0), params)
    for f in range(F):
        ref, rl, rb = oracle.train_wlm(m[f], B, y[f], k[f], w0[f], params)
        np.testing.assert_allclose(w[f].cpu().numpy(), ref, rtol=0, atol=1e-4)
        np.testing.assert_allclose(losses[f].cpu().numpy(), rl, rtol=1e-5)
        assert int(best[f]) == rb


@pytest.mark.parametrize("wlm_path", ["single", "mc", "grid", "grid3"])
def test_wlm_fit_continuation_equals_one_fit(wlm_path, monkeypatch):
    """A fresh fit (xpg_wlm_fit_from: w = w0, zero moments written by the fit's prologue) over
    rows [0, R) gives bitwise the weights of the fit split in two calls: xpg_wlm_fit_from over
    the first half of the batches, then xpg_wlm_fit continuing from its (w, m, v) with
    step0 = the steps taken (Adam bias corrections keyed by the global step)."""
    monkeypatch.setenv("XPG_WLM", wlm_path)
    e = _eng()
    rng = np.random.default_rng(17)
    R, S, B = 1200, 640, 24
    m = rng.random((R, S)) < 0.5
    y = torch.as_tensor(rng.random(R).astype(np.float32))
    k = torch.as_tensor(oracle.shap_kernel(m))
    w0 = torch.as_tensor(((rng.random(S) - 0.5) * 0.1).astype(np.float32))
    params = {"lr": 0.01, "l1_lambda": 1e-4}
    bits = e.pack_masks(torch.as_tensor(m).to(DEV))
    w_all, _, _, _, _ = e.wlm_fit(bits, S, B, y, k, w0, params)
    h = R // 2  # 25 whole batches
    w1, _, _, m1, v1 = e.wlm_fit(bits[:h], S, B, y[:h], k[:h], w0, params)
    w2, _, _, _, _ = e.wlm_fit(bits[h:], S, B, y[h:], k[h:], w1, params, m0=m1, v0=v1,
                               step0=h // B)
    assert torch.equal(w2, w_all)


# ------------------------------------------------------------------ end to end
@pytest.mark.parametrize("name", CASES)
def test_explainer_run_matches_reference_dataframes(name):
    """Explainer.run on the MI355X vs the reference's own DataFrames (same RNG state)."""
    from case_builders import build_explainer
    exp, z, meta = build_explainer(name)
    torch.set_rng_state(torch.as_tensor(z["rng_state"]))
    df, pdf = exp.run(meta["element"], meta["times"])
    assert exp.last_run["engine"]
    ref = meta["df"]
    got = df.reindex(ref["index"])
    np.testing.assert_allclose(got["config_value_mean"].values, ref["config_value_mean"],
                               atol=1e-4, rtol=0)
    np.testing.assert_allclose(got["config_value_std"].values, ref["config_value_std"],
                               atol=1e-4, rtol=0)
    assert df.columns.tolist() == ["config_value_mean", "config_value_std"]
    vals = df["config_value_mean"].values
    assert np.all(vals[:-1] >= vals[1:])
    if meta["pathway_df"] is None:
        assert pdf is None
    else:
        pref = meta["pathway_df"]
        assert sorted(pdf.index.tolist()) == sorted(pref["index"])
        np.testing.assert_allclose(pdf.reindex(pref["index"])["score"].values, pref["score"],
                                   atol=1e-4, rtol=0)


def test_train_model_seam_matches_reference():
    """wlm.train_model(...) with the reference signature on the golden test_run_t1 batches."""
    from torch.utils.data import DataLoader
    from bikg_graph_explainability_public_amd.wlm import LinearRegression, train_model
    from case_builders import build_explainer
    exp, z, meta = build_explainer("test_run_t1")
    exp.arch = exp.arch.to(DEV)
    ctx = exp.prepare(meta["element"], DEV)
    m = torch.as_tensor(repeat_masks(z, meta)[0]).to(DEV)
    lm = LinearRegression(ctx["S"]).to(DEV)
    with torch.no_grad():
        lm.layer.weight.copy_(torch.as_tensor(z["r0_w0"]).view(1, -1))
    w, losses, best = train_model(DataLoader(m, batch_size=meta["r0_batch_size"]), meta["params"],
                                  ctx["sub_feat"], ctx["sub_ei"], lm, exp.arch, "node",
                                  ctx["sub_ind"])
    np.testing.assert_allclose(w[0].detach().cpu().numpy(), z["r0_w_final"], atol=1e-4)
    assert len(losses) == len(z["r0_losses"]) and best == meta["r0_best_epoch"]


def test_device_sampler_run_is_sane():
    from case_builders import build_explainer
    exp, z, meta = build_explainer("gcn2_medium", {"mask_sampler": "device"})
    df, pdf = exp.run(meta["element"], 2)
    assert pdf is None and not np.isnan(df.values).any() and len(df) == len(meta["df"]["index"])


@pytest.mark.parametrize("sampler", ["compat", "device"])
def test_run_queries_shares_masks(sampler):
    """Explainer.run_queries (graph_prediction, one mask set for several queries): with the
    same seed, query 0 reproduces `run` (same masks, same initial weights — the extra queries'
    inits are drawn after it; atol 1e-4, the surrogate-weight bar, since the batched fit launch
    splits each fit over fewer workgroups), and each further query gets its own fit."""
    from case_builders import build_explainer
    exp, z, meta = build_explainer("gcn2_graph", {"mask_sampler": sampler})
    el = meta["element"]
    other = next(n for n in exp.names if str(n) != str(el))
    df_ref, pdf_ref = exp.run(el, 1)
    (df0, pdf0), (df1, pdf1) = exp.run_queries([el, other], 1)
    np.testing.assert_allclose(df0.loc[df_ref.index].values, df_ref.values, rtol=0, atol=1e-4)
    assert list(df1.columns) == list(df_ref.columns) and len(df1) == len(df_ref)
    assert not np.isnan(df1.values).any() and not df1.equals(df0)
    if pdf_ref is not None:
        np.testing.assert_allclose(pdf0.loc[pdf_ref.index].values, pdf_ref.values, atol=1e-4)
    [(dfs, _)] = exp.run_queries([el], 1)
    np.testing.assert_allclose(dfs.loc[df_ref.index].values, df_ref.values, rtol=0, atol=1e-4)


def test_device_community_sampler_run():
    """Explainer.run with communities on the device sampler: the reference's DataFrame schema,
    finite scores, every community scored (explainer.py:490-532, pathways.py:387-429)."""
    from case_builders import build_explainer
    exp, z, meta = build_explainer("test_run", {"mask_sampler": "device"})
    df, pdf = exp.run(meta["element"], 3)
    assert list(df.columns) == ["config_value_mean", "config_value_std"]
    assert not np.isnan(df.values).any() and len(df) == len(meta["df"]["index"])
    assert pdf is not None and list(pdf.columns) == ["score"] and len(pdf) > 0
    assert (np.diff(pdf["score"].values) <= 0).all()


# ------------------------------------------------------------------ full-size properties
def test_c2_scale_forward_properties(fwd_path):
    """configs[1] scale (100k nodes / 1M edges, F=64, 2-layer GCN, 12,800 rows): engine vs the
    oracle on a row subset, plus row-order equivariance and all-on / all-off invariants."""
    from bikg_graph_explainability_public_amd import pipeline
    from bikg_graph_explainability_public_amd.data import Data
    from bikg_graph_explainability_public_amd.nn import ConvStack
    e = _eng()
    g = torch.Generator().manual_seed(0)
    N, E, F = 100_000, 1_000_000, 64
    feat = torch.randn((N, F), generator=g)
    ei = torch.randint(0, N, (2, E), generator=g)
    torch.manual_seed(0)
    arch = ConvStack("gcn", [64, 64, 64], [64, 1]).eval()
    sub_feat, sub_ei, _, sub_ind, _, _ = Data(feat.to(DEV), ei.to(DEV)).comp_graph(
        7, 2, "node", [str(i) for i in range(N)])
    q = int(sub_ind[0])
    S = sub_feat.shape[0]
    plan = pipeline.build_plan(arch.to(DEV), sub_feat, sub_ei, [q])
    R = 12_800
    bits = e.sample_shapley(123, R, S, DEV)
    y = plan.forward(bits)[:, 0]
    m = e.unpack_masks(bits, S).cpu().numpy()
    spec = {"convs": [{"kind": "gcn", "rels": [None], "act": "relu",
                       "params": {None: {"W": arch.conv[2 * i].lin.weight.detach().cpu().numpy(),
                                         "b": arch.conv[2 * i].bias.detach().cpu().numpy()}}}
                      for i in range(2)],
            "fc": [{"W": arch.fc[0].weight.detach().cpu().numpy(),
                    "b": arch.fc[0].bias.detach().cpu().numpy(), "act": "sigmoid"}]}
    sel = np.arange(0, R, 200)
    ref = oracle.masked_query_outputs(spec, sub_feat.cpu().numpy(), {None: sub_ei.cpu().numpy()},
                                      m[sel], q)
    np.testing.assert_allclose(y.cpu().numpy()[sel], ref, atol=1e-5, rtol=0)
    perm = torch.randperm(R, generator=g).to(DEV)
    y2 = plan.forward(bits[perm].contiguous())[:, 0]
    torch.testing.assert_close(y2, y[perm], rtol=0, atol=0)
    on = e.pack_masks(torch.ones((2, S), dtype=torch.bool, device=DEV))
    off = e.pack_masks(torch.zeros((2, S), dtype=torch.bool, device=DEV))
    y_on = plan.forward(on)[:, 0].cpu().numpy()
    y_off = plan.forward(off)[:, 0].cpu().numpy()
    ref_on = oracle.masked_query_outputs(spec, sub_feat.cpu().numpy(),
                                         {None: sub_ei.cpu().numpy()}, np.ones((1, S), bool), q)
    ref_off = oracle.masked_query_outputs(spec, sub_feat.cpu().numpy(),
                                          {None: sub_ei.cpu().numpy()}, np.zeros((1, S), bool), q)
    np.testing.assert_allclose(y_on, ref_on[0], atol=1e-5)
    np.testing.assert_allclose(y_off, ref_off[0], atol=1e-5)
    k = e.shap_kernel(bits, S)
    assert torch.isfinite(k).all() and (k >= 0).all()
    if fwd_path != "unfused":  # the fused paths agree with the multi-kernel path on every row
        import os
        os.environ["XPG_FORWARD"] = "unfused"
        try:
            y3 = plan.forward(bits)[:, 0]
        finally:
            os.environ["XPG_FORWARD"] = fwd_path.split("-")[0]
        torch.testing.assert_close(y3, y, rtol=0, atol=2e-6)


# ------------------------------------------------------------------ k-hop subgraph (§8f1)
def _khop_check(ei, n, seed, hops):
    e = _eng()
    subset, sub_ei, inv, emask = e.khop_subgraph(seed, hops, torch.as_tensor(ei).to(DEV), n)
    o_subset, o_sub_ei, o_inv, o_emask = oracle.k_hop_subgraph(seed, hops, ei, n)
    np.testing.assert_array_equal(subset.cpu().numpy(), o_subset)
    np.testing.assert_array_equal(sub_ei.cpu().numpy().reshape(2, -1), o_sub_ei.reshape(2, -1))
    assert int(inv[0]) == o_inv
    np.testing.assert_array_equal(emask.cpu().numpy(), o_emask)


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("hops", [0, 1, 2, 3, 4])
def test_khop_vs_oracle_golden_graphs(name, hops):
    """The reference graphs of the golden cases (their comp_graph is what pins the oracle's
    subset size: the mask width S of every recorded mask)."""
    from test_oracle_golden import homogenize
    from golden_utils import case_inputs
    z, meta = load_case(name)
    x, ei, _, _ = homogenize(*case_inputs(z))
    for seed in sorted({0, x.shape[0] // 2, x.shape[0] - 1}):
        _khop_check(np.asarray(ei, dtype=np.int64), x.shape[0], seed, hops)


@pytest.mark.parametrize("N,E,hops", [(1, 0, 3), (5, 0, 2), (50, 400, 3), (4097, 9000, 2),
                                      (20000, 8191, 4), (100000, 1000000, 3)])
def test_khop_vs_oracle_random(N, E, hops):
    """Random graphs with self-loops and duplicate edges; block-boundary sizes (4096 items per
    block); isolated seeds; empty edge sets."""
    g = np.random.default_rng(N * 7 + E)
    ei = g.integers(0, N, size=(2, E), dtype=np.int64)
    if E:
        d = E // 50
        ei[:, :d] = ei[0, :d]                        # self-loops
        ei[:, d:2 * d] = ei[:, :d]                   # duplicates
    for seed in sorted({0, N // 3, N - 1}):
        _khop_check(ei, N, seed, hops)


def test_khop_full_size_properties():
    """c3 graph size (1M nodes, 10M edges): subset sorted unique and contains the seed; every
    kept edge lies inside the subset and every edge inside it is kept; relabel is a bijection."""
    e = _eng()
    N, E, seed = 1_000_000, 10_000_000, 7
    gen = torch.Generator(device=DEV).manual_seed(3)
    ei = torch.randint(0, N, (2, E), device=DEV, generator=gen)
    subset, sub_ei, inv, emask = e.khop_subgraph(seed, 3, ei, N)
    assert bool((subset[1:] > subset[:-1]).all()) and int(subset[inv[0]]) == seed
    inset = torch.zeros(N, dtype=torch.bool, device=DEV)
    inset[subset] = True
    assert torch.equal(emask, inset[ei[0]] & inset[ei[1]])
    assert torch.equal(subset[sub_ei], ei[:, emask])
    o = oracle.k_hop_subgraph(seed, 3, ei.cpu().numpy(), N)
    np.testing.assert_array_equal(subset.cpu().numpy(), o[0])


def test_khop_rejects_bad_ids():
    e = _eng()
    ei = torch.tensor([[0, 1, 9], [1, 2, 0]], device=DEV)
    with pytest.raises(IndexError):
        e.khop_subgraph(0, 2, ei, 3)
    with pytest.raises(IndexError):
        e.khop_subgraph(5, 2, ei[:, :2], 3)


def test_comp_graph_device_matches_host():
    """Data.comp_graph on a device graph (HIP k-hop) equals the host-tensor path."""
    from bikg_graph_explainability_public_amd.data import Data
    g = torch.Generator().manual_seed(11)
    feat = torch.randn(300, 8, generator=g)
    ei = torch.randint(0, 300, (2, 1500), generator=g)
    names = [str(i) for i in range(300)]
    for q in (0, 17, 299):
        a = Data(feat, ei).comp_graph(q, 2, "node_prediction", names)
        b = Data(feat.to(DEV), ei.to(DEV)).comp_graph(q, 2, "node_prediction", names)
        assert torch.equal(a[0], b[0].cpu()) and torch.equal(a[1], b[1].cpu())
        assert a[2] == b[2] and int(a[3]) == int(b[3])


# ------------------------------------------------------------------ multi-node-type hetero (§8a6/f2)
def _mt_plan(c, arch):
    from bikg_graph_explainability_public_amd import pipeline
    x = torch.as_tensor(c["x"], dtype=torch.float32, device=DEV)
    ei = torch.as_tensor(c["ei"], device=DEV)
    nt = torch.as_tensor(c["nt"], device=DEV)
    et = torch.as_tensor(c["et"], device=DEV)
    plan = pipeline.build_plan(arch, x, ei, [c["sub_ind"]], nt, et, c["ntypes"], c["rels"],
                               c["pads"])
    return plan, ei


def _mt_check(c, arch, masks, atol=1e-5):
    from bikg_graph_explainability_public_amd import pipeline
    e = _eng()
    plan, ei = _mt_plan(c, arch)
    assert plan is not None and plan.multi_type
    S = c["x"].shape[0]
    for m in masks:
        bits = e.pack_masks(torch.as_tensor(m, device=DEV))
        y = plan.forward(bits)[:, 0]
        y = torch.where(pipeline.empty_copy_rows(bits, S, ei), torch.zeros_like(y), y)
        ref = oracle.hetero_multi_copy_outputs(c["spec"], c["x"], c["nt"], c["ei"], c["et"],
                                               c["ntypes"], c["rels"], c["pads"], m,
                                               c["sub_ind"])
        np.testing.assert_allclose(y.cpu().numpy(), ref, rtol=0, atol=atol)


def test_multi_type_engine_vs_oracle_golden():
    """Node-type-gated HIP forward (unfused path) vs the oracle's per-copy restatement of
    Model.predict_hetero_output on the reference-recorded masks of tests/golden/hetero_multi."""
    from case_builders import build_arch
    from golden_utils import hetero_multi_setup
    z, meta = load_case("hetero_multi")
    c = hetero_multi_setup(z, meta)
    _mt_check(c, build_arch(meta, z).to(DEV), repeat_masks(z, meta))


@pytest.mark.parametrize("hidden,layers", [(64, 2), (32, 3), (128, 1)])
def test_multi_type_engine_vs_oracle_random(hidden, layers):
    """Three node types of different widths, five relations (three bipartite), all-off /
    all-on / sparse rows."""
    from bikg_graph_explainability_public_amd.nn import HeteroSageStack
    from golden_utils import multi_type_setup
    rels = [("A", "ab", "B"), ("B", "ba", "A"), ("A", "aa", "A"), ("C", "ca", "A"),
            ("A", "ac", "C")]
    sizes, dims = {"A": 300, "B": 200, "C": 150}, {"A": 24, "B": 16, "C": 40}
    g = torch.Generator().manual_seed(hidden + layers)
    feat = {t: torch.randn(n, dims[t], generator=g).numpy() for t, n in sizes.items()}
    ei = {r: torch.stack([torch.randint(0, sizes[r[0]], (m,), generator=g),
                          torch.randint(0, sizes[r[-1]], (m,), generator=g)]).numpy()
          for r, m in zip(rels, (900, 700, 800, 400, 400))}
    torch.manual_seed(3)
    arch = HeteroSageStack(rels, dims, hidden, layers, [hidden, 16, 1]).eval()
    names = {t: [f"{t.lower()}{i}" for i in range(n)] for t, n in sizes.items()}
    c = multi_type_setup(feat, ei, names, "b7", "B", layers,
                         {k: v.numpy() for k, v in arch.state_dict().items()}, [hidden, 16, 1])
    S = c["x"].shape[0]
    gm = np.random.default_rng(layers)
    m = gm.random((96, S)) < 0.5
    m[0] = False
    m[1] = True
    m[2] = gm.random(S) < 0.05
    _mt_check(c, arch.to(DEV), [m])


@pytest.mark.parametrize("hidden", [32, 64])
def test_layer1_rows_kernel_and_term_dropping_bitwise(hidden, monkeypatch):
    """The multi-kernel path's layer-1 aggregation with lanes = mask rows (k_agg_l1_rows, the
    default at widths 32 / 64) against the generic k_agg<true> (XPG_AGG_GENERIC=1), bitwise, on a
    multi-type MEAN + ROOT plan (whose reduced in-degree table makes MEAN sources test their own
    mask bit) and on a homogeneous GCN plan; and the ForwardPlan lowering that drops the other
    destination types' relation terms from a single-type layer (the query layer here) against
    the all-terms plan (engine.PLAN_DROP_OTHER_TYPES = False): fewer terms, the same outputs."""
    from bikg_graph_explainability_public_amd import pipeline
    from bikg_graph_explainability_public_amd.nn import ConvStack, HeteroSageStack
    from golden_utils import multi_type_setup
    e = _eng()
    monkeypatch.setenv("XPG_FORWARD", "unfused")
    monkeypatch.setenv("XPG_FORWARD_STRICT", "1")
    rels = [("A", "ab", "B"), ("B", "ba", "A"), ("A", "aa", "A"), ("C", "ca", "A"),
            ("A", "ac", "C")]
    sizes, dims = {"A": 300, "B": 200, "C": 150}, {"A": 24, "B": 16, "C": 40}
    g = torch.Generator().manual_seed(hidden)
    feat = {t: torch.randn(n, dims[t], generator=g).numpy() for t, n in sizes.items()}
    ei = {r: torch.stack([torch.randint(0, sizes[r[0]], (m,), generator=g),
                          torch.randint(0, sizes[r[-1]], (m,), generator=g)]).numpy()
          for r, m in zip(rels, (900, 700, 800, 400, 400))}
    torch.manual_seed(5)
    arch = HeteroSageStack(rels, dims, hidden, 2, [hidden, 1]).eval()
    names = {t: [f"{t.lower()}{i}" for i in range(n)] for t, n in sizes.items()}
    c = multi_type_setup(feat, ei, names, "b7", "B", 2,
                         {k: v.numpy() for k, v in arch.state_dict().items()}, [hidden, 1])
    S = c["x"].shape[0]
    gm = np.random.default_rng(hidden)
    m = gm.random((160, S)) < gm.uniform(0.2, 0.9, (160, 1))
    m[0], m[1] = False, True
    bits = e.pack_masks(torch.as_tensor(m, device=DEV))
    plan, _ = _mt_plan(c, arch.to(DEV))
    monkeypatch.setenv("XPG_DIAGNOSTICS", "1")
    monkeypatch.delenv("XPG_AGG_GENERIC", raising=False)
    y_rows = plan.forward(bits)
    monkeypatch.setenv("XPG_AGG_GENERIC", "1")
    y_gen = plan.forward(bits)
    monkeypatch.delenv("XPG_AGG_GENERIC")
    assert torch.equal(y_rows, y_gen)
    monkeypatch.setattr(e, "PLAN_DROP_OTHER_TYPES", False)
    plan_all, _ = _mt_plan(c, arch)
    monkeypatch.setattr(e, "PLAN_DROP_OTHER_TYPES", True)
    assert plan.terms_kept[-1] < plan_all.terms_kept[-1]
    np.testing.assert_allclose(plan_all.forward(bits).cpu().numpy(), y_rows.cpu().numpy(),
                               rtol=0, atol=1e-6)
    # homogeneous GCN (GCN terms: the kept in-degree of every source)
    n = 400
    x = torch.randn((n, 16), generator=g)
    eih = torch.randint(0, n, (2, 2400), generator=g)
    torch.manual_seed(6)
    gcn = ConvStack("gcn", [16, hidden, hidden], [hidden, 1]).eval().to(DEV)
    hp = pipeline.build_plan(gcn, x.to(DEV), eih.to(DEV), [9])
    mh = gm.random((130, hp.cols)) < 0.6
    bh = e.pack_masks(torch.as_tensor(mh, device=DEV))
    monkeypatch.delenv("XPG_AGG_GENERIC", raising=False)
    yh_rows = hp.forward(bh)
    monkeypatch.setenv("XPG_AGG_GENERIC", "1")
    yh_gen = hp.forward(bh)
    assert torch.equal(yh_rows, yh_gen)


@pytest.mark.parametrize("case,path", [("hetero_multi", "engine"), ("hetero_multi", "generic"),
                                       ("hetero_gat", "generic"), ("hetero_gat", "loop")])
def test_multi_type_explainer_run_matches_reference(case, path, monkeypatch):
    """Explainer.run on the multi-node-type golden cases (quirk Q4 reproduced) vs the
    reference's DataFrames: the HIP engine and the batched generic path (HeteroConv of SAGE);
    the reference's own multi-type conv, GATConv (the engine does not compile it: it runs on
    the batched generic path, and on the reference's per-copy loop for comparison)."""
    import warnings
    from bikg_graph_explainability_public_amd import pipeline
    from case_builders import build_explainer
    if path == "generic" and case == "hetero_multi":
        monkeypatch.setattr(pipeline, "build_plan", lambda *a, **k: None)
    if path == "loop":
        monkeypatch.setattr(pipeline, "HETERO_BATCHED", False)
    exp, z, meta = build_explainer(case)
    warnings.simplefilter("ignore")
    torch.set_rng_state(torch.as_tensor(z["rng_state"]))
    df, _ = exp.run(meta["element"], meta["times"])
    assert exp.last_run["engine"] == (path == "engine")
    for i in range(meta["times"]):
        np.testing.assert_allclose(exp.last_run["repeats"][i]["y"].cpu().numpy().reshape(-1, meta[
            f"r{i}_batch_size"])[:, 0], z[f"r{i}_output"], rtol=0, atol=1e-5)
    ref = meta["df"]
    got = df.reindex(ref["index"])
    np.testing.assert_allclose(got["config_value_mean"].values, ref["config_value_mean"],
                               atol=1e-4, rtol=0)
    np.testing.assert_allclose(got["config_value_std"].values, ref["config_value_std"],
                               atol=1e-4, rtol=0)
