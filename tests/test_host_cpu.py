"""CPU tests of the host side: compat mask sampler vs the reference's masks (golden vectors),
architecture compilation, receptive-field plan arrays, the native library's exports."""
import os
import re

import numpy as np
import pytest
import torch

import oracle
from bikg_graph_explainability_public_amd import _lib
from bikg_graph_explainability_public_amd.engine import plan_arrays
from bikg_graph_explainability_public_amd.explainer import set_seed
from bikg_graph_explainability_public_amd.masks import Mask, dataloader_seed_draw
from bikg_graph_explainability_public_amd.pathways import Pathways
from bikg_graph_explainability_public_amd.program import UnsupportedArch, compile_arch
from bikg_graph_explainability_public_amd.wlm import LinearRegression
from case_builders import build_arch, build_explainer
from golden_utils import CASES, load_case, repeat_masks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("name", CASES)
def test_compat_sampler_reproduces_reference_masks(name):
    """masks.py:262-397 restated with the same torch CPU RNG call order: identical masks, and
    the surrogate's initial weights (LinearRegression init) follow in the same stream."""
    exp, z, meta = build_explainer(name)
    torch.set_rng_state(torch.as_tensor(z["rng_state"]))
    if meta["times"] == 1:
        set_seed(meta["params"]["seed"])
    ctx = exp.prepare(meta["element"], torch.device("cpu"))
    gold = repeat_masks(z, meta)
    for i in range(meta["n_repeats"]):
        mask, rows = Mask(ctx["sub_feat"], ctx["sub_ei"], ctx["sub_pw_inds"], exp.params,
                          exp.problem).generate()
        assert mask.shape == gold[i].shape
        assert np.array_equal(mask.numpy(), gold[i]), f"repeat {i} mask differs"
        if f"r{i}_pathway_rows" in z.files:
            assert np.array_equal(rows.numpy(), z[f"r{i}_pathway_rows"])
        w0 = LinearRegression(ctx["S"]).layer.weight.detach().numpy().reshape(-1)
        assert np.array_equal(w0, z[f"r{i}_w0"])
        dataloader_seed_draw()
        assert mask.shape[0] // meta["params"]["epochs"] == meta[f"r{i}_batch_size"]


@pytest.mark.parametrize("name", CASES)
def test_compat_bits_sampler_reproduces_reference_masks(name):
    """Mask.generate_bits (the Shapley draw replayed from torch's MT19937 state by the native
    host generator, xpg_mt19937_mask_bits; community masks through generate) gives the
    reference's masks bit-packed, and leaves torch's generator where the reference leaves it
    (the initial weights drawn next still match)."""
    exp, z, meta = build_explainer(name)
    torch.set_rng_state(torch.as_tensor(z["rng_state"]))
    if meta["times"] == 1:
        set_seed(meta["params"]["seed"])
    ctx = exp.prepare(meta["element"], torch.device("cpu"))
    gold = repeat_masks(z, meta)
    for i in range(meta["n_repeats"]):
        bits, _ = Mask(ctx["sub_feat"], ctx["sub_ei"], ctx["sub_pw_inds"], exp.params,
                       exp.problem).generate_bits("cpu")
        np.testing.assert_array_equal(bits.numpy().view(np.uint32), oracle.pack_bits(gold[i]))
        w0 = LinearRegression(ctx["S"]).layer.weight.detach().numpy().reshape(-1)
        assert np.array_equal(w0, z[f"r{i}_w0"])
        dataloader_seed_draw()


@pytest.mark.parametrize("rows,cols,pre", [(12800, 1193, 0), (7, 33, 5), (1, 1, 0), (3, 64, 623),
                                           (100, 1001, 1), (41, 31, 624), (5, 2000, 1250)])
def test_native_mt19937_matches_torch_randint(rows, cols, pre):
    """engine.compat_shapley_bits == torch.randint(0, 2, (rows, cols), dtype=torch.bool) packed,
    from any generator position (pre draws: fresh state, block boundaries, mid-block), and the
    generator state afterwards equals torch's (the next draws agree)."""
    from bikg_graph_explainability_public_amd import engine
    torch.manual_seed(rows * 7 + cols)
    torch.randint(0, 2, (pre,), dtype=torch.bool)
    bits = engine.compat_shapley_bits(rows, cols)
    after = torch.randint(0, 2 ** 31, (5,))
    torch.manual_seed(rows * 7 + cols)
    torch.randint(0, 2, (pre,), dtype=torch.bool)
    m = torch.randint(0, 2, (rows, cols), dtype=torch.bool)
    np.testing.assert_array_equal(bits.numpy().view(np.uint32), oracle.pack_bits(m.numpy()))
    assert torch.equal(after, torch.randint(0, 2 ** 31, (5,)))


def test_extract_index_follows_in_place_name_edits():
    """Explainer.extract_index caches a name -> position index per names list; a list edited in
    place at the same length must not answer from the stale index."""
    from bikg_graph_explainability_public_amd.explainer import Explainer
    names = [f"n{i}" for i in range(50)]
    assert Explainer.extract_index("n7", names) == 7
    names[7], names[30] = "moved", "n7"          # same length, n7 now at 30
    assert Explainer.extract_index("n7", names) == 30
    names[3] = "fresh"
    assert Explainer.extract_index("fresh", names) == 3
    with pytest.raises(AssertionError):
        Explainer.extract_index("n3", names)
    assert Explainer.extract_index(12, None) == 12
    # membership is the names' own (explainer.py:222 `element in names`): '5' is no member of
    # integer names, even though numpy's str form of 5 is '5' 
    ints = list(range(10))
    with pytest.raises(AssertionError):
        Explainer.extract_index("5", ints)


@pytest.mark.parametrize("name", CASES)
def test_prepare_matches_oracle_subgraph(name):
    exp, z, meta = build_explainer(name)
    ctx = exp.prepare(meta["element"], torch.device("cpu"))
    m = repeat_masks(z, meta)[0]
    assert ctx["S"] == m.shape[1]
    df_names = set(meta["df"]["index"])
    assert set(ctx["sub_names"]) == df_names


def test_mask_structure_invariant():
    """tests/test_mask.py:286-393 + tests/test_utils.py:283-356: in every community-mask row
    at most one community is mixed; the others are all-on or all-off (shared members aside)."""
    feat = torch.randn(9, 4)
    ei = torch.tensor([[0, 2, 3, 6, 4, 5, 7, 8], [5, 6, 4, 1, 2, 0, 2, 5]])
    comms = [[3], [1, 2, 3, 4], [5, 7], [7, 8, 0, 4]]
    params = {"interpret_samples": 20, "epochs": 50}
    torch.manual_seed(0)
    mask, rows = Mask(feat, ei, [list(c) for c in comms], params, "node").generate()
    assert mask.dtype == torch.bool and mask.shape[1] == 9 and mask.shape[0] >= 1000
    for r in range(mask.shape[0]):
        inner = int(rows[r])
        for i, c in enumerate(comms):
            if i == inner:
                continue
            others = set(e for j, cc in enumerate(comms) if j != i for e in cc)
            own = [e for e in c if e not in others]
            if own:
                vals = mask[r, own]
                assert bool(vals.all()) or not bool(vals.any())


def test_pathway_helpers_known_answers():
    comm = [[3], [1, 2, 3, 4], [5, 7], [7, 8, 0, 4]]
    pm = torch.tensor([[0, 0, 0, 0], [0, 0, 0, 1], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 1, 0],
                       [0, 1, 0, 1], [1, 1, 0, 0], [1, 1, 1, 0], [1, 0, 0, 0]], dtype=torch.bool)
    em, rep = Pathways(comm, None).pathway_mask2node_mask(pm)
    ref_em, ref_rep = oracle.pathway_mask2node_mask(comm, pm.numpy())
    assert np.array_equal(em.numpy(), ref_em) and np.array_equal(rep.numpy(), ref_rep)
    cv = torch.tensor([0.21, 0.23, 0.95, 0.65, 0.98, -0.21, 0.32, 0.94, -0.34])
    df = Pathways(comm, ["1", "2", "3", "4"]).aggregate(cv, comm)
    assert df.index.tolist() == ["2", "1", "4", "3"]
    np.testing.assert_allclose(df["score"].values, [0.7025, 0.65, 0.4475, 0.365], atol=1e-6)
    hp = {"1": [[0, 1, 2, 3, 4], [5, 6, 7]], "2": [[0, 1, 2], [3, 4, 5]]}
    res, names, types = Pathways(hp, {"1": ["1", "2"], "2": ["3", "4"]}).hetero2homo("node",
                                                                                      [0, 8])
    assert res == [[0, 1, 2, 3, 4], [5, 6, 7], [8, 9, 10], [11, 12, 13]]
    assert names == ["1", "2", "3", "4"] and types.int().tolist() == [0, 0, 1, 1]
    dead = torch.zeros((9, 4), dtype=torch.bool)
    dead[3, 2] = dead[4, 2] = True
    out = Pathways(comm, None).activate_dead_mask(dead, 2)
    assert out.shape == dead.shape and not torch.equal(out, dead)


def test_sorted_frame_matches_pandas_sort():
    """frames.sorted_frame == the reference's DataFrame / set_index / sort_values (/ dropna)
    chains (data.py:651-693, pathways.py:420-429) on random columns with ties, NaNs, str and int
    names; the aggregate segment cache follows a change of the communities."""
    import pandas as pd
    from bikg_graph_explainability_public_amd.frames import sorted_frame
    rng = np.random.default_rng(1)
    for trial in range(300):
        n = int(rng.integers(1, 200))
        s = rng.integers(0, 5, n).astype(np.float64) if trial % 2 else rng.standard_normal(n)
        s[rng.random(n) < 0.1] = np.nan
        d = rng.standard_normal(n).astype(np.float32)
        d[rng.random(n) < 0.05] = np.nan
        names = [f"c{i}" for i in range(n)] if trial % 3 else list(range(n))
        ref = (pd.DataFrame({"name": names, "score": s.tolist()}).set_index("name")
               .sort_values(by=["score"], ascending=False).dropna())
        got = sorted_frame(names, {"score": s}, "score", dropna=True)
        assert ref.equals(got) and ref.index.tolist() == got.index.tolist()
        assert ref.index.dtype == got.index.dtype and ref.index.name == got.index.name
        s32 = s.astype(np.float32)
        ref = (pd.DataFrame({"name": names, "config_value_mean": s32, "config_value_std": d})
               .set_index("name").sort_values(by=["config_value_mean"], ascending=False))
        got = sorted_frame(names, {"config_value_mean": s32, "config_value_std": d},
                           "config_value_mean")
        assert ref.equals(got) and ref.index.tolist() == got.index.tolist()
        assert list(ref.columns) == list(got.columns) and ref.dtypes.tolist() == got.dtypes.tolist()
    pw = Pathways([[0, 1], [2]], ["a", "b"])
    cv = torch.tensor([1.0, 2.0, 5.0])
    assert pw.aggregate(cv, [[0, 1], [2]])["score"].tolist() == [5.0, 1.5]
    assert pw.aggregate(cv, [[0], [1, 2]])["score"].tolist() == [3.5, 1.0]


@pytest.mark.parametrize("name", ["test_run", "toy", "hetero_single", "sage_shapley",
                                  "gcn2_medium"])
def test_compile_arch(name):
    exp, z, meta = build_explainer(name)
    rels = meta["arch_spec"].get("hetero_rels")
    prog = compile_arch(exp.arch, [tuple(r) for r in rels] if rels else None)
    a = meta["arch_spec"]
    assert len(prog.convs) == len(a["dims"]) - 1
    assert len(prog.head) == len(a["fc"]) - 1
    assert prog.head[-1].act == "sigmoid"
    assert all(c.act == "relu" for c in prog.convs)
    if a["kind"] == "sage":
        assert [t.kind for t in prog.convs[0].terms] == ["mean", "root"]
    if rels:
        assert [t.rel for t in prog.convs[0].terms] == [0, 1, 2]


def test_compile_rejects_unsupported():
    class Odd(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.bn = torch.nn.BatchNorm1d(4)

        def forward(self, x, ei):
            return self.bn(x)

    with pytest.raises(UnsupportedArch):
        compile_arch(Odd())


def test_plan_arrays_receptive_field():
    rng = np.random.default_rng(0)
    S, E = 60, 240
    ei = rng.integers(0, S, size=(2, E))
    ei[:, :5] = [[3, 4, 5, 6, 7], [3, 4, 5, 6, 7]]  # self-loops
    q = 3
    arr = plan_arrays(S, [ei], [q], 2)
    fr = arr["frontiers"]
    assert fr[2].tolist() == [q]
    assert set(fr[1]) == {q} | set(ei[0][ei[1] == q].tolist())
    assert list(fr[1][:1]) == [q] and list(fr[0][:len(fr[1])]) == list(fr[1])
    # degree CSR: in-edges (no self loops) of every F0 node
    for p, v in enumerate(fr[0]):
        got = sorted(arr["deg_src"][arr["deg_ptr"][p]:arr["deg_ptr"][p + 1]].tolist())
        exp = sorted(ei[0][(ei[1] == v) & (ei[0] != v)].tolist())
        assert got == exp
    lay = arr["layers"][0]
    for t, v in enumerate(fr[1]):
        srcs = fr[0][lay["agg_src"][lay["agg_ptr"][t]:lay["agg_ptr"][t + 1]]]
        assert sorted(srcs.tolist()) == sorted(ei[0][(ei[1] == v) & (ei[0] != v)].tolist())
        assert lay["self_mult"][t] == int(((ei[0] == v) & (ei[1] == v)).sum())


def test_native_library_exports_header_symbols():
    """libxpgnn.so loads (no GPU needed) and exports every entry point include/xpgnn.h declares."""
    hdr = open(os.path.join(ROOT, "include", "xpgnn.h")).read()
    declared = set(re.findall(r"^\s*(?:int|const char\*)\s+(xpg_\w+)\s*\(", hdr, re.M))
    assert declared == set(_lib.EXPORTED)
    lib = _lib.load()
    for name in declared:
        assert hasattr(lib, name)
    assert lib.xpg_abi_version() == _lib.ABI_VERSION


def test_engine_refuses_cpu_tensors():
    from bikg_graph_explainability_public_amd import engine
    with pytest.raises(_lib.NativeLibraryError):
        engine.pack_masks(torch.zeros((2, 3), dtype=torch.bool))


def _plan_mask(S, pathways, samples, epochs=2):
    return Mask(torch.zeros((S, 1)), torch.zeros((2, 0), dtype=torch.long), pathways,
                {"interpret_samples": samples, "epochs": epochs}, "node_prediction")


@pytest.mark.parametrize("S, lens, samples", [
    (36, None, 20),                                  # the test_run communities (golden case)
    (300, [40, 7, 2, 1, 25, 60, 3], 100),            # tiny communities: size_internal < 3
    (5000, [900, 700, 40, 30, 20, 10, 5], 30),       # S > 4000: truncated to the total rows
])
def test_community_plan_matches_compat_blocks(S, lens, samples):
    """Mask.community_plan (the device sampler's host plan) has the compat sampler's block
    sizes, community order and row count (masks.py:309-380)."""
    if lens is None:
        exp, z, meta = build_explainer("test_run")
        ctx = exp.prepare(meta["element"], torch.device("cpu"))
        pathways, S = ctx["sub_pw_inds"], ctx["S"]
        samples = exp.params["interpret_samples"]
    else:
        rng = np.random.default_rng(S)
        perm = rng.permutation(S)
        pathways, o = [], 0
        for n in lens:
            pathways.append(sorted(perm[o:o + n].tolist()))
            o += n
    torch.manual_seed(0)
    mask, prow = _plan_mask(S, [list(p) for p in pathways], samples).generate()
    blocks, src_rows, out_rows, shuffle = _plan_mask(S, [list(p) for p in pathways],
                                                     samples).community_plan()
    b = blocks.numpy()
    assert out_rows == mask.shape[0] and (b[:, 0] == np.concatenate([[0], np.cumsum(b[:-1, 1])])).all()
    assert src_rows == int(b[:, 1].sum()) and shuffle == (S <= 4000 or src_rows <= samples * 2)
    assert (b[:, 2] <= b[:, 1]).all() and sorted(b[:, 4].tolist()) == list(range(len(b)))
    counts = np.bincount(prow.numpy(), minlength=len(pathways))
    if shuffle:
        assert np.array_equal(counts[b[:, 3]], b[:, 1])
    else:  # truncation keeps the largest communities' rows first
        assert counts.sum() == out_rows and set(np.flatnonzero(counts)) <= set(b[:, 3].tolist())


def _random_communities(S, lens, seed, overlap=False):
    rng = np.random.default_rng(seed)
    if overlap:  # members drawn independently: communities share columns
        return [sorted(rng.choice(S, n, replace=False).tolist()) for n in lens]
    perm = rng.permutation(S)
    out, o = [], 0
    for n in lens:
        out.append(rng.permutation(perm[o:o + n]).tolist())  # unsorted: the sampler sorts
        o += n
    return out


@pytest.mark.parametrize("S, lens, samples, overlap, pre", [
    (1193, [60] * 19 + [53], 256, False, 0),          # the communities_c2 shape (c2 subgraph)
    (300, [40, 7, 2, 1, 25, 60, 3], 100, False, 5),   # tiny communities: size_internal < 3
    (64, [3, 2], 7, False, 623),                      # two communities: dead-mask randperm rows
    (50, [1, 1, 1, 1], 3, True, 624),                 # single members, shared columns
    (40, [40], 20, False, 1250),                      # one community (no external coalition)
    (120, [30, 50, 10, 70], 33, True, 17),            # overlapping communities
    (5000, [900, 700, 40, 30, 20, 10, 5], 30, False, 3),  # S > 4000: truncation branch
])
def test_native_community_draw_matches_torch(S, lens, samples, overlap, pre):
    """The compat community sampler's native replay (Mask._community_bits ->
    xpg_mt19937_community_bits, host code) equals the reference's torch call sequence
    (Mask._generate_torch, itself pinned by the golden masks) bit for bit: same rows, same
    pathway_rows, the caller's lists sorted the same way, and torch's generator left at the
    same position, from several generator positions (fresh, mid-block, block boundaries)."""
    from bikg_graph_explainability_public_amd.masks import _unpack_host
    comms = _random_communities(S, lens, S + len(lens), overlap)
    ref_lists, nat_lists = [list(c) for c in comms], [list(c) for c in comms]
    torch.manual_seed(S * 3 + samples)
    torch.randint(0, 2 ** 31, (pre,))
    ref_mask, ref_prow = _plan_mask(S, ref_lists, samples)._generate_torch()
    ref_after = torch.randint(0, 2 ** 31, (6,))
    torch.manual_seed(S * 3 + samples)
    torch.randint(0, 2 ** 31, (pre,))
    bits, prow = _plan_mask(S, nat_lists, samples)._community_bits()
    assert torch.equal(torch.randint(0, 2 ** 31, (6,)), ref_after)
    assert torch.equal(_unpack_host(bits, S), ref_mask)
    np.testing.assert_array_equal(bits.numpy().view(np.uint32), oracle.pack_bits(ref_mask.numpy()))
    assert torch.equal(prow, ref_prow)
    assert nat_lists == ref_lists


def test_native_community_dead_mask_sweep(monkeypatch):
    """Blocks whose external coalitions come out all-off take activate_dead_mask's randperm
    (pathways.py:285-334; only when a block has at most one external row pair): 120 seeds of a
    tiny 3-community problem, most of which take that branch at least once, replay bit-exactly
    with the generator at the same position afterwards."""
    from bikg_graph_explainability_public_amd.masks import _unpack_host
    calls = []
    orig = Pathways.activate_dead_mask
    monkeypatch.setattr(Pathways, "activate_dead_mask",
                        lambda self, *a: calls.append(1) or orig(self, *a))
    comms = [[0, 1, 2], [3, 4], [5]]
    for seed in range(120):
        torch.manual_seed(seed)
        m, p = _plan_mask(8, [list(c) for c in comms], 1)._generate_torch()
        after = torch.randint(0, 2 ** 31, (3,))
        torch.manual_seed(seed)
        b, q = _plan_mask(8, [list(c) for c in comms], 1)._community_bits()
        assert torch.equal(_unpack_host(b, 8), m) and torch.equal(p, q), seed
        assert torch.equal(torch.randint(0, 2 ** 31, (3,)), after), seed
    assert len(calls) > 50


def test_native_community_generate_bits_golden_cases():
    """Explainer-level compat draws through the native community replay reproduce the
    reference's recorded masks of every golden case with communities (generate_bits)."""
    hit = 0
    for name in CASES:
        exp, z, meta = build_explainer(name)
        if exp.pathways is None:
            continue
        hit += 1
        torch.set_rng_state(torch.as_tensor(z["rng_state"]))
        if meta["times"] == 1:
            set_seed(meta["params"]["seed"])
        ctx = exp.prepare(meta["element"], torch.device("cpu"))
        gold = repeat_masks(z, meta)
        for i in range(meta["n_repeats"]):
            m = Mask(ctx["sub_feat"], ctx["sub_ei"], ctx["sub_pw_inds"], exp.params, exp.problem)
            bits, rows = m.generate_bits("cpu")
            np.testing.assert_array_equal(bits.numpy().view(np.uint32), oracle.pack_bits(gold[i]))
            if f"r{i}_pathway_rows" in z.files:
                assert np.array_equal(rows.numpy(), z[f"r{i}_pathway_rows"])
            w0 = LinearRegression(ctx["S"]).layer.weight.detach().numpy().reshape(-1)
            assert np.array_equal(w0, z[f"r{i}_w0"])
            dataloader_seed_draw()
    assert hit >= 1


def test_community_plan_sizes_equal_internal_sizes():
    """community_plan computes every block's (size, size_internal) in one float32 tensor pass;
    they equal the reference's per-community internal_sizes (masks.py:98-125, a float32 0-d
    tensor fraction per call) over many random community length sets and totals."""
    rng = np.random.default_rng(7)
    for trial in range(200):
        n = int(rng.integers(1, 40))
        lens = rng.integers(1, 3000 if trial % 2 else 30, n).tolist()
        samples = int(rng.integers(1, 600))
        epochs = int(rng.integers(1, 60))
        comms = [list(range(k)) for k in lens]
        blocks, _, _, _ = _plan_mask(max(lens) + 1, comms, samples, epochs).community_plan()
        lt = torch.tensor(lens)
        for row in blocks.tolist():
            assert (row[1], row[2]) == Mask.internal_sizes(lens[row[3]], lt, samples * epochs)


def test_community_columns_csr():
    from bikg_graph_explainability_public_amd.engine import community_columns
    ptr_, comm = community_columns([[0, 3, 4], [4, 5], [1]], 7)
    assert ptr_.tolist() == [0, 1, 2, 2, 3, 5, 6, 6]
    assert comm.tolist() == [0, 2, 0, 0, 1, 1]


def test_capture_guard_holds_the_cyclic_collector():
    """engine.capture_guard (wraps every HIP-graph capture): collects before, keeps Python's
    cyclic GC off during the capture (a graph freed mid-capture aborts the process on this HIP
    stack: tools/capture_probe.py graph_gc), restores it afterwards, also on an exception, and
    leaves a caller's disabled collector disabled."""
    import gc
    from bikg_graph_explainability_public_amd import engine
    assert gc.isenabled()
    with engine.capture_guard():
        assert not gc.isenabled()
    assert gc.isenabled()
    try:
        with engine.capture_guard():
            raise RuntimeError("capture failed")
    except RuntimeError:
        pass
    assert gc.isenabled()
    gc.disable()
    try:
        with engine.capture_guard():
            assert not gc.isenabled()
        assert not gc.isenabled()
    finally:
        gc.enable()


@pytest.mark.parametrize("S", [1, 7, 1193, 100_000])
def test_initial_weights_equal_linear_regression_init(S):
    """LinearRegression.initial_weights (the uniform_ draw with kaiming_uniform_'s bound, no
    module) gives nn.Linear(S, 1, bias=False)'s weight bit for bit and leaves the CPU generator
    in the same state (wlm.py:17-61 builds the module per repeat)."""
    from bikg_graph_explainability_public_amd.wlm import LinearRegression
    torch.manual_seed(S)
    a = LinearRegression.initial_weights(S)
    sa = torch.get_rng_state()
    torch.manual_seed(S)
    b = torch.nn.Linear(S, 1, bias=False).weight.detach().reshape(-1)
    assert torch.equal(a, b) and torch.equal(sa, torch.get_rng_state())


def test_take_names_matches_numpy_str_indexing():
    """data.take_names == np.array(names, dtype=str)[idx].tolist() (data.py:341-356) for str,
    int and float names, one index and many."""
    from bikg_graph_explainability_public_amd.data import take_names
    names = [str(i) for i in range(50)] + [5, 3.5, "x", "y\x00", np.str_("z")]
    for idx in ([1], [0, 5, 49], np.array([50, 51, 52, 3]), torch.tensor([2, 2, 0]), [53, 1],
                [54, 2]):
        ref = np.array(names, dtype=str)[np.asarray(idx, dtype=np.int64)].tolist()
        assert take_names(names, idx) == ref
    assert take_names(names, []) == []


@pytest.mark.parametrize("seed,n_rel,L,nq,with_eid", [(0, 1, 2, 1, False), (1, 3, 2, 4, True),
                                                      (2, 2, 3, 1, False), (3, 1, 1, 7, True),
                                                      (4, 5, 2, 2, False)])
def test_native_plan_arrays_match_numpy(seed, n_rel, L, nq, with_eid):
    """engine.plan_arrays (the library's host builder, xpg_plan_arrays_build) == the numpy
    restatement plan_arrays_numpy, array for array: frontiers, degree CSR, every layer's CSRs,
    self-loop counts and columns, on random multi-relation graphs with self-loops, duplicate
    edges and isolated nodes."""
    from bikg_graph_explainability_public_amd.engine import plan_arrays_numpy
    rng = np.random.default_rng(seed)
    S = 90
    rels, eids, col = [], [], 0
    for r in range(n_rel):
        E = int(rng.integers(0, 200))
        ei = rng.integers(0, S - 5, size=(2, E))  # the last 5 nodes stay isolated
        if E > 6:
            ei[1, :3] = ei[0, :3]                 # self-loops
            ei[:, 3:6] = ei[:, :1]                # duplicates of a self-loop
        rels.append(ei)
        eids.append(np.arange(col, col + E))
        col += E
    q = rng.choice(S, size=nq, replace=False)
    got = plan_arrays(S, rels, q, L, eids if with_eid else None)
    ref = plan_arrays_numpy(S, rels, q, L, eids if with_eid else None)
    for a, b in zip(got["frontiers"], ref["frontiers"]):
        np.testing.assert_array_equal(a, b)
    for k in ("deg_ptr", "deg_src", "deg_eid"):
        np.testing.assert_array_equal(got[k], ref[k])
    for lg, lr in zip(got["layers"], ref["layers"]):
        for k in lr:
            np.testing.assert_array_equal(lg[k], lr[k], err_msg=k)
    with pytest.raises(ValueError):
        plan_arrays(S, rels, [S], L)
    with pytest.raises(ValueError):
        plan_arrays(S, rels, [1, 1], L)


def _torch_repeat_draws(times, S):
    """Explainer.run's per-repeat torch calls with the device sampler (explainer.py:490-519)."""
    seeds, w0 = [], []
    for _ in range(times):
        seeds.append(int(torch.randint(0, 2 ** 62, (1,)).item()))
        w0.append(LinearRegression.initial_weights(S))
        dataloader_seed_draw()
    return seeds, torch.stack(w0) if times else torch.empty((0, S))


@pytest.mark.parametrize("S", [1, 7, 300, 623, 624, 625, 1193, 5000])
@pytest.mark.parametrize("times", [1, 3, 10])
@pytest.mark.parametrize("skip", [0, 1, 311, 622, 623, 1500])
def test_native_repeat_draws_match_torch(S, times, skip):
    """engine.repeat_draws (xpg_mt19937_repeat_draws, host code) = the sampler seed, the
    LinearRegression init and the DataLoader seed draw of every repeat, bit for bit, from any
    generator position (skip = outputs drawn before; 622-625 cross a state regeneration), and
    the generator left where the torch calls leave it (the next draw matches too)."""
    from bikg_graph_explainability_public_amd import engine
    _lib.load()
    torch.manual_seed(1234 + S)
    if skip:
        torch.empty(skip, dtype=torch.float32).uniform_()  # one 32-bit output each
    start = torch.get_rng_state()
    ref_seeds, ref_w0 = _torch_repeat_draws(times, S)
    ref_next = torch.rand(5)
    torch.set_rng_state(start)
    seeds, w0 = engine.repeat_draws(times, S)
    nxt = torch.rand(5)
    assert seeds == ref_seeds
    assert torch.equal(w0, ref_w0), float((w0 - ref_w0).abs().max())
    assert torch.equal(nxt, ref_next)


def test_native_repeat_draws_fma_form_differs_somewhere():
    """The fused-multiply-add form of uniform_real is a different rounding (so the pinned form
    above is a real choice, not a coincidence of the inputs)."""
    from bikg_graph_explainability_public_amd import engine
    _lib.load()
    torch.manual_seed(5)
    st = torch.get_rng_state()
    _, a = engine.repeat_draws(10, 5000, fma=0)
    torch.set_rng_state(st)
    _, b = engine.repeat_draws(10, 5000, fma=1)
    assert not torch.equal(a, b)


@pytest.mark.parametrize("comms", [
    [[3, 7, 7, 12, 20], [0, 1, 2], [30, 31, 40, 41]],          # a member listed twice
    [[5, 5, 5], [8, 9, 10, 11], [1, 2]],                        # all one column, three times
    [[0, 4, 9, 4, 0, 13], [20, 21, 22, 23, 24], [30], [4, 40]],  # repeats + a shared column
])
@pytest.mark.parametrize("pre", [0, 311, 623])
def test_native_community_draw_duplicate_members(comms, pre):
    """Communities that list a column more than once: the native replay keeps
    torch's sequential last-write semantics of the member assignment (masks.py:338
    `mask[:, pathway] = internal_mask`) bit for bit, and leaves the generator where the torch
    sequence leaves it."""
    from bikg_graph_explainability_public_amd.masks import _unpack_host
    S = 48
    ref_lists, nat_lists = [list(c) for c in comms], [list(c) for c in comms]
    torch.manual_seed(99 + pre)
    torch.randint(0, 2 ** 31, (pre,))
    ref_mask, ref_prow = _plan_mask(S, ref_lists, 12)._generate_torch()
    ref_after = torch.randint(0, 2 ** 31, (6,))
    torch.manual_seed(99 + pre)
    torch.randint(0, 2 ** 31, (pre,))
    bits, prow = _plan_mask(S, nat_lists, 12)._community_bits()
    assert torch.equal(torch.randint(0, 2 ** 31, (6,)), ref_after)
    assert torch.equal(_unpack_host(bits, S), ref_mask)
    assert torch.equal(prow, ref_prow)
    assert nat_lists == ref_lists


def test_community_filtering_drops_empty_communities():
    """An empty community never reaches the sampler: the computational-subgraph filtering
    (Pathways.comp_graph, pathways.py:33-102) keeps only communities with members in the
    subgraph, so the native replay's zero-length case is not reachable through Explainer."""
    pw = Pathways([["0", "1"], ["50", "51"], ["2"]], ["a", "b", "c"])
    subs, names, _ = pw.comp_graph(["0", "1", "2", "3"])
    assert subs == [["0", "1"], ["2"]] and names == ["a", "c"]
    exp, z, meta = build_explainer("test_run")
    ctx = exp.prepare(meta["element"], torch.device("cpu"))
    assert all(len(c) > 0 for c in ctx["sub_pw_inds"])


@pytest.mark.parametrize("level", ["sse2", "avx2", "avx512", "native"])
def test_compat_replay_every_simd_path(level):
    """The native mt19937 replay's SIMD paths (XPG_HOST_SIMD caps the level: SSE2 baseline, AVX2,
    AVX-512, AVX-512 + VPOPCNTDQ where the CPU has them) all give torch's bool draw bit for bit,
    from generator positions across state regenerations, and leave the generator where torch
    does (each level in its own process: the level is read once)."""
    import subprocess
    import sys
    code = r"""
import numpy as np, torch, oracle
from bikg_graph_explainability_public_amd import engine, _lib
_lib.load()
for seed, skip, rows, cols in [(1, 0, 300, 1193), (2, 623, 77, 40), (3, 311, 129, 33), (4, 1, 64, 1024), (5, 5000, 31, 997)]:
    torch.manual_seed(seed)
    torch.empty(skip).uniform_()
    st = torch.get_rng_state()
    ref = torch.randint(0, 2, (rows, cols), dtype=torch.bool); after = torch.rand(4)
    torch.set_rng_state(st)
    b = engine.compat_shapley_bits(rows, cols); after2 = torch.rand(4)
    assert np.array_equal(b.numpy().view(np.uint32), oracle.pack_bits(ref.numpy())), (seed, skip)
    assert torch.equal(after, after2), (seed, skip)
    torch.set_rng_state(st)
    s1, w1 = engine.repeat_draws(3, cols)
    torch.set_rng_state(st)
    s2 = []; w2 = []
    for _ in range(3):
        s2.append(int(torch.randint(0, 2 ** 62, (1,)).item()))
        from bikg_graph_explainability_public_amd.wlm import LinearRegression
        w2.append(LinearRegression.initial_weights(cols))
        torch.empty((), dtype=torch.int64).random_()
    assert s1 == s2 and torch.equal(w1, torch.stack(w2)), (seed, skip)
print("ok")
"""
    env = dict(os.environ)
    if level != "native":
        env["XPG_HOST_SIMD"] = level
    else:
        env.pop("XPG_HOST_SIMD", None)
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0 and "ok" in out.stdout, out.stderr[-3000:]
