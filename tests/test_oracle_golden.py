"""Pin the numpy ORACLE against golden vectors recorded from the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

import oracle
from golden_utils import CASES, case_inputs, load_case, oracle_spec, repeat_masks, state_dict


def homogenize(feat, ei):
    """data.py:95-147,695-822 for a single node type (pointer offsets 0)."""
    if isinstance(feat, dict):
        x = np.vstack(list(feat.values()))
        rels = list(ei.keys())
        eis = [ei[r] for r in rels]
        et = np.concatenate([np.full(e.shape[1], i) for i, e in enumerate(eis)])
        return x, np.hstack(eis), et, rels
    return feat, ei, None, None


def prepare(name):
    z, meta = load_case(name)
    feat, ei = case_inputs(z)
    x, e, et, rels = homogenize(feat, ei)
    names = meta["names"]
    if isinstance(names, dict):
        names = [n for v in names.values() for n in v]
    q = names.index(meta["element"])
    if "graph" in meta["problem"]:
        sub_x, sub_ei, sub_ind, sub_et = x, e, q, et
    else:
        hops = len(meta["arch_spec"]["dims"]) - 1
        subset, sub_ei, sub_ind, emask = oracle.comp_graph(q, hops, e, x.shape[0])
        sub_x = x[subset]
        sub_et = None if et is None else et[emask]
    if rels is None:
        rel_ei = {None: sub_ei}
    else:
        rel_ei = {r: sub_ei[:, sub_et == i] for i, r in enumerate(rels)}
    spec = oracle_spec(meta, state_dict(z))
    return z, meta, spec, sub_x, rel_ei, sub_ind


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference(name):
    z, meta, spec, sub_x, rel_ei, sub_ind = prepare(name)
    masks = repeat_masks(z, meta)
    for i, m in enumerate(masks):
        assert m.shape[1] == sub_x.shape[0]
        y = oracle.masked_query_outputs(spec, sub_x, rel_ei, m, sub_ind)
        np.testing.assert_allclose(y, z[f"r{i}_output"], rtol=0, atol=2e-6)
        k = oracle.shap_kernel(m)
        np.testing.assert_allclose(k, z[f"r{i}_kernel"], rtol=1e-12, atol=0)
        bs = meta[f"r{i}_batch_size"]
        w, losses, best = oracle.train_wlm(m, bs, z[f"r{i}_output"], z[f"r{i}_kernel"],
                                           z[f"r{i}_w0"], meta["params"])
        np.testing.assert_allclose(w, z[f"r{i}_w_final"], rtol=0, atol=2e-5)
        np.testing.assert_allclose(losses, z[f"r{i}_losses"], rtol=1e-5, atol=1e-12)
        assert best == meta[f"r{i}_best_epoch"]


@pytest.mark.parametrize("cols", [9, 200, 1001, 1002, 1500, 3000, 20000])
def test_oracle_shap_kernel_paths(cols):
    z = np.load(__import__("golden_utils").GOLDEN + "/kernels.npz")
    m = np.unpackbits(z[f"c{cols}_mask_bits"], axis=1, bitorder="little")[:, :cols].astype(bool)
    np.testing.assert_allclose(oracle.shap_kernel(m), z[f"c{cols}_kernel"], rtol=1e-12, atol=0)


def test_oracle_dataframes_match_reference():
    """weight_stacking + config_val_dataframe + aggregate (explainer.py:523-532) on the
    reference's own final weights reproduce the reference DataFrames."""
    for name in ["test_run", "toy", "gcn2_graph", "hetero_single"]:
        z, meta = load_case(name)
        ws = [z[f"r{i}_w_final"] for i in range(meta["n_repeats"])]
        mean, std = oracle.weight_stacking(ws)
        df = meta["df"]
        got = {n: (mu, sd) for n, mu, sd in oracle.config_val_table(
            mean, std, _sub_names(name))}
        for n, mu, sd in zip(df["index"], df["config_value_mean"], df["config_value_std"]):
            assert abs(got[n][0] - mu) < 1e-6 and abs(got[n][1] - sd) < 1e-6


def _sub_names(name):
    z, meta, spec, sub_x, rel_ei, sub_ind = prepare(name)
    names = meta["names"]
    if isinstance(names, dict):
        names = [n for v in names.values() for n in v]
    if "graph" in meta["problem"]:
        return names
    feat, ei = case_inputs(z)
    x, e, et, rels = homogenize(feat, ei)
    hops = len(meta["arch_spec"]["dims"]) - 1
    subset, _, _, _ = oracle.comp_graph(names.index(meta["element"]), hops, e, x.shape[0])
    return [names[i] for i in subset]


def test_oracle_known_answers():
    """Known-answer vectors of the reference unit tests (data as given in the reference tests):
    build_edge_mask (tests/test_data.py:1761-1845), pathway_mask2node_mask
    (tests/test_pathways.py:393-450), aggregate (tests/test_pathways.py:452-494),
    weighted_mse_loss (tests/test_wlm.py:378-404), original SHAP kernel (tests/test_kernels.py:40-95)."""
    mask = np.array([[1, 0, 1, 0, 1, 0, 1], [1, 1, 1, 1, 0, 0, 0], [0, 0, 0, 0, 1, 1, 1]], bool)
    ei = np.array([[0, 2, 3, 6, 4, 5], [5, 6, 4, 1, 2, 0]])
    keep, tiled = oracle.build_edge_mask(mask, ei)
    assert tiled.tolist() == [[0, 2, 3, 6, 4, 5, 7, 9, 10, 13, 11, 12, 14, 16, 17, 20, 18, 19],
                              [5, 6, 4, 1, 2, 0, 12, 13, 11, 8, 9, 7, 19, 20, 18, 15, 16, 14]]
    assert np.flatnonzero(keep).tolist() == [1, 4]
    pe, et = oracle.perturb_node(mask, ei, np.array([0, 0, 0, 1, 1, 1]))
    assert pe.tolist() == [[2, 4], [6, 2]] and et.tolist() == [0, 1]

    comm = [[3], [1, 2, 3, 4], [5, 7], [7, 8, 0, 4]]
    pm = np.array([[0, 0, 0, 0], [0, 0, 0, 1], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 1, 0],
                   [0, 1, 0, 1], [1, 1, 0, 0], [1, 1, 1, 0], [1, 0, 0, 0]], bool)
    em, rep = oracle.pathway_mask2node_mask(comm, pm)
    assert em.shape == (9, 11)
    assert em[1].tolist() == [0] * 7 + [1] * 4 and em[7].tolist() == [1] * 7 + [0] * 4

    cv = np.array([0.21, 0.23, 0.95, 0.65, 0.98, -0.21, 0.32, 0.94, -0.34], np.float32)
    agg = oracle.aggregate(cv, comm, ["1", "2", "3", "4"])
    assert [n for n, _ in agg] == ["2", "1", "4", "3"]
    np.testing.assert_allclose([s for _, s in agg], [0.7025, 0.65, 0.4475, 0.365], atol=1e-6)

    # tests/test_wlm.py:378-404 vectors: flat target, elementwise (no broadcast).  Expected value
    # written out: sum k (p - r)^2 = 0.5*.0025 + .85*.0036 + .34*.0049 + .78*.0049 = 0.009798,
    # / 4 (mean) / 2.47 (sum k)
    p = np.array([0.98, 0.23, -0.12, -0.24])
    r = np.array([0.93, 0.29, -0.19, -0.31])
    kk = np.array([0.5, 0.85, 0.34, 0.78])
    assert abs(oracle.weighted_mse_loss(p, r, kk) - 0.009798 / 4 / 2.47) < 1e-12
    # the train_model call site's [B, 1] target broadcasts to [B, B] (quirk Q1): closed form
    # (1/B) sum_j k_j [(p_j - ybar)^2 + var(y)] / sum k
    q1 = (np.mean(kk * (p - r.mean()) ** 2) + r.var() * kk.mean()) / kk.sum()
    assert abs(oracle.weighted_mse_loss(p, r[:, None], kk) - q1) < 1e-12
    assert abs(oracle.weighted_mse_loss(p, r[:, None], kk) - oracle.weighted_mse_loss(p, r, kk)) > 1e-4

    m9 = np.array([[0] * 9, [1, 0, 0, 0, 1, 0, 0, 1, 1], [0, 1, 1, 1, 1, 0, 0, 0, 0]], bool)
    k9 = oracle.shap_kernel(m9)
    assert k9[0] == 0.0
    assert abs(k9[1] - 8 / (126 * 4 * 5)) < 1e-15
