"""Pin the oracle's multi-node-type restatement (oracle.hetero_multi_copy_outputs +
hetero_multi_targets) against the reference run recorded in tests/golden/hetero_multi.*
(make_golden.py case_hetero_multi: 3 node types, 5 relations, 2-layer HeteroConv(SAGE)).
CPU only."""
import numpy as np

import oracle
from golden_utils import hetero_multi_setup, load_case, repeat_masks


def test_oracle_multi_type_targets_match_reference():
    z, meta = load_case("hetero_multi")
    c = hetero_multi_setup(z, meta)
    masks = repeat_masks(z, meta)
    S = c["x"].shape[0]
    for i, m in enumerate(masks):
        assert m.shape[1] == S
        y = oracle.hetero_multi_copy_outputs(c["spec"], c["x"], c["nt"], c["ei"], c["et"],
                                             c["ntypes"], c["rels"], c["pads"], m, c["sub_ind"])
        tg = oracle.hetero_multi_targets(y, meta[f"r{i}_batch_size"], c["sub_ind"], S)
        got = np.concatenate(tg)
        np.testing.assert_allclose(got, z[f"r{i}_output"], rtol=0, atol=2e-6)


def test_oracle_multi_type_full_fit_matches_reference():
    """Targets -> KernelSHAP -> surrogate fit (Q1 with a single broadcast target) against the
    recorded final weights and losses."""
    z, meta = load_case("hetero_multi")
    c = hetero_multi_setup(z, meta)
    masks = repeat_masks(z, meta)
    S = c["x"].shape[0]
    for i, m in enumerate(masks):
        B = meta[f"r{i}_batch_size"]
        y = oracle.hetero_multi_copy_outputs(c["spec"], c["x"], c["nt"], c["ei"], c["et"],
                                             c["ntypes"], c["rels"], c["pads"], m, c["sub_ind"])
        tg = oracle.hetero_multi_targets(y, B, c["sub_ind"], S)
        y_rows = np.concatenate([np.full(min(B, m.shape[0] - j * B), t[0])
                                 for j, t in enumerate(tg)])
        kern = oracle.shap_kernel(m)
        np.testing.assert_allclose(kern, z[f"r{i}_kernel"], rtol=1e-12)
        w, losses, best = oracle.train_wlm(m, B, y_rows, kern, z[f"r{i}_w0"], meta["params"])
        np.testing.assert_allclose(w, z[f"r{i}_w_final"], rtol=0, atol=2e-5)
        np.testing.assert_allclose(losses, z[f"r{i}_losses"], rtol=1e-4, atol=1e-9)
        assert best == meta[f"r{i}_best_epoch"]
