"""MI355X-native XP-GNN perturbation-scoring engine.

Drop-in for the `pathway_explanations` package of andres2631996/bikg_graph_explainability_public
(same module names: explainer, masks, kernels, model, pathways, wlm, data):

    import bikg_graph_explainability_public_amd as pathway_explanations
    from bikg_graph_explainability_public_amd.explainer import Explainer, set_seed

The hot path (mask sampling x masked k-hop message passing x kernel-weighted linear fit) runs
in hand-written HIP kernels for gfx950 (csrc/xpgnn.hip, C-ABI include/xpgnn.h).
"""
from .data import Data
from .explainer import Explainer, set_seed
from .kernels import Kernel
from .masks import Mask
from .model import Model
from .pathways import Pathways
from .wlm import LinearRegression

__all__ = ["Data", "Explainer", "Kernel", "Mask", "Model", "Pathways", "LinearRegression",
           "set_seed"]
__version__ = "0.1.0"
