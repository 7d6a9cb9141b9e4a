"""`Explainer` — drop-in for pathway_explanations.explainer.Explainer (explainer.py:25-546).

Same constructor, assertions and `run(element, times) -> (config_val_df, pathway_df)`.  The
host orchestration (hetero flattening, computational subgraph, community filtering, output
DataFrames) follows the reference step by step; the per-repeat hot path runs on the MI355X:

  one ForwardPlan per query (receptive-field CSR + layer-1 tables, built once) ->
  per repeat: masks -> bit-pack -> masked forward -> KernelSHAP -> surrogate Adam loop.

Repeats draw masks and the surrogate's initial weights from torch's CPU generator in the
reference's order (compat sampler), so results match the reference CPU path for the same seed.
"""
import collections.abc
import operator
import random
import time
import warnings
import weakref

import numpy as np
import torch

from . import _lib, engine, frames, pipeline, sharding
from .data import Data
from .masks import Mask, dataloader_seed_draw
from .model import Model
from .pathways import Pathways
from .wlm import LinearRegression


class PhaseClock:
    """Phase boundaries of one run: a host timestamp and a CUDA event on the current stream at
    each mark (no synchronisation); `times()` synchronises once and returns, per phase, the
    host wall milliseconds and the device milliseconds between its two events."""

    def __init__(self, stream=None):
        self.marks = []
        self.stream = stream  # the run's stream (torch.cuda.current_stream() per mark: ~9 us)

    def mark(self, name):
        ev = None
        if self.stream is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(self.stream)
        self.marks.append((name, time.perf_counter(), ev))

    def times(self):
        if len(self.marks) < 2:
            return {}
        if self.stream is not None:
            torch.cuda.synchronize()
        out = {}
        for (name, t0, e0), (_, t1, e1) in zip(self.marks, self.marks[1:]):
            out[name] = {"host_ms": (t1 - t0) * 1e3,
                         "device_ms": e0.elapsed_time(e1) if e0 is not None else None}
        out["total_host_ms"] = (self.marks[-1][1] - self.marks[0][1]) * 1e3
        return out


def set_seed(seed=100):
    """explainer.py:14-22."""
    random.seed(seed)
    np.random.seed(seed + 1)
    torch.manual_seed(seed + 2)
    torch.cuda.manual_seed(seed + 3)
    torch.cuda.manual_seed_all(seed + 4)
    torch.backends.cudnn.enabled = False
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False


class Explainer:
    def __init__(self, feat, edge_index, arch, params, names, pathways=None, pathway_names=None,
                 element_type=None, problem="node_prediction", node_types=None,
                 edge_types=None):
        self.initial_assertions(feat, edge_index, arch, params, names, pathways, pathway_names,
                                element_type, problem)
        self.feat = feat
        self.edge_index = edge_index
        self.arch = arch
        self.params = params
        self.names = names
        self.pathways = pathways
        self.pathway_names = pathway_names
        self.element_type = element_type
        self.problem = problem.lower().strip()
        self.node_types = node_types
        self.edge_types = edge_types
        self.last_run = None  # diagnostics of the last run (per-repeat losses, path used)
        self.group = None     # torch.distributed process group for multi-GPU runs (None = world)
        self._verified = set()  # module states whose compiled program passed verify_plan
        self._queries = {}      # per-query (prepare context, plan, arch check): _query_key

    @property
    def edge_masks(self):
        """Non-compat edge problems (params["edge_masks"] = True): mask columns
        are the computational graph's edges (Data.perturb_edge, data.py:500-554) and the arch is
        an edge-level model (nn.LinkModel).  Off (default), edge problems fail as the reference's
        do (masks.py:294)."""
        return "edge" in self.problem and bool(self.params.get("edge_masks", False))

    @staticmethod
    def initial_assertions(feat, edge_index, arch, params, names, pathways, pathway_names,
                           element_type, problem):
        """explainer.py:106-189 (same messages)."""
        if pathways is not None:
            assert isinstance(pathways, (list, dict)), "Pathways is not list or dict"
        if pathway_names is not None:
            assert isinstance(pathway_names, (list, dict)), "Pathway names is not list or dict"
            assert len(pathway_names) == len(pathways), \
                "Length of list with pathway names and list with pathway indexes do not match"
        assert isinstance(feat, (torch.Tensor, dict)), \
            "Feature matrix is not torch tensor or dict"
        assert isinstance(edge_index, (torch.Tensor, dict)), \
            "Edge index matrix is not torch tensor or dict"
        assert isinstance(names, (list, dict)), "Element names is not list or dict"
        assert isinstance(params, dict), "Hyperparameters given is not dictionary"
        assert isinstance(problem, str), "Problem type given is not string"
        if element_type is not None:
            assert isinstance(element_type, (str, tuple)), \
                "Element type is not string (node) nor tuple (edge)"
            if "node" in problem:
                assert isinstance(feat, dict), "Feature given is not a dict of node types"
                assert element_type in list(feat.keys()), \
                    "Node type '{}' is not among input node types in heterogeneous graph" \
                    .format(element_type)
            elif "edge" in problem:
                assert isinstance(edge_index, dict), \
                    "Edge index given is not a dict of edge index types"
                assert element_type in list(edge_index.keys()), \
                    "Edge type '{}' is not among input node types in heterogeneous graph" \
                    .format(element_type)

    @staticmethod
    def extract_index(element, names=None):
        """explainer.py:191-226: the first position whose name (as numpy's str) equals element.
        String elements look up a name -> first position index built once per names list (the
        reference converts the whole list to a numpy str array on every call: ~50 ms at 1M)."""
        if names is None:
            assert isinstance(element, (int, float)), \
                "No element names have been given and the node name given is not numeric"
            return int(element)
        if isinstance(element, str):
            idx = _name_index(names, element)
            assert _is_member(element, names, idx), \
                "Element name '{}' is not present in the graph".format(element)
            return idx[element]
        assert element in names, "Element name '{}' is not present in the graph".format(element)
        return int(np.where(np.array(names, dtype=str) == element)[0][0])

    def filter_hetero_names(self, names, node_type, edge_type, node_type_names,
                            edge_type_names):
        """explainer.py:228-286."""
        arr = np.array(names, dtype=str)
        if isinstance(self.element_type, str):
            idx = torch.where(node_type == node_type_names.index(self.element_type))[0]
        elif isinstance(self.element_type, tuple):
            idx = torch.where(edge_type == edge_type_names.index(self.element_type))[0]
        else:
            idx = torch.where(node_type == 1)[0]
        return arr[idx.cpu().numpy()].tolist()

    @staticmethod
    def weight_stacking(weights):
        """explainer.py:288-314 — mean and population std over repeats (one fused reduction);
        `weights` is the list of per-repeat weight tensors, or already their [times, S] stack."""
        stack = weights if isinstance(weights, torch.Tensor) and weights.dim() == 2 else \
            torch.vstack(weights)
        std, mean = torch.std_mean(stack, 0, unbiased=False)
        return mean, std

    def _place_arch(self, device):
        """self.arch.to(device).eval() (explainer.py:338-339), skipped when every module is
        already in eval mode and every parameter / buffer on `device`: Module.to + eval walk the
        module tree through _apply (~0.15 ms of host time per call); the check is ~20 us.
        Returns the module's parameters and buffers (Module.parameters() / buffers() order, one
        walk of the tree for the whole run) and their state: (storage, in-place version) each."""
        mods = list(self.arch.modules())
        params, bufs, seen = [], [], set()
        for m in mods:
            for group, out in ((m._parameters, params), (m._buffers, bufs)):
                for t in group.values():
                    if t is not None and id(t) not in seen:
                        seen.add(id(t))
                        out.append(t)
        if any(m.training for m in mods) or any(t.device != device for t in params + bufs):
            self.arch = self.arch.to(device).eval()  # same tensor objects, moved storage
        state = (tuple((t.data_ptr(), t._version) for t in params),
                 tuple((t.data_ptr(), t._version) for t in bufs))
        return params, bufs, state

    def _verify_key(self, plan, c, state):
        """What the compiled program's check depends on: the module object, every parameter
        and buffer (`state`: storage and in-place version counter: an optimizer step or
        load_state_dict changes them), the plan kind, the graph's type structure and the plan's
        query-dependent lowering (ForwardPlan drops other destination types' relation terms from a
        layer whose targets share one node type, so two queries can lower the same module
        differently)."""
        return (id(self.arch), state[0], state[1], self.edge_masks, bool(getattr(plan, "multi_type", False)),
                tuple(c["h_ntypes"] or ()), tuple(c["h_etypes"] or ()),
                tuple(getattr(plan, "lowering", ())))

    def _query_key(self, element, device):
        """The cache slot of a query: element, problem, device and modes.  Whether the slot's
        entry still holds for the current inputs is `_query_sources` + `_query_content_ok`'s
        business (prepare() draws no random numbers, so reusing its result leaves every RNG
        stream as the reference's)."""
        return (str(element), type(element).__name__, self.problem, self.edge_masks, str(device),
                _freeze(self.element_type), str(self.params.get("verify_arch", True)))

    def _query_sources(self, params, bufs):
        """Identity snapshot of what prepare() and the query's ForwardPlan read: the graph and
        type tensors (weak reference + storage + in-place version: a replaced tensor, even one
        the allocator put at the freed address, or an in-place edit never matches), the names /
        pathways inputs and the module (identity), the module's parameters and buffers."""
        return _snapshot((self.feat, self.edge_index, self.node_types, self.edge_types,
                          self.names, self.pathways, self.pathway_names, self.arch,
                          tuple(params), tuple(bufs)))

    def _query_fingerprints(self):
        """Full-content fingerprints of the inputs read in full by prepare(): pathways and
        their names (community filtering), and hetero (dict) names."""
        return (_content_fp(self.pathways), _content_fp(self.pathway_names),
                _content_fp(self.names) if isinstance(self.names, dict) else None)

    def _query_content_ok(self, element, entry):
        """A cached entry's inputs are the same objects; check that their content did not change
        in place where prepare() read it: the pathways in full, the element's position in the
        names and the subgraph's names at their positions (O(S), not O(N))."""
        if entry["fp"] != self._query_fingerprints():
            return False
        c = entry["c"]
        if isinstance(self.names, dict) or c["ind"] is None:
            return True
        try:
            if self.extract_index(element, self.names) != c["ind"]:
                return False
        except AssertionError:
            return False
        if c["pos"] is not None:
            # the subgraph's name objects at their positions, compared as a tuple (identity
            # first, then ==): ~10 us at S = 1.2k instead of re-deriving the str forms (0.3 ms)
            return _pick(self.names, c["pos"]) == c["pos_names"]
        return True

    def clear_cache(self):
        """Drop every cached query (computational subgraph, plan and its device buffers), the
        architecture checks and the compiled programs with their padded weights.  The caches
        are keyed on the inputs' storage and in-place version counters; an edit that bumps no
        counter (through `param.data` or `tensor.data`, e.g. `p.data.copy_(w)`) is not seen by
        them: call this after one."""
        self._queries.clear()
        self._verified.clear()
        pipeline.clear_programs()

    def _trim_cache(self, keep):
        """Keep the cache within params["plan_cache_bytes"] device bytes (default 2 GiB) and
        8 queries: oldest entries out first; the entry of the query just run always stays."""
        limit = int(self.params.get("plan_cache_bytes", 2 << 30))
        user = None

        def nbytes(e):  # once per entry (an entry's tensors never change)
            nonlocal user
            if "bytes" not in e:
                if user is None:
                    user = _tensor_ptrs((self.feat, self.edge_index, self.node_types, self.edge_types))
                ctx = sum(t.numel() * t.element_size() for t in e["c"].values()
                          if isinstance(t, torch.Tensor) and t.data_ptr() not in user)
                e["bytes"] = ctx + (e["plan"].device_bytes() if e["plan"] is not None else 0)
            return e["bytes"]
        total = {k: nbytes(e) for k, e in self._queries.items()}
        for k in list(self._queries):
            if k == keep:
                continue
            if len(self._queries) <= 8 and sum(total.values()) <= limit:
                break
            del self._queries[k]
            total.pop(k)

    # ------------------------------------------------------------------------------ run
    def prepare(self, element, device):
        """Host orchestration of explainer.py:345-480 (no RNG consumed): heterogeneous
        flattening, computational subgraph, community filtering.  Returns a dict context."""
        feat, ei = _to_device(self.feat, device), _to_device(self.edge_index, device)
        raw = Data(feat, ei)
        pw_raw = Pathways(self.pathways, self.pathway_names) if self.pathways is not None else None
        (h_ntypes, h_etypes, feat, ei, node_types, edge_types, node_ptrs, edge_ptrs,
         padded_dims) = raw.preprocess_hetero_graph()
        if node_types is None and self.node_types is not None:
            node_types = self.node_types.clone().to(device)
        if edge_types is None and self.edge_types is not None:
            edge_types = self.edge_types.clone().to(device)
        names, _ = raw.hetero2homo_names(self.names)
        pathways = pathway_names = pathway_types = None
        if pw_raw is not None:
            pathways, pathway_names, pathway_types = pw_raw.hetero2homo(self.problem, node_ptrs,
                                                                       edge_ptrs)
        data = Data(feat, ei)
        sub_pw = sub_pw_names = None
        sub_nt = sub_et = None
        link = pos = None
        if self.edge_masks:
            # edge problem, edge masks (non-compat: the reference's edge path is broken at
            # masks.py:294 and data.py:331): mask columns = the computational graph's edges
            if h_etypes is not None or node_types is not None or edge_types is not None:
                raise NotImplementedError("edge masks: homogeneous graphs only")
            n_hops = Model(self.arch).get_hops(0)
            ind = self.extract_index(element, names)
            sub_feat, sub_ei, sub_names, sub_ind, link, pos = data.edge_comp_graph(
                ind, n_hops, names, return_pos=True)
            if pathways is not None:
                sub_pw, sub_pw_names, _ = Pathways(pathways, pathway_names,
                                                   pathway_types).comp_graph(sub_names)
        elif "graph" not in self.problem:
            rels = len(h_etypes) if h_etypes is not None else 0
            n_hops = Model(self.arch).get_hops(rels)
            ind = self.extract_index(element, names)
            sub_feat, sub_ei, sub_names, sub_ind, sub_nt, sub_et, pos = data.comp_graph(
                ind, n_hops, self.problem, names, node_types, edge_types, return_pos=True)
            if pathways is not None:
                sub_pw, sub_pw_names, _ = Pathways(pathways, pathway_names,
                                                   pathway_types).comp_graph(sub_names)
        else:
            # the whole graph (explainer.py:427-447; the reference clones it, nothing here
            # writes to it, so the run reads the caller's tensors and names directly)
            sub_feat, sub_ei, sub_names = feat, ei, names
            ind = sub_ind = self.extract_index(element, sub_names)
            sub_nt, sub_et = node_types, edge_types
            if pathways is not None:
                sub_pw, sub_pw_names = pathways, pathway_names
        if "graph" not in self.problem and not self.edge_masks and (self.element_type is not None or
                                            self.node_types is not None or
                                            self.edge_types is not None):
            filt = self.filter_hetero_names(sub_names, sub_nt, sub_et, h_ntypes, h_etypes)
            sub_ind = self.extract_index(element, filt)
        sub_pw_inds = None
        if pathways is not None:
            spc = Pathways(sub_pw, sub_pw_names)
            if isinstance(sub_pw[0][0], str):
                sub_pw_inds = spc.names2inds(sub_names)
            elif isinstance(sub_pw[0][0], int):
                sub_pw_inds = sub_pw
        if isinstance(sub_ind, torch.Tensor):
            sub_ind = int(sub_ind.reshape(-1)[0])
        S = Data(sub_feat, sub_ei).element_size(self.problem)
        return {"link": link, "sub_feat": sub_feat, "sub_ei": sub_ei, "sub_names": sub_names,
                "sub_ind": sub_ind, "sub_nt": sub_nt, "sub_et": sub_et, "h_ntypes": h_ntypes,
                "h_etypes": h_etypes, "padded_dims": padded_dims, "sub_pw": sub_pw,
                "sub_pw_names": sub_pw_names, "sub_pw_inds": sub_pw_inds, "S": S,
                "has_pathways": pathways is not None, "ind": ind,
                "pos": tuple(pos.tolist()) if pos is not None else None,
                "pos_names": _pick(names, tuple(pos.tolist())) if pos is not None else None}

    def run(self, element, times=1):
        """explainer.py:316-546."""
        if not torch.cuda.is_available():
            raise _lib.NativeLibraryError("Explainer.run needs an MI355X (HIP) device; "
                                          "there is no CPU fallback")
        _lib.load()
        device = torch.device("cuda", torch.cuda.current_device())
        clock = PhaseClock(torch.cuda.current_stream(device))
        clock.mark("setup")
        if times == 1:
            set_seed(self.params["seed"])
        # multi-GPU: every rank continues from rank 0's generator, so all ranks draw the same
        # masks / sampler seeds / initial weights (checked by checksum below)
        sharding.sync_rng(self.group)
        params, bufs, mstate = self._place_arch(device)
        clock.mark("prepare")
        # a query explained again (same graph, names, module state) reuses its computational
        # subgraph, plan and arch check: prepare() and the plan build are the run's largest host
        # costs (explainer.py:345-480 redone by the reference on every call)
        qkey = self._query_key(element, device) if self.params.get("plan_cache", True) else None
        entry = self._queries.get(qkey) if qkey is not None else None
        cached = None
        if entry is not None:
            if _matches(self._query_sources(params, bufs), entry["src"]) and \
                    self._query_content_ok(element, entry):
                cached = (entry["c"], entry["plan"], entry["arch_check"])
            else:
                del self._queries[qkey]  # stale: the inputs changed since it was prepared
        hit = cached is not None
        c = cached[0] if cached else self.prepare(element, device)
        sub_feat, sub_ei, sub_ind, S = c["sub_feat"], c["sub_ei"], c["sub_ind"], c["S"]
        geo = (c["sub_nt"], c["sub_et"], c["h_ntypes"], c["h_etypes"], c["padded_dims"])

        # masks before the plan: the sampler kernels and the initial-weight copy run on the device
        # while the host builds the plan (the plan build and its arch check draw no numbers from
        # the global generators, so the reference's RNG order is unchanged)
        clock.mark("sample")
        sampler = self.params.get("mask_sampler", "compat")
        _, epochs = Mask.assertions_mask_generator(self.params)
        # draw every repeat's masks and initial surrogate weights first, in the reference's
        # RNG order (mask_generator -> LinearRegression init -> DataLoader seed, per repeat);
        # then run all repeats' forward / KernelSHAP / surrogate fits as batched launches.
        bits_list, w0_list, masks = [], [], []
        on_device = sampler == "device" and ("edge" not in self.problem or self.edge_masks)
        # edge masks: the samplers see S = edge count columns (the element size of
        # data.py:383-385) through a node-problem Mask over an [S, 1] placeholder feature
        mfeat = torch.zeros((S, 1), device=device) if self.edge_masks else sub_feat
        mproblem = "node_prediction" if self.edge_masks else self.problem
        if on_device and c["sub_pw_inds"] is not None:
            # device community sampler: the block plan and column -> community CSR are
            # repeat-invariant; each repeat draws a new seed (masks.py:262-397)
            cmask = Mask(mfeat, sub_ei, c["sub_pw_inds"], self.params, mproblem)
            cplan = cmask.community_plan()
            ctabs = engine.community_tables(cplan, c["sub_pw_inds"], S, device)
        seeds = []  # device Shapley sampler: every repeat's seed first, then one native call
        draws = None
        if on_device and c["sub_pw_inds"] is None:
            # every repeat's seed, initial weights and DataLoader draw replayed natively from the
            # generator state (the same numbers and end state as the torch calls below)
            draws = engine.repeat_draws(times, S)
        if draws is not None:
            seeds = draws[0]
            w0_list = draws[1]  # [times, S]: indexed per repeat like the list
            masks = [None] * times
        for _ in range(0 if draws is not None else times):
            if on_device and c["sub_pw_inds"] is None:
                seeds.append(torch.randint(0, 2 ** 62, (1,)))  # read together below
                masks.append(None)
            elif on_device:
                seed = int(torch.randint(0, 2 ** 62, (1,)).item())
                bits_list.append(engine.sample_communities(seed, cplan, c["sub_pw_inds"], S,
                                                           device, tables=ctabs)[0])
                masks.append(None)
            else:  # compat: the reference's CPU draws, bit-identical, packed on the device
                bits_c, _ = Mask(mfeat, sub_ei, c["sub_pw_inds"], self.params,
                                 mproblem).generate_bits(device)
                bits_list.append(bits_c)
                masks.append(None)
            w0_list.append(LinearRegression.initial_weights(S))
            dataloader_seed_draw()
        if seeds:
            if draws is None:
                seeds = torch.cat(seeds).tolist()
            bits = engine.sample_shapley_sets(seeds, int(self.params["interpret_samples"] * epochs),
                                              S, device)       # [times, R, W]
        else:
            bits = torch.stack(bits_list)                   # [times, R, W]
        R = bits.shape[1]
        batch = R // epochs
        # multi-GPU (torch.distributed initialised, one process per GPU): rows of the forward /
        # KernelSHAP and whole surrogate fits are sharded over ranks, outputs all-gathered, so
        # every rank returns the single-GPU result (sharding.py).
        flat = bits.reshape(times * R, -1)
        g = self.group
        sharding.assert_replicated(bits, "mask rows", g)
        w0_all = draws[1] if draws is not None else torch.stack(w0_list)
        sharding.assert_replicated(w0_all, "initial surrogate weights", g)
        # the initial weights go to the device through the pinned staging ring (a pageable host ->
        # device copy waits for everything queued on the stream first)
        w0_dev = engine.h2d(w0_all.numpy(), device)

        clock.mark("plan")

        if cached:
            plan, verify = cached[1], None
        elif self.edge_masks:
            plan = pipeline.build_edge_plan(self.arch, sub_feat, sub_ei, *c["link"],
                                            module_state=mstate)
            verify = lambda: pipeline.verify_edge_plan(plan, self.arch, sub_feat, sub_ei, *c["link"])
        else:
            plan = pipeline.build_plan(self.arch, sub_feat, sub_ei, [sub_ind], *geo,
                                       module_state=mstate)
            verify = lambda: pipeline.verify_plan(plan, self.arch, sub_feat, sub_ei, sub_ind, *geo)
        clock.mark("verify")
        arch_check = "off"
        mode = self.params.get("verify_arch", True)
        if cached:
            arch_check = cached[2] if cached[2] in ("off", "failed") else "cached"
            if mode == "always" and plan is not None:
                cached = None  # checked again below
        if plan is not None and mode and not cached:
            if verify is None:
                verify = lambda: pipeline.verify_plan(plan, self.arch, sub_feat, sub_ei, sub_ind, *geo) \
                    if not self.edge_masks else pipeline.verify_edge_plan(plan, self.arch, sub_feat, sub_ei,
                                                                          *c["link"])
            # the check guards the arch lowering (program.compile_arch + the plan's term
            # dropping), which depends on the module, the graph's type structure and the query
            # layer's node types: once per module state (parameter storage + in-place version
            # counters), type structure and lowering per Explainer; params["verify_arch"] =
            # "always" checks every run
            key = self._verify_key(plan, c, mstate)
            if mode == "always" or key not in self._verified:
                ok, err = verify()
                if not ok:
                    warnings.warn(f"compiled arch disagrees with its torch forward (max err "
                                  f"{err:.3g}); using the generic torch path")
                    plan = None
                    arch_check = "failed"
                else:
                    self._verified.add(key)
                    arch_check = "verified"
            else:
                arch_check = "cached"
        if qkey is not None:
            self._queries.pop(qkey, None)  # (re)inserted as the newest entry
            self._queries[qkey] = {"c": c, "plan": plan, "arch_check": arch_check,
                                   "src": self._query_sources(params, bufs),
                                   "fp": entry["fp"] if hit else self._query_fingerprints()}
            if hit and "bytes" in entry and plan is entry["plan"]:
                self._queries[qkey]["bytes"] = entry["bytes"]

        # multi-node-type graphs: the reference's per-copy loop zeroes copies without edges and
        # its extraction re-cuts the [B] outputs (quirk Q4); params["hetero_q4"] = False keeps
        # the per-copy outputs instead (model.py:118-253, wlm.py:435-436)
        q4 = bool(self.params.get("hetero_q4", True))

        def kernel_rows(s, e):
            if e == s:
                return torch.empty(0, dtype=torch.float64, device=device)
            return engine.shap_kernel(flat[s:e], S)
        kern = None
        clock.mark("forward_shap")
        if plan is not None:
            # KernelSHAP needs only the mask bits: its kernels run on a side stream beside the
            # masked forward (sharding.gather_map_beside)
            y, kern = sharding.gather_map_beside(times * R, lambda s, e: plan.forward(flat[s:e])[:, 0],
                                                 kernel_rows, g)
            y = y.reshape(times, R)
            kern = kern.reshape(times, R)
            if getattr(plan, "multi_type", False):
                empty = pipeline.empty_copy_rows(flat, S, sub_ei).reshape(times, R)
                y = torch.stack([pipeline.multi_type_targets(y[i], empty[i], batch, sub_ind, S, q4)
                                 for i in range(times)])
        elif self.edge_masks:
            def generic(t0, t1):
                ys = [pipeline.generic_edge_outputs(
                    self.arch, sub_feat, sub_ei,
                    engine.unpack_masks(bits[i], S) if masks[i] is None else masks[i],
                    *c["link"], max_rows=batch) for i in range(t0, t1)]
                return torch.stack(ys) if ys else torch.empty((0, R), device=device)
            y = sharding.gather_map(times, generic, g)
        else:
            def generic(t0, t1):
                ys = [pipeline.generic_outputs(
                    self.arch, sub_feat, sub_ei,
                    engine.unpack_masks(bits[i], S) if masks[i] is None else masks[i],
                    sub_ind, self.problem, *geo, batch=batch, q4=q4) for i in range(t0, t1)]
                return torch.stack(ys) if ys else torch.empty((0, R), device=device)
            y = sharding.gather_map(times, generic, g)

        if kern is None:
            kern = sharding.gather_map(times * R, kernel_rows, g).reshape(times, R)

        fits = {}
        clock.mark("fit")
        # the fits' exchange status is read with the results (one host synchronisation, in the
        # output phase) instead of by a wait of its own right after the launch
        status = torch.zeros(1, dtype=torch.int32, device=device)

        def fit(t0, t1):
            if t1 == t0:
                n_steps = -(-R // batch)
                fits["losses"] = torch.empty((0, n_steps), dtype=torch.float64, device=device)
                fits["best"] = torch.empty(0, dtype=torch.int32, device=device)
                return torch.empty((0, S), device=device)
            w_, fits["losses"], fits["best"], _, _ = engine.wlm_fit(
                bits[t0:t1], S, batch, y[t0:t1], kern[t0:t1], w0_dev[t0:t1],
                self.params, check=False, status=status)
            return w_
        w = sharding.gather_map(times, fit, g)
        losses = sharding.gather_rows(fits["losses"], times, g)
        best = sharding.gather_rows(fits["best"], times, g)
        diag = _Repeats(losses=losses, best_epoch=best, rows=R, batch=batch, y=y, bits=bits,
                        kernel=kern, w0=w0_list)
        clock.mark("output")
        mean, std = self.weight_stacking(w)
        status_h = engine.status_to_host(status)
        # Data.config_val_dataframe (data.py:651-693); a computational subgraph's row labels are
        # derived once per cached query (its names list is built by prepare() and belongs to the
        # cache entry; the whole graph's columns are the caller's own names list, read each call)
        labels = None
        if c["pos"] is not None:
            if "labels" not in c:
                c["labels"] = frames.name_labels(c["sub_names"])
            labels = c["labels"]
        ms = torch.stack([mean.detach(), std.detach()]).cpu().numpy()
        config_val_df = frames.sorted_frame(c["sub_names"], {"config_value_mean": ms[0],
                                                             "config_value_std": ms[1]},
                                            "config_value_mean", labels=labels)
        engine.check_status_host(status_h)  # the frame's .cpu() waited for the copy
        pathway_df = None
        if c["has_pathways"]:
            pathway_df = Pathways(c["sub_pw"], c["sub_pw_names"]).aggregate(mean,
                                                                            c["sub_pw_inds"])
        clock.mark("end")
        if qkey is not None:
            self._trim_cache(qkey)
        self.last_run = {"engine": plan is not None, "repeats": diag, "S": S,
                         "sub_ind": sub_ind, "plan": plan, "weights": w.unbind(0),
                         "phases": clock, "arch_check": arch_check,
                         "query_cache": "off" if qkey is None else "hit" if hit else "miss"}
        return config_val_df, pathway_df

    def run_queries(self, elements, times=1):
        """Several graph_prediction queries over ONE mask set per repeat.

        The reference explains one element per `run` (explainer.py:316-546) and draws new masks
        each time.  In graph_prediction every query perturbs the same S = N columns
        (explainer.py:427-447), so here each repeat's masks are drawn once, one masked forward
        produces every query's logit per row (a multi-query ForwardPlan), KernelSHAP runs once,
        and each query gets its own surrogate fits (all of them in one launch while the
        replicated mask rows stay under params["run_queries_batch_bytes"], default 2 GiB; else
        one launch per query).  RNG order per repeat: masks, then one LinearRegression init per
        query, then the DataLoader seed draw — with one query this is exactly `run`'s order, so
        `run_queries([e]) == [run(e)]` (to the fit's 1e-4 bar when the batched launch splits each
        fit over fewer workgroups).  Multi-GPU: like `run`, the rows of the forward / KernelSHAP
        are sharded over ranks with one all-gather each, and the Q x times fits are sharded over
        ranks.  Returns [(config_val_df, pathway_df)] in `elements` order.  Engine-compilable
        single-node-type archs only."""
        assert "graph" in self.problem, \
            "run_queries shares one mask set across queries: graph_prediction problems only"
        if not torch.cuda.is_available():
            raise _lib.NativeLibraryError("Explainer.run_queries needs an MI355X (HIP) device; "
                                          "there is no CPU fallback")
        _lib.load()
        device = torch.device("cuda", torch.cuda.current_device())
        if times == 1:
            set_seed(self.params["seed"])
        g = self.group
        sharding.sync_rng(g)
        _, _, mstate = self._place_arch(device)
        c = self.prepare(elements[0], device)
        # graph_prediction: every query indexes the same (whole) graph, so only the element
        # lookup of `prepare` differs per query (explainer.py:427-447)
        inds = [c["sub_ind"]]
        for e in elements[1:]:
            ind = self.extract_index(e, c["sub_names"])
            inds.append(int(ind.reshape(-1)[0]) if isinstance(ind, torch.Tensor) else ind)
        sub_feat, sub_ei, S = c["sub_feat"], c["sub_ei"], c["S"]
        geo = (c["sub_nt"], c["sub_et"], c["h_ntypes"], c["h_etypes"], c["padded_dims"])
        Q = len(inds)
        assert len(set(inds)) == Q, "run_queries: duplicate query elements"
        plan = pipeline.build_plan(self.arch, sub_feat, sub_ei, inds, *geo, module_state=mstate)
        assert plan is not None and not getattr(plan, "multi_type", False), \
            "run_queries needs an engine-compilable single-node-type architecture"
        if self.params.get("verify_arch", True):
            ok, err = pipeline.verify_plan(plan, self.arch, sub_feat, sub_ei, inds, *geo)
            assert ok, f"compiled arch disagrees with its torch forward (max err {err:.3g})"
        sampler = self.params.get("mask_sampler", "compat")
        _, epochs = Mask.assertions_mask_generator(self.params)
        if sampler == "device" and c["sub_pw_inds"] is not None:
            cmask = Mask(sub_feat, sub_ei, c["sub_pw_inds"], self.params, self.problem)
            cplan = cmask.community_plan()
            ctabs = engine.community_tables(cplan, c["sub_pw_inds"], S, device)
        bits_list, w0 = [], [[] for _ in range(Q)]
        for _ in range(times):
            if sampler == "device":
                R = int(self.params["interpret_samples"] * epochs)
                seed = int(torch.randint(0, 2 ** 62, (1,)).item())
                bits_list.append(engine.sample_shapley(seed, R, S, device)
                                 if c["sub_pw_inds"] is None else
                                 engine.sample_communities(seed, cplan, c["sub_pw_inds"], S,
                                                           device, tables=ctabs)[0])
            else:  # compat: the reference's CPU draws, bit-identical, packed on the device
                bits_list.append(Mask(sub_feat, sub_ei, c["sub_pw_inds"], self.params,
                                      self.problem).generate_bits(device)[0])
            for q in range(Q):
                w0[q].append(LinearRegression.initial_weights(S))
            dataloader_seed_draw()
        R = bits_list[0].shape[0]
        batch = R // epochs
        bits = torch.stack(bits_list)                       # [times, R, W]
        w0_all = torch.stack([w for wq in w0 for w in wq])  # [Q * times, S], query-major
        sharding.assert_replicated(bits, "mask rows", g)
        sharding.assert_replicated(w0_all, "initial surrogate weights", g)
        flat = bits.reshape(times * R, -1)
        y = sharding.gather_map(times * R, lambda s, e: plan.forward(flat[s:e])[:, :Q],
                                g).reshape(times, R, Q)

        def kernel_rows(s, e):
            if e == s:
                return torch.empty(0, dtype=torch.float64, device=device)
            return engine.shap_kernel(flat[s:e], S)
        kern = sharding.gather_map(times * R, kernel_rows, g).reshape(times, R)
        limit = int(self.params.get("run_queries_batch_bytes", 2 << 30))

        def fit(u0, u1):
            # units u = q * times + i (query q, repeat i), a contiguous shard of them
            if u1 == u0:
                return torch.empty((0, S), device=device)
            us = torch.arange(u0, u1, device=device)
            q_of, i_of = us // times, us % times
            if (u1 - u0) * bits[0].numel() * 4 <= limit:
                ws, _, _, _, _ = engine.wlm_fit(
                    bits[i_of], S, batch, y[i_of, :, q_of], kern[i_of], w0_all[u0:u1],
                    self.params)
                return ws
            out = []  # one launch per query (its repeats batched)
            for q in range(int(q_of[0]), int(q_of[-1]) + 1):
                sel = (q_of == q).nonzero().reshape(-1)
                ii = i_of[sel]
                out.append(engine.wlm_fit(bits[ii], S, batch, y[ii, :, q], kern[ii],
                                          w0_all[(u0 + sel).cpu()], self.params)[0])
            return torch.cat(out)
        fitted = sharding.gather_map(Q * times, fit, g).reshape(Q, times, S)
        out = []
        for q in range(Q):
            w = fitted[q]
            mean, std = self.weight_stacking(w)
            df = Data(sub_feat, sub_ei).config_val_dataframe(mean, std, c["sub_names"])
            pdf = None
            if c["has_pathways"]:
                pdf = Pathways(c["sub_pw"], c["sub_pw_names"]).aggregate(mean, c["sub_pw_inds"])
            out.append((df, pdf))
        self.last_run = {"engine": True, "queries": inds, "S": S, "rows": R, "batch": batch,
                         "bits": bits, "y": y, "kernel": kern, "w0": w0_all.reshape(Q, times, S),
                         "weights": fitted, "plan": plan}
        return out


class _Repeats(collections.abc.Sequence):
    """last_run["repeats"]: per repeat i a dict of its losses, best epoch, rows, batch, forward
    outputs y, mask bits, KernelSHAP weights and initial surrogate weights, built when asked for
    (the run keeps the stacked tensors; 60 tensor views per times=10 call cost ~0.16 ms)."""

    def __init__(self, rows, batch, **stacked):
        self._rows, self._batch, self._t = rows, batch, stacked

    def __len__(self):
        return len(self._t["w0"])

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        t = self._t
        return {"losses": t["losses"][i], "best_epoch": t["best_epoch"][i], "rows": self._rows,
                "batch": self._batch, "y": t["y"][i], "bits": t["bits"][i],
                "kernel": t["kernel"][i], "w0": t["w0"][i]}


_NAME_INDEX = {}


def _name_index(names, element=None):
    """{str(name): first position} of a names list — the reference's
    np.where(np.array(names, dtype=str) == element)[0][0] as a lookup — cached by identity and
    length.  A hit is validated against the list itself (the cached position of `element` must
    still hold it, and a name missing from the index is looked for again), so a list edited in
    place is re-indexed instead of answering from a stale index; an edit that adds an EARLIER
    copy of an indexed name at the same length is not detected.  The index is a dict of str ->
    int (not tracked by Python's cyclic collector): a set or list of 1M names built per query
    would be traversed by the next collections (~3 ms each for 100k names, the first-call
    pauses of round 4)."""
    key = (id(names), len(names))
    hit = _NAME_INDEX.get(key)
    if hit is not None and hit[0] is names:
        idx = hit[1]
        if element is None:
            return idx
        i = idx.get(element)
        if i is not None and str(names[i]) == element:
            return idx
        if i is None and element not in names:
            return idx  # truly absent: the caller's assertion reports it
    idx = {}
    for i, n in enumerate(np.array(names, dtype=str).tolist() if len(names) else []):
        idx.setdefault(n, i)
    if len(_NAME_INDEX) > 8:
        _NAME_INDEX.clear()
    _NAME_INDEX[key] = (names, idx)
    return idx


def _is_member(element, names, idx):
    """The reference's `element in names` (explainer.py:222) for a str element: membership of
    the names themselves, not of their str forms ('5' is no member of [5]); O(1) when the name
    at the element's indexed position is the element itself (str names), else a scan."""
    i = idx.get(element)
    if i is None:
        return False
    return names[i] == element or element in names


def _pick(names, pos):
    """The name objects at positions `pos` (a tuple of ints) as a tuple (tuples of atoms leave
    the cyclic collector's lists; a list of S ints would stay tracked)."""
    if not pos:
        return ()
    if len(pos) == 1:
        return (names[pos[0]],)
    return operator.itemgetter(*pos)(names)


def _snapshot(x):
    """Identity snapshot of a run's input: tensors by weak reference + storage + in-place
    version, tuples / dicts entry by entry (dict key order included), anything else (lists,
    modules) by identity."""
    if isinstance(x, torch.Tensor):
        return ("t", weakref.ref(x), x.data_ptr(), x._version, tuple(x.shape))
    if isinstance(x, tuple):
        return ("u", tuple(_snapshot(v) for v in x))
    if isinstance(x, dict):
        return ("d", tuple(x.keys()), tuple(_snapshot(v) for v in x.values()))
    return ("o", x)


def _matches(a, b):
    """Do two snapshots (`_snapshot`) name the same objects in the same state?"""
    if a[0] != b[0]:
        return False
    if a[0] == "t":
        return a[1]() is not None and a[1]() is b[1]() and a[2:] == b[2:]
    if a[0] == "u":
        return len(a[1]) == len(b[1]) and all(_matches(x, y) for x, y in zip(a[1], b[1]))
    if a[0] == "d":
        return a[1] == b[1] and all(_matches(x, y) for x, y in zip(a[2], b[2]))
    return a[1] is b[1]


def _freeze(x):
    """Hashable, content-equal form of a nested list / tuple / dict of plain values."""
    if isinstance(x, (list, tuple)):
        return tuple(_freeze(v) for v in x)
    if isinstance(x, dict):
        return tuple((k, _freeze(v)) for k, v in x.items())
    if isinstance(x, torch.Tensor):
        return ("tensor", x.data_ptr(), x._version, tuple(x.shape))
    return x


def _content_fp(x):
    """Full-content fingerprint of a names / pathways input (None stays None)."""
    if x is None:
        return None
    f = _freeze(x)
    try:
        return (len(x), hash(f))
    except TypeError:
        return (len(x), repr(f))


def _tensor_ptrs(xs):
    """Storage pointers of the tensors in a nested tuple / dict of inputs."""
    out = set()
    for x in xs:
        if isinstance(x, torch.Tensor):
            out.add(x.data_ptr())
        elif isinstance(x, dict):
            out |= _tensor_ptrs(tuple(x.values()))
    return out


def _to_device(x, device):
    if isinstance(x, dict):
        return {k: v.to(device) for k, v in x.items()}
    return x.to(device)
