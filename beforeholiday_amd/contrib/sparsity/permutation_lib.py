"""Offline input-channel permutation of a model before 2:4 pruning (reference:
apex/contrib/sparsity/permutation_lib.py:42-925 — torch.fx graph, "siblings" sharing a
permutation, C-dim permutation of consumers and K-dim permutation of producers).

A permutation of the input channels of a sparse layer keeps the network function unchanged when the
same permutation is applied to every tensor carrying those channels. The graph analysis here
(torch.fx) groups layers into *channel spaces*:

* producers: Linear / Conv (groups=1) whose output channels define the space — permuted in K
  (weight rows, bias);
* channel-wise ops the space flows through: BatchNorm (weight, bias, running stats), LayerNorm over
  the channel dim, depthwise conv, pooling, activations, dropout — their parameters are permuted;
* joins: elementwise ``add``/``sub``/``mul``/``div`` of two spaces merge them (residual branches);
* consumers: Linear / Conv whose input channels live in the space — permuted in C.

A space is permutable iff every producer is a permutable layer, it never reaches the model output,
an unknown op, a reshape/flatten/cat, or a parameter used directly by the graph, and it has at least
one sparse consumer. One permutation is searched per space over the row-concatenation of its sparse
consumers' weights (convs viewed ``[R*S*K, C]``); on multi-rank jobs rank 0's permutation is
broadcast so all replicas stay identical.
"""
import json
import operator
import os

import torch
import torch.fx

from ...utils.logging import get_logger
from .permutation_search import accelerated_search_for_good_permutation, sum_after_2_to_4

_log = get_logger(__name__)

_CONV = (torch.nn.Conv1d, torch.nn.Conv2d, torch.nn.Conv3d)
_LAYERS = (torch.nn.Linear,) + _CONV
_BN = (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d, torch.nn.BatchNorm3d, torch.nn.SyncBatchNorm)
_TRANSPARENT_MODULES = (
    torch.nn.ReLU, torch.nn.ReLU6, torch.nn.GELU, torch.nn.SiLU, torch.nn.Sigmoid, torch.nn.Tanh, torch.nn.LeakyReLU,
    torch.nn.ELU, torch.nn.Hardswish, torch.nn.Hardsigmoid, torch.nn.Mish, torch.nn.Dropout, torch.nn.Dropout1d,
    torch.nn.Dropout2d, torch.nn.Dropout3d, torch.nn.Identity, torch.nn.MaxPool1d, torch.nn.MaxPool2d,
    torch.nn.MaxPool3d, torch.nn.AvgPool1d, torch.nn.AvgPool2d, torch.nn.AvgPool3d, torch.nn.AdaptiveAvgPool1d,
    torch.nn.AdaptiveAvgPool2d, torch.nn.AdaptiveAvgPool3d, torch.nn.AdaptiveMaxPool2d)
_UNARY_FUNCS = {
    torch.relu, torch.nn.functional.relu, torch.nn.functional.relu6, torch.nn.functional.gelu, torch.sigmoid,
    torch.tanh, torch.nn.functional.silu, torch.nn.functional.leaky_relu, torch.nn.functional.elu,
    torch.nn.functional.hardswish, torch.nn.functional.dropout, torch.nn.functional.max_pool2d,
    torch.nn.functional.avg_pool2d, torch.nn.functional.adaptive_avg_pool2d, torch.nn.functional.sigmoid,
    torch.nn.functional.tanh, operator.neg, torch.neg, torch.clone}
_UNARY_METHODS = {"relu", "relu_", "sigmoid", "tanh", "contiguous", "clone", "float", "half", "bfloat16", "neg",
                  "detach", "sigmoid_", "tanh_"}
_BINARY_FUNCS = {operator.add, operator.sub, operator.mul, operator.truediv, operator.iadd, operator.imul, torch.add,
                 torch.sub, torch.mul, torch.div}
_BINARY_METHODS = {"add", "add_", "sub", "sub_", "mul", "mul_", "div", "div_"}


def _is_depthwise(mod):
    return isinstance(mod, _CONV) and mod.groups > 1 and mod.groups == mod.in_channels == mod.out_channels


class _Space:
    __slots__ = ("parent", "producers", "consumers", "channelwise", "blocked", "cdim", "why")

    def __init__(self, cdim):
        self.parent = self
        self.producers, self.consumers, self.channelwise = [], [], []
        self.blocked = False
        self.cdim = cdim  # "last" (Linear) or 1 (conv)
        self.why = ""

    def find(self):
        s = self
        while s.parent is not s:
            s.parent = s.parent.parent
            s = s.parent
        return s


def _union(a, b):
    a, b = a.find(), b.find()
    if a is b:
        return a
    b.parent = a
    a.producers += b.producers
    a.consumers += b.consumers
    a.channelwise += b.channelwise
    if a.cdim != b.cdim:
        a.blocked, a.why = True, "channel dims differ"
    if b.blocked:
        a.blocked, a.why = True, b.why
    return a


def _block(space, why):
    s = space.find()
    if not s.blocked:
        s.blocked, s.why = True, why


class Permutation:
    """Class-level configuration + entry points, mirroring the reference's classmethod API."""
    __model = None
    __sparse_parameters = []
    __all_parameters = []
    __optimizer = None
    __save_permutation_graph = False
    __permutation_output_dir = "."
    __search_options = None
    __seed = 1

    @classmethod
    def set_permutation_params_from_asp(cls, model, sparse_parameters, all_parameters, optimizer=None):
        cls.__model = model
        cls.__sparse_parameters = sparse_parameters
        cls.__all_parameters = all_parameters
        cls.__optimizer = optimizer

    @classmethod
    def set_optimizer(cls, optimizer):
        cls.__optimizer = optimizer

    @classmethod
    def set_identical_seed(cls, identical_seed=1):
        cls.__seed = identical_seed
        torch.manual_seed(identical_seed)

    @classmethod
    def set_permutation_saving_params(cls, allow_permutation=False, save_permutation_graph=False,
                                      permutation_output_dir="."):
        cls.__save_permutation_graph = save_permutation_graph
        cls.__permutation_output_dir = permutation_output_dir

    @classmethod
    def set_search_options(cls, options):
        """Options for ``accelerated_search_for_good_permutation`` (strategy, escape_attempts, ...)."""
        cls.__search_options = dict(options) if options else None

    # ------------------------------------------------------------------ graph
    @classmethod
    def build_offline_permutation_graph(cls, model, dump_fx_graph=False,
                                        save_dumped_fx_graph="./model_offline_permutation_graph.json"):
        """Returns (groups, success). ``groups``: list of dicts with producers / consumers /
        channelwise module names, channel count and the reason a group is not permutable."""
        try:
            gm = torch.fx.symbolic_trace(model)
        except Exception as e:  # noqa: BLE001 - untraceable models are simply not permuted
            _log.warning("[permutation] torch.fx could not trace the model (%s); skipping permutation", e)
            return None, False
        modules = dict(gm.named_modules())
        calls = {}
        for n in gm.graph.nodes:
            if n.op == "call_module":
                calls[n.target] = calls.get(n.target, 0) + 1
        space_of = {}
        all_spaces = []

        def new_space(cdim):
            s = _Space(cdim)
            all_spaces.append(s)
            return s

        def in_space(arg):
            return space_of.get(arg) if isinstance(arg, torch.fx.Node) else None

        def block_args(n, why):
            for a in n.all_input_nodes:
                s = space_of.get(a)
                if s is not None:
                    _block(s, why)

        for n in gm.graph.nodes:
            if n.op == "placeholder":
                s = new_space(None)
                _block(s, "graph input")
                space_of[n] = s
            elif n.op == "get_attr":
                s = new_space(None)
                _block(s, f"parameter {n.target} used in the graph")
                space_of[n] = s
            elif n.op == "output":
                block_args(n, "reaches the model output")
            elif n.op == "call_module":
                mod = modules[n.target]
                src = in_space(n.args[0]) if n.args else None
                shared = calls[n.target] > 1
                if isinstance(mod, _LAYERS) and not _is_depthwise(mod):
                    grouped = isinstance(mod, _CONV) and mod.groups != 1
                    if src is not None:
                        s = src.find()
                        s.consumers.append(n.target)
                        if grouped or shared:
                            _block(s, f"{n.target} is grouped or shared")
                    out = new_space(1 if isinstance(mod, _CONV) else "last")
                    out.producers.append(n.target)
                    if grouped or shared:
                        _block(out, f"{n.target} is grouped or shared")
                    space_of[n] = out
                elif isinstance(mod, _BN) or _is_depthwise(mod) or isinstance(mod, torch.nn.LayerNorm) or \
                        isinstance(mod, _TRANSPARENT_MODULES):
                    if src is None:
                        space_of[n] = new_space(None)
                        _block(space_of[n], f"{n.target} input unknown")
                        continue
                    s = src.find()
                    if isinstance(mod, torch.nn.LayerNorm) and (len(mod.normalized_shape) != 1 or s.cdim != "last"):
                        _block(s, f"{n.target} normalises over more than the channel dim")
                    if isinstance(mod, _BN) and s.cdim != 1 and not isinstance(mod, torch.nn.BatchNorm1d):
                        _block(s, f"{n.target} channel dim mismatch")
                    if isinstance(mod, _BN) or _is_depthwise(mod) or isinstance(mod, torch.nn.LayerNorm):
                        s.channelwise.append(n.target)
                        if shared:
                            _block(s, f"{n.target} is shared")
                    space_of[n] = s
                else:
                    block_args(n, f"unsupported module {type(mod).__name__} ({n.target})")
                    space_of[n] = new_space(None)
                    _block(space_of[n], f"output of {n.target}")
            else:  # call_function / call_method
                tgt = n.target
                unary = (n.op == "call_function" and tgt in _UNARY_FUNCS) or \
                        (n.op == "call_method" and tgt in _UNARY_METHODS)
                binary = (n.op == "call_function" and tgt in _BINARY_FUNCS) or \
                         (n.op == "call_method" and tgt in _BINARY_METHODS)
                tensor_args = [a for a in n.args if isinstance(a, torch.fx.Node)]
                if unary and tensor_args and in_space(n.args[0]) is not None and len(tensor_args) == 1:
                    space_of[n] = in_space(n.args[0]).find()
                elif binary and tensor_args and all(in_space(a) is not None for a in tensor_args) and \
                        len(tensor_args) <= 2 and isinstance(n.args[0], torch.fx.Node):
                    s = in_space(tensor_args[0])
                    for a in tensor_args[1:]:
                        s = _union(s, in_space(a))
                    space_of[n] = s.find()
                else:
                    block_args(n, f"unsupported op {getattr(tgt, '__name__', tgt)}")
                    space_of[n] = new_space(None)
                    _block(space_of[n], f"output of {getattr(tgt, '__name__', tgt)}")

        roots = []
        for s in all_spaces:
            r = s.find()
            if r not in roots:
                roots.append(r)
        groups = []
        for r in roots:
            if not r.consumers and not r.producers:
                continue
            groups.append({
                "producers": list(dict.fromkeys(r.producers)),
                "consumers": list(dict.fromkeys(r.consumers)),
                "channelwise": list(dict.fromkeys(r.channelwise)),
                "permutable": (not r.blocked) and bool(r.producers) and bool(r.consumers),
                "reason": r.why if r.blocked else ("" if r.producers and r.consumers else "no producer/consumer"),
            })
        if dump_fx_graph:
            cls.save_graph_to_json(groups, save_dumped_fx_graph)
        return groups, True

    # ------------------------------------------------------------------ search + apply
    @classmethod
    def _sparse_weight(cls, name):
        for module_name, module, p_name, p, mask, pruned in cls.__sparse_parameters:
            if module_name == name and p_name == "weight":
                return p
        return None

    @classmethod
    def search_for_good_permutation(cls, model, groups):
        modules = dict(model.named_modules())
        for g in groups:
            g["permutation_sequence"] = None
            if not g["permutable"]:
                continue
            mats = []
            for c in g["consumers"]:
                w = cls._sparse_weight(c)
                if w is None:
                    continue
                w = w.detach().float()
                if w.dim() == 2:
                    mats.append(w)
                else:  # conv [K, C, *k] -> [prod(k) * K, C]
                    mats.append(w.permute(*range(2, w.dim()), 0, 1).reshape(-1, w.shape[1]))
            if not mats:
                g["permutable"], g["reason"] = False, "no sparse consumer"
                continue
            C = mats[0].shape[1]
            if any(m.shape[1] != C for m in mats) or C % 4 != 0:
                g["permutable"], g["reason"] = False, "channel count mismatch"
                continue
            matrix = torch.cat(mats, dim=0).contiguous()
            before = sum_after_2_to_4(matrix)
            total = float(matrix.abs().sum())
            if total == 0 or abs(total - before) / total < 1e-3:
                g["permutation_sequence"] = list(range(C))
                continue
            opts = dict(cls.__search_options or {})
            if not matrix.is_cuda:
                opts.setdefault("escape_attempts", 10)
            if "strategy" not in opts and C > 2048:
                opts.update(strategy="progressive channel swap", progressive_search_time_limit=120)
            perm = accelerated_search_for_good_permutation(matrix, opts)
            perm = cls._broadcast_perm(perm, matrix.device)
            after = sum_after_2_to_4(matrix[:, torch.tensor(perm, device=matrix.device)])
            g["permutation_sequence"] = perm
            g["kept_magnitude_before"], g["kept_magnitude_after"] = before, after
            _log.info("[permutation] %s: kept 2:4 magnitude %.6g -> %.6g", g["consumers"], before, after)
        return groups

    @staticmethod
    def _broadcast_perm(perm, device):
        dist = torch.distributed
        if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
            return perm
        dev = device if dist.get_backend() != "gloo" else torch.device("cpu")
        t = torch.tensor(perm, dtype=torch.int64, device=dev)
        dist.broadcast(t, 0)
        return [int(v) for v in t.cpu()]

    @classmethod
    def _permute_param(cls, p, idx, dim):
        with torch.no_grad():
            p.data.copy_(p.data.index_select(dim, idx.to(p.device)))
        opt = cls.__optimizer
        if opt is not None and p in opt.state:
            for v in opt.state[p].values():
                if torch.is_tensor(v) and v.shape == p.shape:
                    v.copy_(v.index_select(dim, idx.to(v.device)))

    @classmethod
    def apply_offline_permutation(cls, model, fx_graph):
        """Apply every searched permutation (C dim of consumers, K dim of producers, channel-wise
        parameters). Returns the number of permuted groups."""
        modules = dict(model.named_modules())
        done = 0
        for g in fx_graph:
            perm = g.get("permutation_sequence")
            if not g.get("permutable") or perm is None or perm == list(range(len(perm))):
                continue
            idx = torch.tensor(perm, dtype=torch.long)
            for name in g["consumers"]:
                mod = modules[name]
                cls._permute_param(mod.weight, idx, 1)
                for bname, buf in list(mod.named_buffers(recurse=False)):
                    if buf.shape == mod.weight.shape:  # ASP mask / pruned-value buffers
                        buf.copy_(buf.index_select(1, idx.to(buf.device)))
            for name in g["producers"]:
                mod = modules[name]
                cls._permute_param(mod.weight, idx, 0)
                if mod.bias is not None:
                    cls._permute_param(mod.bias, idx, 0)
                for bname, buf in list(mod.named_buffers(recurse=False)):
                    if buf.shape == mod.weight.shape:
                        buf.copy_(buf.index_select(0, idx.to(buf.device)))
            for name in g["channelwise"]:
                mod = modules[name]
                for p in (getattr(mod, "weight", None), getattr(mod, "bias", None)):
                    if p is not None:
                        cls._permute_param(p, idx, 0)
                for bname in ("running_mean", "running_var"):
                    buf = getattr(mod, bname, None)
                    if buf is not None:
                        buf.copy_(buf.index_select(0, idx.to(buf.device)))
            done += 1
        return done

    @classmethod
    def permute_model(cls, model):
        """Build the graph, search and apply. Returns the group list (or None if untraceable)."""
        groups, ok = cls.build_offline_permutation_graph(
            model, cls.__save_permutation_graph,
            os.path.join(cls.__permutation_output_dir, "model_offline_permutation_graph.json"))
        if not ok:
            return None
        groups = cls.search_for_good_permutation(model, groups)
        cls.apply_offline_permutation(model, groups)
        if cls.__save_permutation_graph:
            cls.save_graph_to_json(groups, os.path.join(cls.__permutation_output_dir,
                                                        "model_graph_permutation_applied.json"))
        return groups

    @staticmethod
    def save_graph_to_json(graph, save_dumped_graph_path_with_name="./model_fx_graph.json"):
        d = os.path.dirname(os.path.abspath(save_dumped_graph_path_with_name))
        os.makedirs(d, exist_ok=True)
        with open(save_dumped_graph_path_with_name, "w") as f:
            json.dump(graph, f, indent=1, default=str)
