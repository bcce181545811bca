"""Hook runtime with TransformerLens semantics, built natively (no TL dependency).

The reference outsources this layer to TransformerLens (call
sites ``/root/reference/iit/model_pairs/base_model_pair.py:80-98``,
``/root/reference/iit/model_pairs/stop_grad_pair.py:80-100``).  Contract kept:

* ``HookPoint`` is an identity module; ``add_hook(fn, dir)`` registers
  ``fn(activation, hook=HookPoint)`` which may return a replacement.  Backward
  hooks receive the gradient flowing into the hook's output and may return a
  replacement (a tensor or a 1-element list/tuple, TL style).
* ``HookedRootModule.setup()`` names every ``HookPoint`` by its module path and
  builds ``hook_dict`` / ``mod_dict``.
* ``run_with_hooks(..., fwd_hooks, bwd_hooks, reset_hooks_end)`` and
  ``run_with_cache(...)`` (cache holds ``act.detach()``).
* Hooks installed with ``reset_hooks_end=False`` persist (reference quirk Q7).

Unlike TL, a ``HookPoint`` with no hooks costs one attribute test (``__call__``
is short-circuited), so the hot path of the native engine never pays module-call
overhead for the ~20 hook sites per block.  Models can also ask
``hook_point.is_live`` to decide whether an intermediate must be materialised at
all (fused HIP kernels skip materialising hook sites nobody listens to).
"""
from __future__ import annotations

import contextlib
import itertools
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple, Union

import torch
from torch import nn

HookFn = Callable[..., Optional[torch.Tensor]]
NameOrFilter = Union[str, Callable[[str], bool]]


class _HookEntry:
    __slots__ = ("fn", "permanent", "level", "alive", "uid")
    _uids = itertools.count()

    def __init__(self, fn: HookFn, permanent: bool, level: Optional[int]):
        self.fn = fn
        self.permanent = permanent
        self.level = level
        self.alive = True
        self.uid = next(self._uids)


class HookPoint(nn.Module):
    """Identity module that exposes an activation to user hooks."""

    def __init__(self):
        super().__init__()
        self.name: Optional[str] = None
        self.fwd_hooks: List[_HookEntry] = []
        self.bwd_hooks: List[_HookEntry] = []
        self.ctx: dict = {}

    # -- registration ---------------------------------------------------------
    def add_hook(self, hook: HookFn, dir: str = "fwd", is_permanent: bool = False,
                 level: Optional[int] = None, prepend: bool = False) -> _HookEntry:
        if dir not in ("fwd", "bwd"):
            raise ValueError(f"Invalid direction {dir}")
        entry = _HookEntry(hook, is_permanent, level)
        lst = self.fwd_hooks if dir == "fwd" else self.bwd_hooks
        if prepend:
            lst.insert(0, entry)
        else:
            lst.append(entry)
        return entry

    def remove_hooks(self, dir: str = "fwd", including_permanent: bool = False,
                     level: Optional[int] = None) -> None:
        dirs = ("fwd", "bwd") if dir == "both" else (dir,)
        for d in dirs:
            lst = self.fwd_hooks if d == "fwd" else self.bwd_hooks
            keep = []
            for e in lst:
                drop = (including_permanent or not e.permanent) and (level is None or e.level == level)
                if drop:
                    e.alive = False
                else:
                    keep.append(e)
            lst[:] = keep

    def clear_context(self):
        self.ctx.clear()

    @property
    def is_live(self) -> bool:
        return bool(self.fwd_hooks or self.bwd_hooks or self._forward_hooks or self._forward_pre_hooks)

    # -- execution ------------------------------------------------------------
    def __call__(self, x, *args, **kwargs):
        if not (self.fwd_hooks or self.bwd_hooks or self._forward_hooks or self._forward_pre_hooks
                or self._backward_hooks):
            return x
        return super().__call__(x, *args, **kwargs)

    def forward(self, x):
        for e in list(self.fwd_hooks):
            if not e.alive:
                continue
            out = e.fn(x, hook=self)
            if out is not None:
                x = out
        if self.bwd_hooks and isinstance(x, torch.Tensor) and x.requires_grad:
            entries = list(self.bwd_hooks)

            def _grad_hook(grad, _entries=entries, _hp=self):
                for e in _entries:
                    if not e.alive:
                        continue
                    out = e.fn(grad, hook=_hp)
                    if isinstance(out, (list, tuple)):
                        out = out[0]
                    if out is not None:
                        grad = out
                return grad

            x = x.view_as(x)  # fresh autograd node so the hook only sees this site's grad
            x.register_hook(_grad_hook)
        return x

    def extra_repr(self) -> str:
        return f"name={self.name!r}"


class ActivationCache:
    """Dict-like activation cache (subset of ``transformer_lens.ActivationCache``)."""

    def __init__(self, cache_dict: Dict[str, torch.Tensor], model=None, has_batch_dim: bool = True):
        self.cache_dict = cache_dict
        self.model = model
        self.has_batch_dim = has_batch_dim

    def _key(self, key):
        if isinstance(key, tuple):
            return get_act_name(*key)
        return key

    def __getitem__(self, key) -> torch.Tensor:
        key = self._key(key)
        if key in self.cache_dict:
            return self.cache_dict[key]
        if isinstance(key, str) and key not in self.cache_dict:
            alias = get_act_name(key) if "." not in key else key
            if alias in self.cache_dict:
                return self.cache_dict[alias]
        raise KeyError(key)

    def __setitem__(self, key, value):
        self.cache_dict[self._key(key)] = value

    def __contains__(self, key) -> bool:
        return self._key(key) in self.cache_dict

    def __len__(self) -> int:
        return len(self.cache_dict)

    def __iter__(self):
        return iter(self.cache_dict)

    def keys(self):
        return self.cache_dict.keys()

    def values(self):
        return self.cache_dict.values()

    def items(self):
        return self.cache_dict.items()

    def get(self, key, default=None):
        try:
            return self[key]
        except KeyError:
            return default

    def to(self, device) -> "ActivationCache":
        self.cache_dict = {k: v.to(device) for k, v in self.cache_dict.items()}
        return self

    def remove_batch_dim(self) -> "ActivationCache":
        if self.has_batch_dim:
            for k, v in self.cache_dict.items():
                if v.shape[0] != 1:
                    raise AssertionError(f"cannot remove batch dim of {k} with shape {tuple(v.shape)}")
                self.cache_dict[k] = v[0]
            self.has_batch_dim = False
        return self

    def __repr__(self) -> str:
        return f"ActivationCache({list(self.cache_dict.keys())})"


_ACT_ALIASES = {
    "embed": "hook_embed", "pos_embed": "hook_pos_embed",
    "resid_pre": "hook_resid_pre", "resid_mid": "hook_resid_mid", "resid_post": "hook_resid_post",
    "attn_out": "hook_attn_out", "mlp_out": "hook_mlp_out",
    "q": "attn.hook_q", "k": "attn.hook_k", "v": "attn.hook_v", "z": "attn.hook_z",
    "result": "attn.hook_result", "attn_scores": "attn.hook_attn_scores", "pattern": "attn.hook_pattern",
    "attn": "attn.hook_pattern", "pre": "mlp.hook_pre", "post": "mlp.hook_post",
    "scale": "ln1.hook_scale", "normalized": "ln1.hook_normalized",
}


def get_act_name(name: str, layer: Optional[int] = None, layer_type: Optional[str] = None) -> str:
    """TL-style shorthand: ``get_act_name("z", 3) -> "blocks.3.attn.hook_z"``."""
    if "." in name or name.startswith("hook_") and layer is None:
        return name
    full = _ACT_ALIASES.get(name, name)
    if layer is None:
        return full if full.startswith("hook_") else full
    if layer_type is not None and name in ("scale", "normalized"):
        full = f"{layer_type}.hook_{name}"
    return f"blocks.{layer}.{full}"


class HookedRootModule(nn.Module):
    """Root module that owns and drives ``HookPoint`` children."""

    def __init__(self, *args, **kwargs):
        super().__init__()
        self.is_caching = False
        self.context_level = 0

    def setup(self) -> None:
        self.mod_dict: Dict[str, nn.Module] = {}
        self.hook_dict: Dict[str, HookPoint] = {}
        for name, module in self.named_modules():
            if name == "":
                continue
            module.name = name
            self.mod_dict[name] = module
            if isinstance(module, HookPoint):
                self.hook_dict[name] = module

    def hook_points(self) -> Iterable[HookPoint]:
        return self.hook_dict.values()

    # -- hook management ------------------------------------------------------
    def _resolve(self, name: NameOrFilter) -> List[HookPoint]:
        if isinstance(name, str):
            if name not in self.hook_dict:
                raise KeyError(f"hook {name!r} not found in {type(self).__name__}")
            return [self.hook_dict[name]]
        return [hp for n, hp in self.hook_dict.items() if name(n)]

    def add_hook(self, name: NameOrFilter, hook: HookFn, dir: str = "fwd", is_permanent: bool = False,
                 level: Optional[int] = None, prepend: bool = False) -> None:
        for hp in self._resolve(name):
            hp.add_hook(hook, dir=dir, is_permanent=is_permanent, level=level, prepend=prepend)

    def add_perma_hook(self, name: NameOrFilter, hook: HookFn, dir: str = "fwd") -> None:
        self.add_hook(name, hook, dir=dir, is_permanent=True)

    def reset_hooks(self, clear_contexts: bool = True, direction: str = "both",
                    including_permanent: bool = False, level: Optional[int] = None) -> None:
        for hp in self.hook_dict.values():
            hp.remove_hooks(direction, including_permanent=including_permanent, level=level)
            if clear_contexts:
                hp.clear_context()
        self.is_caching = False

    def clear_contexts(self) -> None:
        for hp in self.hook_dict.values():
            hp.clear_context()

    @contextlib.contextmanager
    def hooks(self, fwd_hooks: Sequence[Tuple[NameOrFilter, HookFn]] = (),
              bwd_hooks: Sequence[Tuple[NameOrFilter, HookFn]] = (),
              reset_hooks_end: bool = True, clear_contexts: bool = False):
        self.context_level += 1
        level = self.context_level
        try:
            for name, fn in fwd_hooks:
                self.add_hook(name, fn, dir="fwd", level=level)
            for name, fn in bwd_hooks:
                self.add_hook(name, fn, dir="bwd", level=level)
            yield self
        finally:
            if reset_hooks_end:
                self.reset_hooks(clear_contexts, including_permanent=False, level=level)
            self.context_level -= 1

    def run_with_hooks(self, *model_args, fwd_hooks: Sequence = (), bwd_hooks: Sequence = (),
                       reset_hooks_end: bool = True, clear_contexts: bool = False, **model_kwargs):
        if bwd_hooks and reset_hooks_end:
            # TL semantics: backward hooks are removed before any backward pass can run.
            pass
        with self.hooks(fwd_hooks, bwd_hooks, reset_hooks_end, clear_contexts):
            return self(*model_args, **model_kwargs)

    # -- caching --------------------------------------------------------------
    def get_caching_hooks(self, names_filter=None, incl_bwd: bool = False, device=None,
                          remove_batch_dim: bool = False, cache: Optional[dict] = None):
        cache = {} if cache is None else cache
        if names_filter is None:
            names_filter = lambda n: True  # noqa: E731
        elif isinstance(names_filter, str):
            single = names_filter
            names_filter = lambda n: n == single  # noqa: E731
        elif isinstance(names_filter, (list, tuple, set)):
            allowed = set(names_filter)
            names_filter = lambda n: n in allowed  # noqa: E731

        def save(tensor, hook, suffix=""):
            t = tensor.detach()
            if device is not None:
                t = t.to(device)
            cache[hook.name + suffix] = t[0] if remove_batch_dim else t

        fwd = [(n, save) for n in self.hook_dict if names_filter(n)]
        bwd = [(n, lambda g, hook: save(g, hook, "_grad")) for n in self.hook_dict if names_filter(n)] if incl_bwd else []
        return cache, fwd, bwd

    def run_with_cache(self, *model_args, names_filter=None, device=None, remove_batch_dim: bool = False,
                       incl_bwd: bool = False, reset_hooks_end: bool = True, clear_contexts: bool = False,
                       return_cache_object: bool = True, **model_kwargs):
        cache, fwd, bwd = self.get_caching_hooks(names_filter, incl_bwd, device, remove_batch_dim)
        with self.hooks(fwd, bwd, reset_hooks_end=reset_hooks_end, clear_contexts=clear_contexts):
            out = self(*model_args, **model_kwargs)
        if return_cache_object:
            return out, ActivationCache(cache, self, has_batch_dim=not remove_batch_dim)
        return out, cache

    def cache_all(self, cache: dict, incl_bwd: bool = False, device=None, remove_batch_dim: bool = False):
        _, fwd, bwd = self.get_caching_hooks(None, incl_bwd, device, remove_batch_dim, cache=cache)
        for n, fn in fwd:
            self.add_hook(n, fn, "fwd")
        for n, fn in bwd:
            self.add_hook(n, fn, "bwd")

    def cache_some(self, cache: dict, names: Callable[[str], bool], incl_bwd: bool = False, device=None,
                   remove_batch_dim: bool = False):
        _, fwd, bwd = self.get_caching_hooks(names, incl_bwd, device, remove_batch_dim, cache=cache)
        for n, fn in fwd:
            self.add_hook(n, fn, "fwd")
        for n, fn in bwd:
            self.add_hook(n, fn, "bwd")
