"""Give any ``nn.Module`` TL-style hook points (parity: ``/root/reference/iit/utils/wrapper.py:6-70``).

``HookedModuleWrapper(mod, name, recursive=True, hook_self=False)`` wraps every
child (ModuleLists element-wise) so that each child's output passes through a
``HookPoint``; hook names look like ``mod.layer3.mod.1.mod.conv2.hook_point``
exactly as in the reference (``/root/reference/iit/tasks/task_loader.py:41``).

Like the hooked transformer, a top-level wrapper executes :class:`iit_amd.engine.plan.RunPlan`s natively
(``supports_run_plan``): ``run_capture(x, names)`` stores only the named hook activations and stops the forward after
the last one (the reference's ``run_with_cache`` stores all of the ResNet's ~60 submodule outputs), and
``forward(x, plan=...)`` splices the source activations in at the planned sites -- on the GPU as one launch of the
patch-spec splice kernel per site (channel / spatial quadrants of a conv output: ``csrc/splice.hip``), whose
backward zeroes the spliced gradient.  Only the one or two planned sites run any Python per forward; every other
hook point is a no-op pass-through.
"""
from __future__ import annotations

import torch
from torch import nn

from .hook_points import HookedRootModule, HookPoint

_TUPLE_RETURNING = ("intermediate_value_head", "value_head")


class _StopForward(Exception):
    pass


# the RunPlan of the plan-driven forward in progress (None outside one): lets a module that fuses a hooked site's
# consumer into one kernel (iit_amd.models.resnet: a conv hook's splice read by the fused BatchNorm) take the site
# over instead of running the hook
_ACTIVE_PLAN = []


def active_plan():
    return _ACTIVE_PLAN[-1] if _ACTIVE_PLAN else None


class HookedModuleWrapper(HookedRootModule):
    def __init__(self, mod: nn.Module, name: str = "model", recursive: bool = False, hook_self: bool = True,
                 top_level: bool = True, hook_pre: bool = False):
        super().__init__()
        self.mod = mod
        self.hook_self = hook_self
        self.hook_pre = None
        if hook_pre:
            self.hook_pre = HookPoint()
            self.hook_pre.name = name + "pre"
        if hook_self:
            self.hook_point = HookPoint()
            self.hook_point.name = name
        if recursive:
            self.wrap_hookpoints_recursively()
        self.setup()

    def wrap_hookpoints_recursively(self, verbose: bool = False) -> None:
        for key, child in list(self.mod._modules.items()):
            if child is None or isinstance(child, HookedModuleWrapper) or key in _TUPLE_RETURNING:
                continue
            if isinstance(child, nn.ModuleList):
                for i, sub in enumerate(child):
                    child[i] = HookedModuleWrapper(sub, name=f"{key}.{i}", recursive=True, top_level=False)
                continue
            setattr(self.mod, key, HookedModuleWrapper(child, name=key, recursive=True, top_level=False))

    supports_run_plan = True

    def forward(self, *args, plan=None, **kwargs):
        if plan is not None:
            return self._planned_forward(plan, *args, **kwargs)
        if self.hook_pre is not None:
            args = (self.hook_pre(args[0]),) + tuple(args[1:])
        out = self.mod(*args, **kwargs)
        if not self.hook_self:
            return out
        if not isinstance(out, torch.Tensor):
            raise TypeError(f"wrapped module returned {type(out)}, expected Tensor")
        return self.hook_point(out)


    # ------------------------------------------------------------------ plan-driven execution
    def _planned_forward(self, plan, *args, **kwargs):
        from ..engine.plan import scale_site, zero_grad_site
        names = [n for n in self.hook_dict if plan.touches(n)]
        remaining = set(plan.capture) if (plan.logits == "none" and plan.truncate and plan.capture) else None

        def site(name):
            def fn(act, hook):
                out = act
                for spl in plan.splice.get(name, ()):
                    out = spl.apply(out)
                if name in plan.scale:
                    out = scale_site(out, plan.scale[name])
                if name in plan.zero_grad and out.requires_grad:
                    out = zero_grad_site(out, plan.zero_grad[name])
                if name in plan.capture:
                    plan.cache[name] = out.detach()
                    if remaining is not None:
                        remaining.discard(name)
                        if not remaining:
                            raise _StopForward()
                return out
            return fn

        entries = [(self.hook_dict[n], self.hook_dict[n].add_hook(site(n))) for n in names]
        _ACTIVE_PLAN.append(plan)
        try:
            out = self.forward(*args, **kwargs)
        except _StopForward:
            return None
        finally:
            _ACTIVE_PLAN.pop()
            for hp, e in entries:
                e.alive = False
                if e in hp.fwd_hooks:
                    hp.fwd_hooks.remove(e)
        if plan.logits == "none":
            return None
        if plan.logits == "last" and out.dim() == 3:
            return out[:, -1]
        if plan.logits == "argmax":
            return out.argmax(dim=-1)
        return out

    def run_capture(self, x, names, truncate: bool = True, base_plan=None):
        """Source run of an interchange intervention: no grad, capture ``names`` only, stop after the last."""
        from ..engine.plan import RunPlan
        plan = RunPlan.capture_only(list(names), truncate=truncate)
        if base_plan is not None:
            plan = base_plan.merged(plan)
        with torch.no_grad():
            self.forward(x, plan=plan)
        return plan.cache


def get_hook_points(model: HookedRootModule):
    """Conv hook points of a wrapped CNN (parity: ``wrapper.py:69-70``)."""
    return [k for k in model.hook_dict.keys() if "conv" in k]
