"""ResNet-18 with torchvision's module names, shapes and init (the PVR LL model).

The reference uses ``torchvision.models.resnet18()`` with ``fc -> Linear(512, 10)``
wrapped by ``HookedModuleWrapper(recursive=True, hook_self=False)``
(``/root/reference/iit/tasks/mnist_pvr/get_alignment.py:10-15``).  torchvision is
not part of this stack, so this is a self-contained network with the identical
parameter/buffer names (``conv1``, ``bn1``, ``layer{1..4}.{0,1}.conv{1,2}``,
``...downsample.{0,1}``, ``fc``) -- state_dicts are interchangeable -- and hook
names like ``mod.layer3.mod.1.mod.conv2.hook_point`` after wrapping.

Convolutions run through PyTorch-ROCm (MIOpen); pass ``memory_format=torch.channels_last`` to :func:`resnet18`
for the NHWC layout MIOpen's MFMA convolution kernels prefer on gfx950.  On channels-last bf16 activations (the
bf16 PVR step: channels-last autocast) every ``BatchNorm -> ReLU`` and ``BatchNorm -> + identity -> ReLU`` chain
runs as one fused HIP op (:mod:`iit_amd.ops.bn`, ``csrc/bn_nhwc.hip``) unless a hook on one of its sites is live;
other inputs take the module path.
"""
from __future__ import annotations

import os

import torch
from torch import nn


class Conv2d(nn.Conv2d):
    """``nn.Conv2d`` (same parameters, state_dict keys and init) that, under bf16 autocast on the GPU with its weight
    in a flat parameter arena, convolves with the arena's bf16 mirror (``torch_ops._MirrorWeight``, written by the
    fused Adam): no per-forward weight cast (autocast's weight cache is off in graph-captured steps), and the bf16
    weight gradient is added straight into the fp32 grad slot instead of a cast + AccumulateGrad add.
    ``IIT_CONV_MIRROR=0`` keeps the plain autocast path."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        w = self.weight
        if (x.is_cuda and self.bias is None and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16 and w.dtype == torch.float32
                and getattr(w, "_iit_flat", None) is not None and os.environ.get("IIT_CONV_MIRROR", "1") != "0"):
            from ..ops.torch_ops import _MirrorWeight, _arena_mirror
            m = _arena_mirror(w)
            if m is not None:
                from ..ops import conv as hconv
                if hconv.covered(x, self):  # 3x3 / 1x1, stride 1 / 2: the repo's implicit-GEMM kernels where they win
                    return hconv.conv(x, w, m[0], hconv.geometry(self))
                w16 = _MirrorWeight.apply(w, m[0]) if torch.is_grad_enabled() else m[1]
                return self._conv_forward(x.to(torch.bfloat16), w16, None)
        return super().forward(x)


def conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return Conv2d(cin, cout, kernel_size=3, stride=stride, padding=1, bias=False)


def conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return Conv2d(cin, cout, kernel_size=1, stride=stride, bias=False)


def _hooked(m: nn.Module) -> bool:
    """A live hook on a (possibly HookedModuleWrapper-wrapped) module's output or input."""
    hp, pre = getattr(m, "hook_point", None), getattr(m, "hook_pre", None)
    return (hp is not None and hp.is_live) or (pre is not None and pre.is_live)


def fused_bn_act(bn_m: nn.Module, relu_m, x: torch.Tensor, res: torch.Tensor = None, splice=None):
    """``relu(bn(x) (+ res))`` as one fused op when covered (:mod:`iit_amd.ops.bn`), else None; ``relu_m`` None =
    no activation; ``splice`` = (index, src) of the producing conv's hook, applied as the kernels read x.
    ``bn_m`` / ``relu_m`` may be HookedModuleWrapper-wrapped: a live hook on either refuses."""
    if not x.is_cuda or x.dtype not in (torch.bfloat16, torch.float32) or _hooked(bn_m) or \
            (relu_m is not None and _hooked(relu_m)):
        return None
    from ..ops import bn as fbn
    bn = getattr(bn_m, "mod", bn_m)
    if not isinstance(bn, nn.BatchNorm2d) or not fbn.enabled() or not fbn.covered(x, bn, res):
        return None
    return fbn.bn_act(x, bn, res, relu=relu_m is not None, splice=splice)


def _conv_with_splice(conv_m: nn.Module, bn_m: nn.Module, x: torch.Tensor):
    """(conv output, splice) where ``splice`` = (index, src) when the active plan's only business at the conv's hook
    is one interchange splice and the fused BatchNorm can take it over: the conv then runs without its hook and the
    splice is applied by the BatchNorm kernels' reads (no splice pass, csrc/bn_nhwc.hip); else (conv(x), None)."""
    hp = getattr(conv_m, "hook_point", None)
    if hp is None or not x.is_cuda or os.environ.get("IIT_BN_SPLICE", "1") == "0" or _hooked(bn_m):
        return conv_m(x), None
    from ..hooks.wrapper import active_plan
    plan = active_plan()
    name = hp.name
    spl = plan.splice.get(name) if plan is not None else None
    if not spl or len(spl) != 1 or spl[0].whole or name in plan.capture or name in plan.scale or \
            name in plan.zero_grad or len(hp.fwd_hooks) != 1 or hp.bwd_hooks or hp._forward_hooks or \
            hp._forward_pre_hooks or getattr(conv_m, "hook_pre", None) is not None:
        return conv_m(x), None
    h = conv_m.mod(x)  # the conv without its hook: the splice moves into the BatchNorm's reads
    if h.dtype not in (torch.bfloat16, torch.float32):
        return conv_m.hook_point(h), None
    return h, (spl[0].index, spl[0].src)


def _pool_covered(x: torch.Tensor, pool: nn.Module) -> bool:
    if not x.is_cuda:
        return False
    from ..ops import bn as fbn
    return fbn.maxpool_covered(x, pool)


def _bn_after_conv(conv_m, bn_m, relu_m, x, res=None):
    """relu?(bn(conv(x)) (+ res)) with the fused BatchNorm (and a conv-hook splice inside it) when covered, else the
    module path."""
    from ..ops import conv as hconv
    bn = getattr(bn_m, "mod", bn_m)
    # a training BatchNorm reading the conv's output unhooked: the conv's epilogue writes its statistics
    with hconv.stats_for_bn(isinstance(bn, nn.BatchNorm2d) and bn.training and not _hooked(bn_m)):
        h, splice = _conv_with_splice(conv_m, bn_m, x)
    out = fused_bn_act(bn_m, relu_m, h, res, splice=splice)
    if out is None:
        if splice is not None:  # the fused op could not take the splice: run the conv's hook after all
            h = conv_m.hook_point(h)
        out = bn_m(h)
        if res is not None:
            out = out + res
        if relu_m is not None:
            out = relu_m(out)
    return out


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module = None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        identity = x
        out = _bn_after_conv(self.conv1, self.bn1, self.relu, x)
        if self.downsample is not None:
            identity = None
            ds = getattr(self.downsample, "mod", self.downsample)  # Sequential(conv1x1, BatchNorm2d), maybe wrapped
            if not _hooked(self.downsample) and isinstance(ds, nn.Sequential) and len(ds) == 2:
                from ..ops import conv as hconv
                with hconv.stats_for_bn(isinstance(ds[1], nn.BatchNorm2d) and ds[1].training):
                    h = ds[0](x)
                identity = fused_bn_act(ds[1], None, h)
            if identity is None:
                identity = self.downsample(x)
        return _bn_after_conv(self.conv2, self.bn2, self.relu, out, identity)


class ResNet(nn.Module):
    def __init__(self, layers=(2, 2, 2, 2), num_classes: int = 1000, in_channels: int = 3):
        super().__init__()
        self.inplanes = 64
        self.conv1 = Conv2d(in_channels, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2)
        self.layer3 = self._make_layer(256, layers[2], stride=2)
        self.layer4 = self._make_layer(512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != planes:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes, stride), nn.BatchNorm2d(planes))
        layers = [BasicBlock(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes
        layers += [BasicBlock(planes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # a channels-last model gets channels-last activations from the first convolution on (an NCHW batch into
        # NHWC weights made every MIOpen convolution transpose its operands and kept the fused BN path off)
        conv = getattr(self.conv1, "mod", self.conv1)
        if x.dim() == 4 and conv.weight.is_contiguous(memory_format=torch.channels_last) and \
                not conv.weight.is_contiguous() and not x.is_contiguous(memory_format=torch.channels_last):
            x = x.contiguous(memory_format=torch.channels_last)
        x = _bn_after_conv(self.conv1, self.bn1, self.relu, x)
        pool = getattr(self.maxpool, "mod", self.maxpool)
        if not _hooked(self.maxpool) and _pool_covered(x, pool):
            from ..ops.bn import MaxPool3s2Fn
            x = MaxPool3s2Fn.apply(x)  # NHWC bf16, byte argmax, gather backward (csrc/bn_nhwc.hip)
        else:
            x = self.maxpool(x)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


def resnet18(num_classes: int = 1000, memory_format=None) -> ResNet:
    m = ResNet((2, 2, 2, 2), num_classes=num_classes)
    if memory_format is not None:
        m = m.to(memory_format=memory_format)
    return m
