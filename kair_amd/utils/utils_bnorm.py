"""BatchNorm folding for DnCNN (restatement of /root/reference/utils/utils_bnorm.py:20-91).

merge_bn        utils_bnorm.py:32-63  fold every Conv/Linear/ConvTranspose + following BatchNorm into
                the conv (w <- w * gamma / sqrt(var + eps), b <- (b - mean) * gamma / sqrt(var + eps) +
                beta), using the RUNNING statistics, and delete the BN module
tidy_sequential utils_bnorm.py:84-91  unwrap one-element Sequentials left behind
deleteLayer     utils_bnorm.py:20-26
add_bn          utils_bnorm.py:69-78

Called by ModelBase.merge_bnorm_train / merge_bnorm_test (model_base.py:264-275) at
opt['merge_bn_startpoint'] (main_train_dncnn.py:139-141, 179-182).  The DnCNN step program is
rebuilt from the merged module list on the next forward (network_dncnn.DnCNN.invalidate_engine).
"""
import torch
import torch.nn as nn

_PREV = (nn.Conv2d, nn.Linear, nn.ConvTranspose2d)


def deleteLayer(model, layer_type=nn.BatchNorm2d):
    for name, child in list(model.named_children()):
        if isinstance(child, layer_type):
            del model._modules[name]
        deleteLayer(child, layer_type)


@torch.no_grad()
def merge_bn(model):
    prev = None
    for name, m in list(model.named_children()):
        if isinstance(m, (nn.BatchNorm2d, nn.BatchNorm1d)) and isinstance(prev, _PREV):
            w = prev.weight.data
            if prev.bias is None:
                prev.bias = nn.Parameter(torch.zeros(prev.out_channels, dtype=w.dtype, device=w.device))
            b = prev.bias.data
            invstd = (m.running_var + m.eps).pow(-0.5)
            # ConvTranspose2d weights are [Cin, Cout, kh, kw]: the output channel is dim 1
            shape = (1, -1, 1, 1) if isinstance(prev, nn.ConvTranspose2d) else (-1,) + (1,) * (w.dim() - 1)
            w.mul_(invstd.view(shape))
            b.sub_(m.running_mean).mul_(invstd)
            if m.affine:
                w.mul_(m.weight.data.view(shape))
                b.mul_(m.weight.data).add_(m.bias.data)
            del model._modules[name]
        prev = m
        merge_bn(m)
    if hasattr(model, "invalidate_engine"):
        model.invalidate_engine()


def add_bn(model):
    for name, m in list(model.named_children()):
        if isinstance(m, _PREV):
            bn = nn.BatchNorm2d(m.out_channels, momentum=0.1, affine=True)
            bn.weight.data.fill_(1)
            model._modules[name] = nn.Sequential(m, bn)
        add_bn(m)


def tidy_sequential(model):
    for name, m in list(model.named_children()):
        if isinstance(m, nn.Sequential) and len(m) == 1:
            model._modules[name] = m[0]
        tidy_sequential(m)
    if hasattr(model, "invalidate_engine"):
        model.invalidate_engine()
