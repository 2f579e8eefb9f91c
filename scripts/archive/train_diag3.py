"""Diagnostic: layer.6.0.bn1 pre-ReLU values, HIP vs fp64 oracle (golden case step 1): sign flips."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "video-seg-model-compress_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import torch
import torch.nn.functional as F
import train_case as TC
from oracle import drn_oracle as O
from drnmi.train import TrainRunner

g = TC.load()
m, pr = TC.model_and_masks(g)
xs, ts = TC.inputs(g)
x = xs[0]
sd = {k: (v.detach().clone().double() if v.is_floating_point() else v.clone()) for k, v in m.state_dict().items()}
O._TRAIN["on"] = True
_, stages = O.backbone(sd, "drn_d_22", x.double())
l5 = stages["layer5"]
y = F.conv2d(l5, sd["layer.6.0.conv1.weight"], padding=4, dilation=4)
pre = F.batch_norm(y, None, None, sd["layer.6.0.bn1.weight"], sd["layer.6.0.bn1.bias"], training=True, eps=1e-5)
O._TRAIN["on"] = False
mc = m.cuda().train()
r = TrainRunner(mc)
lp, logits, saved = r.forward(x.cuda(), save=True)
idx = [i for i, nd in enumerate(r.nodes) if nd.name == "layer.6.0.conv1"][0]
yh, mean, invstd = saved["nodes"][idx]
nd = r.nodes[idx]
yh = yh.double().cpu()
preh = (yh - mean.double().cpu()) * invstd.double().cpu() * nd.bn.weight.detach().double().cpu() + nd.bn.bias.detach().double().cpu()
n, c, h, w = pre.shape
pre_nhwc = pre.permute(0, 2, 3, 1).reshape(-1, c)
y_nhwc = y.permute(0, 2, 3, 1).reshape(-1, c)
print("y rel err", TC.rel_err(yh.numpy(), y_nhwc.numpy()))
print("pre rel err", TC.rel_err(preh.numpy(), pre_nhwc.numpy()))
flip = (preh > 0) != (pre_nhwc > 0)
print("sign flips", int(flip.sum()), "of", flip.numel())
if flip.any():
    print("flipped pre values (fp64):", pre_nhwc[flip][:10].tolist())
    print("flipped pre values (hip):", preh[flip][:10].tolist())
var = y_nhwc.var(0, unbiased=False)
print("smallest channel std", var.sqrt().min().item(), "mean |y|", y_nhwc.abs().mean().item())
ch = torch.nonzero(flip.any(0)).reshape(-1)[:5]
for cc in ch.tolist():
    print("chan", cc, "std", var[cc].sqrt().item(), "gamma", nd.bn.weight[cc].item(), "beta", nd.bn.bias[cc].item())
