"""Oracle: RMILoss (region mutual information, sigmoid form) on the CPU.  TEST INFRASTRUCTURE ONLY.

Restates reference losses.RMILoss as the default config builds it (configs/default_config.py:147:
num_classes=2, rmi_radius=3, rmi_pool='avg', rmi_pool_size=4, rmi_pool_stride=4), in torch-CPU with
the reference's precisions: sigmoid / clamp / avg-pool in fp32, covariances and the 9x9 algebra in fp64.
The gradient is torch autograd through the same graph.

  rmi_loss(logits, target, num_classes, radius, pool, pool_size, pool_stride)
      forward                <- RMILoss.forward -> forward_sigmoid      losses.py:480-483, 505-518
      probs                  <- sigmoid(x).clamp(1e-6, 1.0)             losses.py:515, _CLIP_MIN/_MAX :281-282
      pooling                <- F.avg_pool2d(k, s, padding=k // 2)      losses.py:531-538, kernel_padding :308
                                ('none', or a stride <= 1, skips it)    losses.py:529-533
      map_get_pairs          <- the radius^2 shifted crops              losses.py:313-355
      centred fp64 covariances, inverse(pr_cov + 5e-4 I),
      appro_var, 0.5 * logdet by Cholesky (+1e-8 on the diagonal)       losses.py:553-580, :401-411
      mean over rows of view(-1, num_classes), .float(), / radius^2,
      sum over classes                                                  losses.py:583-592

The reference itself cannot run on a CPU (`.type(torch.cuda.DoubleTensor)`, losses.py:549-550); this
restatement is pinned by tests/golden/rmi_*.npz, which tests/golden/gen_golden.py (G12) produces by running
the reference's own RMILoss with that one device type mapped to the CPU double tensor.
"""
import torch
import torch.nn.functional as F

CLIP_MIN, CLIP_MAX, POS_ALPHA = 1e-6, 1.0, 5e-4


def pool_params(pool, pool_size, pool_stride):
    """(kernel, stride, padding) of the pooling losses.py:529-538 applies; (1, 1, 0) = no pooling."""
    if pool_stride <= 1 or pool == 'none':
        return 1, 1, 0
    if pool != 'avg':
        raise NotImplementedError(f'rmi_pool={pool!r}: only avg and none are restated')
    return pool_size, pool_stride, pool_size // 2


def _pairs(x, radius):
    """losses.py:313-355 (is_combine=False): [N, C, radius^2, (H-r+1)*(W-r+1)], vector index y*radius + x."""
    n, c, h, w = x.shape
    nh, nw = h - (radius - 1), w - (radius - 1)
    crops = [x[:, :, y:y + nh, xx:xx + nw] for y in range(radius) for xx in range(radius)]
    return torch.stack(crops, dim=2).reshape(n, c, radius * radius, -1)


def rmi_loss(logits, target, num_classes=2, radius=3, pool='avg', pool_size=4, pool_stride=4):
    """logits, target: fp32 [N, C, H, W] CPU tensors (logits may require grad).  Returns the fp32 scalar loss."""
    probs = torch.sigmoid(logits).clamp(min=CLIP_MIN, max=CLIP_MAX)
    k, s, p = pool_params(pool, pool_size, pool_stride)
    labels = target
    if (k, s, p) != (1, 1, 0):
        labels = F.avg_pool2d(labels, kernel_size=k, stride=s, padding=p)
        probs = F.avg_pool2d(probs, kernel_size=k, stride=s, padding=p)
    half_d = radius * radius
    la = _pairs(labels, radius).double().detach()
    pr = _pairs(probs, radius).double()
    eye = torch.eye(half_d, dtype=torch.float64)
    la = la - la.mean(dim=3, keepdim=True)
    la_cov = la @ la.transpose(2, 3)
    pr = pr - pr.mean(dim=3, keepdim=True)
    pr_cov = pr @ pr.transpose(2, 3)
    pr_cov_inv = torch.inverse(pr_cov + eye * POS_ALPHA)
    la_pr_cov = la @ pr.transpose(2, 3)
    appro_var = la_cov - (la_pr_cov @ pr_cov_inv) @ la_pr_cov.transpose(-2, -1)
    chol = torch.linalg.cholesky(appro_var + eye * POS_ALPHA)
    rmi_now = 0.5 * (2.0 * torch.sum(torch.log(torch.diagonal(chol, dim1=-2, dim2=-1) + 1e-8), dim=-1))
    per_class = rmi_now.reshape(-1, num_classes).mean(dim=0).float()
    per_class = per_class / float(half_d)
    return per_class.sum()


def rmi_loss_and_grad(logits, target, gout=1.0, **kw):
    """(loss, d(gout * loss)/d logits) as numpy fp32."""
    x = torch.as_tensor(logits, dtype=torch.float32).clone().requires_grad_(True)
    t = torch.as_tensor(target, dtype=torch.float32)
    loss = rmi_loss(x, t, **kw)
    loss.backward(torch.tensor(gout, dtype=torch.float32))
    return loss.detach().numpy(), x.grad.numpy()
