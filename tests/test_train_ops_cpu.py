"""CPU numerics of the training autograd ops: ResNormFn (the residual join folded into the RMSNorm backward)
against plain autograd of h -> (h, rmsnorm(h))."""
import torch

from xotorch_support_jetson_amd.train import autograd_ops as A


def test_res_rmsnorm_matches_autograd_join():
  torch.manual_seed(0)
  h0 = torch.randn(6, 64, dtype=torch.float32)
  w0 = torch.randn(64, dtype=torch.float32)
  up = torch.randn(6, 64)   # gradient arriving on the carried residual stream
  ub = torch.randn(6, 64)   # gradient arriving through the normalised branch

  h, w = h0.clone().requires_grad_(), w0.clone().requires_grad_()
  hc, xn = A.res_rmsnorm(h, w, 1e-5)
  ((hc * up).sum() + (xn * ub).sum()).backward()

  hr, wr = h0.clone().requires_grad_(), w0.clone().requires_grad_()
  xr = hr * torch.rsqrt(hr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
  ((hr * up).sum() + (xr * ub).sum()).backward()
  assert torch.allclose(h.grad, hr.grad, atol=1e-4, rtol=1e-4)
  assert torch.allclose(w.grad, wr.grad, atol=1e-4, rtol=1e-4)
  assert torch.allclose(xn, xr.detach(), atol=1e-5)


def test_res_rmsnorm_branch_only():
  """Only the branch receives a gradient (the carried h unused): the backward is the plain RMSNorm one."""
  torch.manual_seed(1)
  h = torch.randn(3, 32, requires_grad=True)
  w = torch.randn(32, requires_grad=True)
  _, xn = A.res_rmsnorm(h, w, 1e-5)
  xn.sum().backward()
  hr = h.detach().clone().requires_grad_()
  (hr * torch.rsqrt(hr.pow(2).mean(-1, keepdim=True) + 1e-5) * w.detach()).sum().backward()
  assert torch.allclose(h.grad, hr.grad, atol=1e-5)
