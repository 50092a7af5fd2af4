"""lbwn::dilconv_gate (one residual layer, tmodel.py:117-184) forward and backward through the
C ABI (lbwn_layer_forward / lbwn_layer_backward), against a plain PyTorch float64 reference of
the same layer with autograd: z, x_out, dL/d(halo buffer incl. the SAVE rows) and every weight
and bias gradient.  Dilations below, at and above the 128-position tile, ragged T."""
import numpy as np
import pytest
import torch

from lbwn import torch_ops  # noqa: F401

pytestmark = pytest.mark.gpu


def reference(xh, ws, wg, bs, bg, wr, br, d, H):
    T = xh.shape[1] - H
    prev, cur = xh[:, H - d:H - d + T], xh[:, H:]
    vs = prev @ ws[0] + cur @ ws[1] + bs
    vg = prev @ wg[0] + cur @ wg[1] + bg
    z = torch.tanh(vs) * torch.sigmoid(vg)
    return z, cur + z @ wr + br


@pytest.mark.parametrize('d,T,Cr,Cd', [(1, 300, 32, 32), (16, 257, 32, 32), (128, 300, 32, 32), (256, 600, 32, 32),
                                       (4, 200, 24, 16)])
def test_dilconv_gate_fwd_bwd_vs_torch_fp64(d, T, Cr, Cd):
    H, B = 256, 2
    g = torch.Generator().manual_seed(d * 7 + T)
    r = lambda *s, sc=1.0: (torch.randn(*s, generator=g, dtype=torch.float64) * sc)   # noqa: E731
    cpu = [r(B, H + T, Cr), r(2, Cr, Cd, sc=0.2), r(2, Cr, Cd, sc=0.2), r(Cd, sc=0.1), r(Cd, sc=0.1),
           r(Cd, Cr, sc=0.2), r(Cr, sc=0.1)]
    gz, gx = r(B, T, Cd), r(B, T, Cr)
    ref_in = [t.clone().requires_grad_(True) for t in cpu]
    z_r, xo_r = reference(*ref_in, d, H)
    ((z_r * gz).sum() + (xo_r * gx).sum()).backward()
    dev_in = [t.float().cuda().requires_grad_(True) for t in cpu]
    z, xo = torch.ops.lbwn.dilconv_gate(*dev_in, d, H)
    ((z * gz.float().cuda()).sum() + (xo * gx.float().cuda()).sum()).backward()
    torch.cuda.synchronize()
    np.testing.assert_allclose(z.detach().cpu().numpy(), z_r.detach().numpy(), rtol=0, atol=1e-5)
    np.testing.assert_allclose(xo.detach().cpu().numpy(), xo_r.detach().numpy(), rtol=0, atol=2e-5)
    names = ['x_halo', 'w_sig', 'w_gate', 'b_sig', 'b_gate', 'w_res', 'b_res']
    for n, a, b in zip(names, dev_in, ref_in):
        ref = b.grad.numpy()
        got = a.grad.cpu().double().numpy()
        scale = max(1.0, float(np.abs(ref).max()))
        np.testing.assert_allclose(got, ref, rtol=0, atol=2e-5 * scale, err_msg=n)
    # rows before the layer's SAVE never reach the conv
    if H > d:
        assert float(dev_in[0].grad[:, :H - d].abs().max()) == 0.0


def test_module_stack_and_save_state():
    """Two stacked DilatedResidualLayer modules, two consecutive slices: the SAVE buffers carry
    the last d inputs across slices (D-separation, tmodel.py:122-127, :165) and autograd runs
    through both layers."""
    torch.manual_seed(0)
    B, T = 2, 96
    l1 = torch_ops.DilatedResidualLayer(32, 32, 1, B).cuda()
    l2 = torch_ops.DilatedResidualLayer(32, 32, 2, B).cuda()
    x_all = torch.randn(B, 2 * T, 32, device='cuda')
    outs = []
    for s in range(2):
        x = x_all[:, s * T:(s + 1) * T]
        z1, x1 = l1(x)
        z2, x2 = l2(x1)
        outs.append((z1, z2))
    # unstaged: one slice of 2T through fresh layers with the same weights
    m1 = torch_ops.DilatedResidualLayer(32, 32, 1, B).cuda()
    m2 = torch_ops.DilatedResidualLayer(32, 32, 2, B).cuda()
    m1.load_state_dict({k: v for k, v in l1.state_dict().items() if k != 'save'}, strict=False)
    m2.load_state_dict({k: v for k, v in l2.state_dict().items() if k != 'save'}, strict=False)
    z1u, x1u = m1(x_all)
    z2u, _ = m2(x1u)
    for s in range(2):
        np.testing.assert_allclose(outs[s][0].detach().cpu().numpy(), z1u[:, s * T:(s + 1) * T].detach().cpu().numpy(),
                                   rtol=0, atol=1e-6)
        np.testing.assert_allclose(outs[s][1].detach().cpu().numpy(), z2u[:, s * T:(s + 1) * T].detach().cpu().numpy(),
                                   rtol=0, atol=1e-6)
    loss = sum((z1 ** 2).sum() + (z2 ** 2).sum() for z1, z2 in outs)
    loss.backward()
    assert l1.w_sig.grad is not None and torch.isfinite(l1.w_sig.grad).all()
    assert l2.w_res.grad is not None and torch.isfinite(l2.w_res.grad).all()
