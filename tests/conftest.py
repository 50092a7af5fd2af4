import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'lb-wavenet_amd')):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through the HIP C-ABI)')


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope='session')
def lib():
    """The HIP library, loaded the product way (fails loudly when missing)."""
    from lbwn import _lib
    return _lib.load()


@pytest.fixture(params=['w32', '128', '64', '128:w32', '128+wg'])
def chain_tile(request, monkeypatch):
    """The chains' form (LBWN_CHAIN_TILE = <fwd>[:<bwd>], read at plan creation): 'w32' =
    32-position waves on 128-position tiles (chain_fwd_kernel / chain_bwd_x3_kernel), '128' /
    '64' = 16-position waves on 128- / 64-position tiles (chain_fwd16_kernel / chain_bwd16_kernel
    with 8 / 4 waves) -- the C4 tile axis; '128:w32' mixes the forms.  '+wg': the residual
    stack's weight gradients outside the backward chain (LBWN_BWD_WGRAD=1: the chain exports DV
    and G, layer_wgrad_kernel sums them); every other form keeps them in the chain."""
    tile, _, wg = request.param.partition('+')
    monkeypatch.setenv('LBWN_CHAIN_TILE', tile)
    monkeypatch.setenv('LBWN_BWD_WGRAD', '1' if wg else '0')
    return request.param
